"""MPI_THREAD_MULTIPLE: four threads at once making synchronous MPI_Pack /
MPI_Unpack calls on device objects of their own (config 1's vector, 8-, 4-
and 1-byte-word rows), so requests of several threads meet at the resident
packer (its mutex, one server per device) and at TEMPI's lock. Every round:
fresh random contents, the packed bytes against a torch gather, the
unpacked object (gaps included) against the expected one.
usage: resident_threads.py ROUNDS -> "RESULT errors=0 served=N" """
import ctypes
import os
import sys
import threading

import torch  # noqa: F401  (first: one HIP runtime in the process)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
import tempi_amd  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 100
mpi = tempi_amd.get_mpi()
provided = mpi.Init_thread(mpi.const("MPI_THREAD_MULTIPLE"))
assert provided == mpi.const("MPI_THREAD_MULTIPLE"), provided
H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
dev = torch.device("cuda", 0)
shapes = [(1024, 512, 1024), (4096, 24, 4608), (300, 500, 1000), (20000, 3, 7)]
types = [mpi.Type_commit(mpi.Type_vector(r, b, s, mpi.BYTE)) for r, b, s in shapes]
errors = [0] * len(shapes)
lock = threading.Lock()


def stats():
    a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    H.tempi_hip_resident_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return a.value


def worker(k):
    torch.cuda.set_device(0)
    rows, block, stride = shapes[k]
    ext = (rows - 1) * stride + block
    idx = (torch.arange(rows, device=dev).unsqueeze(1) * stride + torch.arange(block, device=dev)).reshape(-1)
    g = torch.Generator(device=dev).manual_seed(100 + k)
    for r in range(rounds):
        src = torch.randint(0, 256, (ext,), dtype=torch.uint8, device=dev, generator=g)
        packed = torch.zeros(rows * block, dtype=torch.uint8, device=dev)
        back = torch.full((ext,), 0x5A, dtype=torch.uint8, device=dev)
        exp = src[idx]
        ref = back.clone()
        ref[idx] = exp
        torch.cuda.synchronize()
        mpi.Pack(src.data_ptr(), 1, types[k], packed.data_ptr(), packed.numel(), 0)
        mpi.Unpack(packed.data_ptr(), packed.numel(), 0, back.data_ptr(), 1, types[k])
        if not torch.equal(packed, exp) or not torch.equal(back, ref):
            with lock:
                errors[k] += 1
                print(f"thread {k} round {r}: wrong bytes", flush=True)


s0 = stats()
ts = [threading.Thread(target=worker, args=(k,)) for k in range(len(shapes))]
for t in ts:
    t.start()
for t in ts:
    t.join(300)
hung = any(t.is_alive() for t in ts)
served = stats() - s0
for t in types:
    mpi.Type_free(t)
mpi.Finalize()
if hung:
    print("RESULT a thread never finished", flush=True)
    os._exit(3)
print(f"RESULT errors={sum(errors)} served={served}", flush=True)
