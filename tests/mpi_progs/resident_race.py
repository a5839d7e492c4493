"""The resident packer's exit race (pack_kernels.hip, "resident packer"), in a
process of its own so that TEMPI_RESIDENT_IDLE_US can be tiny: the server
leaves after IDLE microseconds without a request, and the calls here come
after random gaps of 0 .. 3 x IDLE, so requests keep landing before, during
and after the leader's exit -- served, posted again to a new instance, or
taken by a freshly launched one. Every round rewrites the source (torch, on
torch's stream, synchronised), packs it with MPI_Pack (config 1's vector, or
a 4-byte-word / 3D / misaligned shape in turn), checks the bytes against a
torch gather, then unpacks into a cleared buffer and checks that too.
usage: resident_race.py IDLE_US ROUNDS -> "RESULT errors=0 served=.. launches=.. reposts=.." """
import ctypes
import os
import random
import sys
import time

import torch  # noqa: F401  (first: one HIP runtime in the process)

idle_us = int(sys.argv[1]) if len(sys.argv) > 1 else 20
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 400
os.environ["TEMPI_RESIDENT_IDLE_US"] = str(idle_us)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
import tempi_amd  # noqa: E402

mpi = tempi_amd.get_mpi()
mpi.Init()
H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)


def stats():
    a, b, c = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    H.tempi_hip_resident_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
    return a.value, b.value, c.value


dev = torch.device("cuda", 0)
# (rows, block, stride, packed offset): 16-, 4- and 8-byte words, a packed side
# 4 bytes into its buffer (partial first / last chunks)
shapes = [(1024, 512, 1024, 0), (100, 500, 1000, 0), (4096, 24, 4608, 0), (257, 48, 80, 4)]
types = [mpi.Type_commit(mpi.Type_vector(r, b, s, mpi.BYTE)) for r, b, s, _ in shapes]
rng = random.Random(idle_us)
errors = 0
s0 = stats()
for i in range(rounds):
    k = i % len(shapes)
    rows, block, stride, off = shapes[k]
    ext = (rows - 1) * stride + block
    src = torch.randint(0, 256, (ext,), dtype=torch.uint8, device=dev)
    packed = torch.zeros(rows * block + off, dtype=torch.uint8, device=dev)
    idx = (torch.arange(rows, device=dev).unsqueeze(1) * stride + torch.arange(block, device=dev)).reshape(-1)
    exp = src[idx]
    torch.cuda.synchronize()
    t_end = time.perf_counter() + rng.uniform(0, 3 * idle_us) * 1e-6
    while time.perf_counter() < t_end:
        pass
    mpi.Pack(src.data_ptr(), 1, types[k], packed.data_ptr() + off, rows * block, 0)
    if not torch.equal(packed[off:], exp) or (off and int(packed[:off].count_nonzero())):
        errors += 1
        print(f"round {i}: packed bytes wrong (shape {shapes[k]})", flush=True)
    back = torch.zeros(ext, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    mpi.Unpack(packed.data_ptr() + off, rows * block, 0, back.data_ptr(), 1, types[k])
    ref = torch.zeros(ext, dtype=torch.uint8, device=dev)
    ref[idx] = exp
    if not torch.equal(back, ref):
        errors += 1
        print(f"round {i}: unpacked bytes wrong (shape {shapes[k]})", flush=True)
s1 = stats()
for t in types:
    mpi.Type_free(t)
mpi.Finalize()
H.tempi_hip_resident_lost.restype = ctypes.c_uint64
lost = H.tempi_hip_resident_lost()
print(f"RESULT errors={errors} served={s1[0] - s0[0]} launches={s1[1] - s0[1]} reposts={s1[2] - s0[2]} lost={lost}",
      flush=True)
