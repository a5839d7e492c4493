"""Run under `mpiexec -n 2`: strided point-to-point through libtempi.so.

--device: buffers on the GPU (each rank uses cuda:0 or its own GPU); otherwise
host numpy buffers (TEMPI forwards to the library). Checks every received
byte against what the sender packed (oracle/typemap.c), for MPI_Send/Recv,
MPI_Isend/Irecv + MPI_Wait / MPI_Waitall / MPI_Test, several datatypes, and a
mix of TEMPI and library requests in one MPI_Waitall. The reference's own
point-to-point tests only check that such calls complete
(/root/reference/test/send.cpp, send_vector.cpp:13-60, isend.cu,
isend_contiguous.cu, sender.cpp); here every byte is compared.
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402
from oracle import pyoracle  # noqa: E402
from tests import typezoo  # noqa: E402

device = "--device" in sys.argv
mpi = tempi_amd.get_mpi()
if device:
    import torch

    torch.cuda.set_device(0)
mpi.Init()
rank, size = mpi.Comm_rank(), mpi.Comm_size()
assert size == 2, size
peer = 1 - rank

RECIPES = [
    ("vector(1024,512,1024,byte)", 1),
    ("subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", 2),
    ("hvector(5,1,53,hvector(3,1,16,contig(13,byte)))", 3),
    ("subarray(C,[100],[10],[5],byte)", 3),
    ("vector(300,3,7,byte)", 2),
    ("hindexed([3,1,4],[0,9,20],byte)", 2),  # not strided: library path (staged)
    ("subarray(C,[256,600],[200,520],[3,4],byte)", 1),  # > 64 KiB: IPC under AUTO
]


def make_buf(n, seed):
    h = np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)
    if device:
        return h, torch.from_numpy(h).cuda()
    return h, h.copy()


def ptr(b):
    return b.data_ptr() if device else b.ctypes.data


def host(b):
    if device:
        torch.cuda.synchronize()
        return b.cpu().numpy()
    return b


errors = 0
for i, (recipe, count) in enumerate(RECIPES):
    tm = pyoracle.TypeMap(recipe)
    origin, buflen = tm.geometry(count)
    t, temps, basic = typezoo.build(mpi, recipe)
    sh, sbuf = make_buf(buflen, 100 + i + 1000 * rank)
    peer_src = np.random.default_rng(100 + i + 1000 * peer).integers(0, 256, buflen, dtype=np.uint8)
    rh, rbuf = make_buf(buflen, 7 + i)
    canvas = rh.copy()
    expected = canvas.copy()
    tm.unpack(tm.pack(peer_src, origin, count), expected, origin, count)
    if device:
        torch.cuda.synchronize()
    # blocking, ordered so it cannot deadlock
    if rank == 0:
        mpi.Send(ptr(sbuf) + origin, count, t, peer, i)
        mpi.Recv(ptr(rbuf) + origin, count, t, peer, i)
    else:
        mpi.Recv(ptr(rbuf) + origin, count, t, peer, i)
        mpi.Send(ptr(sbuf) + origin, count, t, peer, i)
    if not np.array_equal(host(rbuf), expected):
        errors += 1
        print(f"[{rank}] Send/Recv mismatch for {recipe}", flush=True)
    # non-blocking both ways + a library request in the same Waitall
    rh2, rbuf2 = make_buf(buflen, 7 + i)
    hs = np.full(4, rank, dtype=np.int32)
    hr = np.zeros(4, dtype=np.int32)
    if device:
        torch.cuda.synchronize()
    reqs = [mpi.Irecv(ptr(rbuf2) + origin, count, t, peer, 100 + i),
            mpi.Irecv(hr.ctypes.data, 4, mpi.INT, peer, 200 + i),
            mpi.Isend(ptr(sbuf) + origin, count, t, peer, 100 + i),
            mpi.Isend(hs.ctypes.data, 4, mpi.INT, peer, 200 + i)]
    if i % 2:
        reqs = mpi.Waitall(reqs)
    else:
        for k in (2, 0):  # Test until done, then Wait the rest
            done = False
            while not done:
                done, reqs[k] = mpi.Test(reqs[k])
        reqs[1] = mpi.Wait(reqs[1])
        reqs[3] = mpi.Wait(reqs[3])
    assert all(r == mpi.REQUEST_NULL for r in reqs), reqs
    if not np.array_equal(host(rbuf2), expected):
        errors += 1
        print(f"[{rank}] Isend/Irecv mismatch for {recipe}", flush=True)
    if not (hr == peer).all():
        errors += 1
        print(f"[{rank}] library request payload wrong", flush=True)
    typezoo.free(mpi, t, temps, basic)

c = mpi.counters()
total = mpi.Allreduce_double(float(errors), op=mpi.SUM)
if rank == 0:
    print(f"RESULT errors={int(total)} counters={c}", flush=True)
mpi.Finalize()
sys.exit(1 if total else 0)
