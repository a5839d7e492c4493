"""Run under mpiexec -n 2: TEMPI device requests (and library host requests
mixed in) completed through MPI_Testall / MPI_Testany / MPI_Waitany /
MPI_Testsome / MPI_Waitsome / MPI_Request_free, which the reference does not
interpose. Every received byte is checked against the oracle.
--device puts the strided buffers on the GPU."""
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
assert size == 2
peer = 1 - rank
recipe, count = "subarray(C,[40,38,512],[30,3,24],[5,3,24],byte)", 2
tm = pyoracle.TypeMap(recipe)
origin, buflen = tm.geometry(count)
t, temps, basic = typezoo.build(mpi, recipe)
errors = 0


def buf(seed):
    h = np.random.default_rng(seed).integers(0, 256, buflen, dtype=np.uint8)
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


def expected(canvas, src_seed):
    src = np.random.default_rng(src_seed).integers(0, 256, buflen, dtype=np.uint8)
    exp = canvas.copy()
    tm.unpack(tm.pack(src, origin, count), exp, origin, count)
    return exp


for mode in ("testall", "testany", "waitany", "testsome", "waitsome", "request_free"):
    K = 4
    sends, recvs = [], []
    for k in range(K):
        sends.append(buf(1000 * rank + k))
        recvs.append(buf(7 + 31 * k))
    hs = np.full(8, rank, dtype=np.int32)
    hr = np.zeros(8, dtype=np.int32)
    if device:
        torch.cuda.synchronize()
    reqs = [mpi.Irecv(ptr(recvs[k][1]) + origin, count, t, peer, 10 + k) for k in range(K)]
    reqs.append(mpi.Irecv(hr.ctypes.data, 8, mpi.INT, peer, 99))
    sreqs = [mpi.Isend(ptr(sends[k][1]) + origin, count, t, peer, 10 + k) for k in range(K)]
    sreqs.append(mpi.Isend(hs.ctypes.data, 8, mpi.INT, peer, 99))
    if mode == "testall":
        done = False
        while not done:
            done, reqs = mpi.Testall(reqs)
        reqs = mpi.Waitall(reqs)
        sreqs = mpi.Waitall(sreqs)
    elif mode in ("testany", "waitany"):
        left = len(reqs)
        while left:
            if mode == "testany":
                idx, flag, reqs = mpi.Testany(reqs)
                if not flag:
                    continue
            else:
                idx, reqs = mpi.Waitany(reqs)
            assert idx != mpi.UNDEFINED and reqs[idx] == mpi.REQUEST_NULL
            left -= 1
        idx, flag, reqs = mpi.Testany(reqs)
        assert flag and idx == mpi.UNDEFINED  # nothing active any more
        sreqs = mpi.Waitall(sreqs)
    elif mode in ("testsome", "waitsome"):
        seen = set()
        while len(seen) < len(reqs):
            got, reqs = (mpi.Testsome if mode == "testsome" else mpi.Waitsome)(reqs)
            assert got is not None
            seen.update(got)
        got, reqs = mpi.Testsome(reqs)
        assert got is None  # MPI_UNDEFINED: no active request
        sreqs = mpi.Waitall(sreqs)
    else:  # request_free on the sends, then a barrier-synchronised check
        for s in sreqs:
            assert mpi.Request_free(s) == mpi.REQUEST_NULL
        reqs = mpi.Waitall(reqs)
        mpi.Barrier()
    assert all(r == mpi.REQUEST_NULL for r in reqs)
    for k in range(K):
        canvas = np.random.default_rng(7 + 31 * k).integers(0, 256, buflen, dtype=np.uint8)
        if not np.array_equal(host(recvs[k][1]), expected(canvas, 1000 * peer + k)):
            errors += 1
            print(f"[{rank}] {mode}: message {k} wrong", flush=True)
    if not (hr == peer).all():
        errors += 1
        print(f"[{rank}] {mode}: library message wrong", flush=True)

typezoo.free(mpi, t, temps, basic)
total = mpi.Allreduce_double(float(errors), op=mpi.SUM)
if rank == 0:
    print(f"RESULT errors={int(total)}", flush=True)
mpi.Finalize()
sys.exit(1 if total else 0)
