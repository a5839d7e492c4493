"""Run under mpiexec -n 1 or 2: the reference's isend tests
(/root/reference/test/isend.cu:19-42: 100 MPI_FLOAT; isend_contiguous.cu:
16-48: make_contiguous_contiguous(800), an MPI_Type_contiguous of 800
bytes) -- each rank MPI_Isend's to itself, then posts the MPI_Irecv, then
waits on the send before the receive, on host buffers and (--device) on
device buffers, twice. The reference only checks that the waits return;
here every received byte is compared with what was sent. (Its third,
TEMPI-disabled device case needs a GPU-aware library; the image's MPICH is
not one.)"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402

device = "--device" in sys.argv
mpi = tempi_amd.get_mpi()
if device:
    import torch

    torch.cuda.set_device(0)
mpi.Init()
rank = mpi.Comm_rank()
errors = 0


def fail(msg):
    global errors
    errors += 1
    print(f"[{rank}] {msg}", flush=True)


contig = mpi.Type_contiguous(800, mpi.BYTE)
mpi.Type_commit(contig)
CASES = [("100 MPI_FLOAT", 100, mpi.FLOAT, 400), ("contiguous(800, MPI_BYTE)", 1, contig, 800)]
for label, count, dt, nbytes in CASES:
    for where in ["host"] + (["device", "device again"] if device else []):
        rng = np.random.default_rng(100 * rank + len(where) + nbytes)
        h = rng.integers(0, 256, nbytes, dtype=np.uint8)
        if where == "host":
            sbuf, rbuf = h.copy(), np.zeros(nbytes, dtype=np.uint8)
            sp, rp = sbuf.ctypes.data, rbuf.ctypes.data
        else:
            sbuf = torch.from_numpy(h).cuda()
            rbuf = torch.zeros(nbytes, dtype=torch.uint8, device="cuda")
            torch.cuda.synchronize()
            sp, rp = sbuf.data_ptr(), rbuf.data_ptr()
        s = mpi.Isend(sp, count, dt, rank, 0)
        r = mpi.Irecv(rp, count, dt, rank, 0)
        mpi.Wait(s)
        mpi.Wait(r)
        got = rbuf if where == "host" else rbuf.cpu().numpy()
        if not np.array_equal(got, h):
            fail(f"{label}, {where}: wrong bytes")
mpi.Type_free(contig)
total = mpi.Allreduce_double(float(errors), op=mpi.SUM)
if rank == 0:
    print(f"RESULT errors={int(total)}", flush=True)
mpi.Finalize()
sys.exit(1 if total else 0)
