"""Run under mpiexec: MPI_Alltoallv through libtempi.so with a random sparse
byte-count matrix (the shape of SquareMat::make_random_sparse,
/root/reference/support/squaremat.cpp:52-75), verifying every received byte.
Args: [--device] [--scale S] [--nnz K] [--mixed alt|hostrank]
--mixed (with --device) puts some blocks in host memory: alt = even ranks
send from the GPU and receive into the host, odd ranks the reverse;
hostrank = rank 0's buffers are all on the host. The ranks then disagree on
where their memory is, and must still meet (one route on every
rank, descriptor-aware host receives)."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
import tempi_amd  # noqa: E402

args = sys.argv[1:]
device = "--device" in args
scale = int(args[args.index("--scale") + 1]) if "--scale" in args else 1000
nnz = int(args[args.index("--nnz") + 1]) if "--nnz" in args else 2
mixed = args[args.index("--mixed") + 1] if "--mixed" in args else None
mpi = tempi_amd.get_mpi()
if device:
    import torch

    torch.cuda.set_device(0)
mpi.Init()
rank, n = mpi.Comm_rank(), mpi.Comm_size()
rng = np.random.default_rng(101)
mat = np.zeros((n, n), dtype=np.int64)
for r in range(n):
    cols = rng.permutation(n)[:min(nnz, n)]
    mat[r, cols] = rng.integers(1, 10, len(cols)) * scale

scounts = [int(x) for x in mat[rank]]
rcounts = [int(mat[s, rank]) for s in range(n)]
sdispl = np.concatenate([[0], np.cumsum(scounts)[:-1]]).astype(int).tolist()
# leave gaps in the receive buffer: they must stay untouched
rdispl = []
off = 0
for c in rcounts:
    rdispl.append(off)
    off += c + 7
rlen = off + 1
slen = int(sum(scounts)) + 1


def payload(src, dst, nbytes):
    return ((np.arange(nbytes, dtype=np.int64) * 31 + src * 7 + dst * 13) & 0xFF).astype(np.uint8)


send = np.zeros(slen, dtype=np.uint8)
for d in range(n):
    send[sdispl[d]:sdispl[d] + scounts[d]] = payload(rank, d, scounts[d])
recv = np.full(rlen, 0xEE, dtype=np.uint8)
expected = recv.copy()
for s in range(n):
    expected[rdispl[s]:rdispl[s] + rcounts[s]] = payload(s, rank, rcounts[s])

send_dev = recv_dev = device
if mixed == "alt":
    send_dev, recv_dev = rank % 2 == 0, rank % 2 == 1
elif mixed == "hostrank":
    send_dev = recv_dev = rank != 0
if send_dev:
    dsend = torch.from_numpy(send).cuda()
if recv_dev:
    drecv = torch.from_numpy(recv).cuda()
if device:
    torch.cuda.synchronize()
sp = dsend.data_ptr() if send_dev else send.ctypes.data
rp = drecv.data_ptr() if recv_dev else recv.ctypes.data
for it in range(3):
    mpi.Alltoallv(sp, scounts, sdispl, mpi.BYTE, rp, rcounts, rdispl, mpi.BYTE)
got = drecv.cpu().numpy() if recv_dev else recv
errors = int((got != expected).sum())
total = mpi.Allreduce_double(float(errors), op=mpi.SUM)
if rank == 0:
    print(f"RESULT errors={int(total)} ranks={n} scale={scale} nnz={nnz} counters={mpi.counters()}", flush=True)
mpi.Finalize()
sys.exit(1 if total else 0)
