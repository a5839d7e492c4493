"""Run under mpiexec -n 1 or -n 2: many TEMPI requests in flight at once.

Each rank posts N receives from its predecessor (host buffers: with TEMPI's
host paths on -- a GPU, or TEMPI_TEST_HOST_ONLY -- each one is a TEMPI
request, since a descriptor may land there), then N sends to its successor,
then completes them in a scrambled order with MPI_Wait / MPI_Test, twice
over, so the request table grows past its first size (4 096 slots) and
handles are reused. Every request handle must be distinct while in flight,
and every received byte checked.
usage: manyreq.py [N]"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

import tempi_amd  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6000
mpi = tempi_amd.get_mpi()
mpi.Init()
rank, size = mpi.Comm_rank(), mpi.Comm_size()
peer, src = (rank + 1) % size, (rank - 1) % size
errors = 0
L = 16
for rnd in range(2):
    rbuf = np.zeros((n, L), dtype=np.uint8)
    sbuf = (np.arange(n * L, dtype=np.int64).reshape(n, L) * (rank + 3) + rnd).astype(np.uint8)
    reqs = [mpi.Irecv(rbuf[i].ctypes.data, L, mpi.BYTE, src, i % 30000, None) for i in range(n)]
    reqs += [mpi.Isend(sbuf[i].ctypes.data, L, mpi.BYTE, peer, i % 30000, None) for i in range(n)]
    live = [r for r in reqs if r != mpi.REQUEST_NULL]
    tempi_held = sum(1 for r in live if 0 < r < (1 << 26))  # TEMPI's handle space (MPICH never issues these)
    if os.environ.get("TEMPI_DISABLE") is None and tempi_held < n:
        errors += 1
        print(f"rank {rank} round {rnd}: only {tempi_held} of the receives are TEMPI requests", flush=True)
    if len(set(live)) != len(live):
        errors += 1
        print(f"rank {rank} round {rnd}: {len(live) - len(set(live))} duplicate request handles", flush=True)
    order = np.random.default_rng(rnd + 11 * rank).permutation(len(reqs))
    for k, i in enumerate(order):
        if k % 3 == 0:
            while True:
                done, reqs[i] = mpi.Test(reqs[i])
                if done:
                    break
        else:
            reqs[i] = mpi.Wait(reqs[i])
    exp = (np.arange(n * L, dtype=np.int64).reshape(n, L) * (src + 3) + rnd).astype(np.uint8)
    if not np.array_equal(rbuf, exp):
        errors += 1
        print(f"rank {rank} round {rnd}: received bytes wrong", flush=True)
mpi.Finalize()
print(f"RESULT errors={errors}", flush=True)
sys.exit(1 if errors else 0)
