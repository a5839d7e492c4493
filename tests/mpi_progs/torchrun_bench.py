"""Under torch.distributed.run (gloo, CPU): bench.py's own multi-rank
plumbing -- dist_setup (gloo group + one MPI job wired over the torch
ranks), barrier, the max / sum reductions of the timing -- and an MPI
exchange through libtempi.so between the wired ranks, and the line's
config-5 sections (alltoallv, nbr_alltoallv) and the contiguous ping-pong
on host buffers."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import tempi_amd  # noqa: E402

rank, world, local, pg, keep = bench.dist_setup(None)
assert pg is not None and world == int(os.environ["WORLD_SIZE"])
bench.barrier(pg)
assert bench.allreduce_max(pg, float(rank)) == float(world - 1)
assert bench.allreduce_sum(pg, 1.5) == 1.5 * world
mpi = tempi_amd.get_mpi()
mpi.Init()
assert mpi.Comm_rank() == rank and mpi.Comm_size() == world
src = np.full(4096, rank, dtype=np.uint8)
dst = np.zeros(4096, dtype=np.uint8)
got = mpi.Sendrecv(src.ctypes.data, 4096, mpi.BYTE, (rank + 1) % world, 9, dst.ctypes.data, 4096, mpi.BYTE,
                   (rank - 1) % world, 9)
assert got == ((rank - 1) % world, 9, 4096), got
assert (dst == (rank - 1) % world).all()
# the N > 1 line's config-5 sections, on host buffers (no GPU here)
os.environ["TEMPI_BENCH_HOST"] = "1"


class Args:
    a2av_iters = 2
    pp_iters = 2


for fn in (bench.alltoallv, bench.nbr_alltoallv):
    sec = fn(Args, world)
    if rank == 0:
        assert len(sec["points"]) == 3 and all(p["errors"] == 0 and p["buffers"] == "host" for p in sec["points"]), sec
        assert all(p["min_us"] > 0 and p["xgmi_frac"] is not None for p in sec["points"]), sec
sec = bench.pingpong_1d(Args, world)
if rank == 0:
    assert [p["total"] for p in sec["points"]] == [1 << 21, 1 << 24] and all(p["oneway_us"] > 0 for p in sec["points"])
mpi.Finalize()
print(f"RESULT ok rank={rank}", flush=True)
pg.destroy_process_group()
