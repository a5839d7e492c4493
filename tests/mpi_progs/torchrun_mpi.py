"""Under torch.distributed.run: wire MPICH through tempi_amd.pmi, then run
MPI through libtempi.so across the torch-launched ranks."""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
import torch.distributed as dist  # noqa: E402

import tempi_amd  # noqa: E402
from tempi_amd import pmi  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
srv, sock = pmi.wire_torch_ranks(rank, world, dist)
mpi = tempi_amd.get_mpi()
mpi.Init()
assert mpi.Comm_rank() == rank and mpi.Comm_size() == world, (mpi.Comm_rank(), mpi.Comm_size())
tot = mpi.Allreduce_double(float(rank + 1), op=mpi.SUM)
assert tot == world * (world + 1) / 2
# strided ring exchange through the interposer (host buffers: library path)
t = mpi.Type_commit(mpi.Type_vector(100, 3, 7, mpi.BYTE))
src = np.full(700, rank, dtype=np.uint8)
dst = np.zeros(700, dtype=np.uint8)
r1 = mpi.Irecv(dst.ctypes.data, 1, t, (rank - 1) % world, 5)
r2 = mpi.Isend(src.ctypes.data, 1, t, (rank + 1) % world, 5)
mpi.Waitall([r1, r2])
assert (dst.reshape(100, 7)[:, :3] == (rank - 1) % world).all()
mpi.Type_free(t)
mpi.Barrier()
print(f"RESULT ok rank={rank}", flush=True)
mpi.Finalize()
dist.destroy_process_group()
