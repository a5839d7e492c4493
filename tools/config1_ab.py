"""BASELINE config 1 (bench.config1: MPI_Pack of vector(1024, 512, 1024) on
device buffers, trimean of 300 calls, beside MPICH's host MPI_Pack) with the
resident packer on and off in turn, ROUNDS rotations, one JSON line each.
usage: python tools/config1_ab.py [ROUNDS] [on]   (on: the packer on only;
$VARIANT labels the lines)"""
import ctypes
import json
import os
import sys

import torch  # noqa: F401  (first: one HIP runtime, as bench.py)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import tempi_amd  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
settings = (1,) if len(sys.argv) > 2 and sys.argv[2] == "on" else (1, 0)
variant = os.environ.get("VARIANT", "")
mpi = tempi_amd.get_mpi()
mpi.Init()
H = ctypes.CDLL(tempi_amd.LIBTEMPI_HIP)
dev = torch.device("cuda", 0)
for r in range(rounds):
    for on in settings:
        H.tempi_hip_resident_enable(on)
        c = bench.config1(mpi, torch, dev)
        c.pop("workload", None)
        c.pop("cpu", None)
        print(json.dumps({"variant": variant, "round": r, "resident": on, **c}), flush=True)
mpi.Finalize()
