#!/usr/bin/env python3
"""The 2-rank halo of bench.py's torchrun line, taken apart: one launch mode
per run, to find which part of the torchrun-launched process makes its halo
slower than the same halo under mpiexec on the same box.

  --mode plain     only torch.distributed (gloo) + the PMI wiring, no HIP
                   from torch: libtempi_apps' tempi_bench_halo, as bench.py calls it
  --mode cuda      + torch.cuda initialised on this rank's device (a small tensor)
  --mode headline  + bench.py's headline first (1 GiB MPI_Pack/MPI_Unpack on
                   5 GiB of torch tensors, then torch.cuda.empty_cache())

Launched by torch.distributed.run (RANK / WORLD_SIZE set: gloo + PMI wiring)
or by mpiexec (PMI from hydra, no torch.distributed). Prints one JSON line
per rank 0: mode, launcher, halo us/iter, rank-0 phases, TEMPI counters."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=("plain", "cuda", "headline"), default="plain")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--grid", type=int, default=512)
    a = ap.parse_args()
    torchrun = "RANK" in os.environ and "WORLD_SIZE" in os.environ
    keep = None
    if torchrun:
        import torch.distributed as dist

        from tempi_amd import pmi

        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        dist.init_process_group("gloo", rank=rank, world_size=world)
        keep = pmi.wire_torch_ranks(rank, world, dist)
    torch = None
    if a.mode in ("cuda", "headline"):
        import torch

        torch.cuda.set_device(0)
        torch.zeros(16, device="cuda").sum().item()
    import tempi_amd

    mpi = tempi_amd.get_mpi()
    mpi.Init()
    rank = mpi.Comm_rank()
    if a.mode == "headline":
        rows, pitch, block = 2 << 20, 1024, 512
        t = mpi.Type_commit(mpi.Type_create_subarray([rows, pitch], [rows, block], [0, 0], mpi.ORDER_C, mpi.BYTE))
        src = (torch.arange(rows * pitch, dtype=torch.int64, device="cuda") & 0xFF).to(torch.uint8)
        pk = torch.empty(rows * block, dtype=torch.uint8, device="cuda")
        dst = torch.zeros(rows * pitch, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        for _ in range(8):
            mpi.Pack(src.data_ptr(), 1, t, pk.data_ptr(), rows * block, 0)
            mpi.Unpack(pk.data_ptr(), rows * block, 0, dst.data_ptr(), 1, t)
        torch.cuda.synchronize()
        mpi.Type_free(t)
        del src, pk, dst
        torch.cuda.empty_cache()
    L = ctypes.CDLL(os.path.join(tempi_amd.LIBDIR, "libtempi_apps.so"), mode=ctypes.RTLD_GLOBAL)
    L.tempi_bench_halo.argtypes = [ctypes.c_int] * 9 + [ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(4096)
    mpi.reset_counters()
    t0 = time.perf_counter()
    rc = L.tempi_bench_halo(a.iters, a.grid, a.grid, a.grid, 8, 3, 0, 0, 0 if torch else 1, buf, 4096)
    el = time.perf_counter() - t0
    c = mpi.counters()
    # the library's own intra-node channel: a host-buffer ping-pong (shared
    # memory runs 4 MiB at several GB/s, a socket channel far less)
    L.tempi_bench_pingpong_1d.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                          ctypes.c_int]
    hostpp = {}
    if mpi.Comm_size() >= 2:
        os.environ["TEMPI_BENCH_HOST"] = "1"
        for total in (8, 4 << 20):
            pb = ctypes.create_string_buffer(1024)
            L.tempi_bench_pingpong_1d(20, total, 0, 0, pb, 1024)
            if rank == 0 and pb.value:
                hostpp[str(total)] = json.loads(pb.value.decode()).get("oneway_us")
        del os.environ["TEMPI_BENCH_HOST"]
    if rank == 0:
        r = json.loads(buf.value.decode()) if buf.value else {}
        print(json.dumps({"mode": a.mode, "launcher": "torchrun" if torchrun else "mpiexec", "rc": rc,
                          "us_per_iter": r.get("us_per_iter"), "us_min": r.get("us_min"),
                          "rank0_phase_us": r.get("rank0_us_per_iter"), "wall_s": round(el, 2),
                          "host_pingpong_oneway_us": hostpp,
                          "counters": {k: v for k, v in c.items() if v}}), flush=True)
    mpi.Finalize()
    if torchrun:
        import torch.distributed as dist

        dist.destroy_process_group()
    del keep


if __name__ == "__main__":
    main()
