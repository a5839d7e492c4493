#!/usr/bin/env python3
"""TEMPI-MI355X headline benchmark (driver contract: one JSON line on rank 0).

Metric (BASELINE.json): MPI_Pack/Unpack GB/s vs HBM peak. One STEP = one
MPI_Pack + one MPI_Unpack, through libtempi.so, of one object of config 2
(2D/3D subarray sweep, 1 MiB - 1 GiB objects on one MI355X). The default
object is the bench-mpi-pack type of config 1 (MPI_Type_vector(1024, 512,
1024, MPI_BYTE), /root/reference/bin/bench_mpi_pack.cpp) scaled to a 1 GiB
packed size: MPI_Type_create_subarray({2^21, 1024}, {2^21, 512}, {0, 0}),
extent 2 GiB (>> the 256 MiB Infinity Cache, so HBM is what is measured).

value = algorithmic bytes moved by all ranks / max-over-ranks wall time, where
one pack or unpack of P payload bytes moves 2P (read P + write P; SURVEY
8(d)). N > 1 (torchrun): every rank packs its own object on its own GPU, no
collective on the data path (weak scaling, replicas).

The same line carries "halo": the 3D halo exchange of config 4 (512^3 grid,
8 quantities of 8 B, radius 3, 26 neighbours, periodic, 3 substeps per
iteration) run through MPI_Isend/MPI_Irecv/MPI_Wait on the same ranks
(strong scaling of the fixed grid), with its xGMI roofline. Under torchrun
the ranks are wired into one MPI job by tempi_amd.pmi.

At N > 1 the line also carries "pingpong" (config 3, ranks 0 <-> 1),
"pingpong_1d" (the contiguous ping-pong, all pairs),
"alltoallv" (config 5, all ranks) and "nbr_alltoallv" (config 5's
neighbourhood form), each with its xGMI fraction.

Other modes (not the driver's line):
  --sweep FILE   the config-2 sweep (block 1 B - 4 KiB, 2D and 3D, 1 MiB -
                 1 GiB), one JSON record per point, written to FILE
"""
import argparse
import json
import math
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
METRIC = "MPI_Pack/Unpack GB/s vs HBM peak; 3D halo-exchange µs/iter at 1–8 GPUs"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--rows", type=int, default=2 * 1024 * 1024)
    p.add_argument("--pitch", type=int, default=1024)
    p.add_argument("--block", type=int, default=512)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=8.0)
    p.add_argument("--no-traffic", action="store_true",
                   help="skip the rocprofv3 FETCH_SIZE / WRITE_SIZE passes (child processes) for roofline.traffic")
    p.add_argument("--no-halo", action="store_true")
    p.add_argument("--halo-grid", type=int, default=512)
    p.add_argument("--halo-iters", type=int, default=30)  # (trimean of >= 30 iterations)
    p.add_argument("--pp-iters", type=int, default=50)
    p.add_argument("--a2av-iters", type=int, default=20)
    p.add_argument("--no-p2p", action="store_true", help="skip configs 3 and 5 at N > 1")
    p.add_argument("--sweep", default=None, help="run the config-2 sweep and write JSON records here")
    p.add_argument("--sweep-sizes", default=None,
                   help="comma-separated packed sizes for --sweep (default 1 MiB, 16 MiB, 256 MiB, 1 GiB)")
    p.add_argument("--sweep-traffic", default="2:2:18,3:1:2,2:24:40,2:8:512", metavar="SHAPES",
                   help="comma-separated DIMS:BLOCK:STRIDE sweep shapes whose FETCH / WRITE traffic is counted "
                        "against the touched model (tools/sweep_pmc.py; sweep_geomean.traffic_checked in the "
                        "detail); 'none' skips it")
    p.add_argument("--no-sweep-geomean", action="store_true",
                   help="skip the 1 GiB points of the config-2 sweep in the default line (sweep_geomean)")
    p.add_argument("--no-measure-system", action="store_true",
                   help="N > 1: do not measure this node's perf.json when it is missing")
    # 400 s: with a fresh box's first `import torch` (1-2 min) and the headline
    # before it, the line is out well inside the driver's 600 s per run
    p.add_argument("--extras-deadline", type=float, default=400.0,
                   help="seconds after the headline within which the line's other sections must finish; past it "
                        "rank 0 prints the line so far, marked incomplete, and every rank exits")
    p.add_argument("--detail-name", default=None,
                   help="file name under gpurun_out/ for the full record (default bench_detail_nN.json)")
    p.add_argument("--inner", action="store_true", help=argparse.SUPPRESS)  # child for --traffic
    return p.parse_args()


class stdout_to_stderr:
    """fd 1 -> fd 2 for a block: torch's gloo backend prints its connection
    messages on stdout, which carries the bench line only"""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def dist_setup(args):
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    pg = None
    keep = None
    if world > 1:
        import torch.distributed as dist

        from tempi_amd import pmi

        with stdout_to_stderr():
            dist.init_process_group("gloo", rank=rank, world_size=world)
            dist.barrier()
            pg = dist
            keep = pmi.wire_torch_ranks(rank, world, dist)  # one MPI job over the torch ranks
    return rank, world, local, pg, keep


def barrier(pg):
    if pg is not None:
        pg.barrier()


def allreduce_max(pg, x):
    if pg is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.MAX)
    return float(t.item())


def allreduce_sum(pg, x):
    if pg is None:
        return x
    import torch

    t = torch.tensor([x], dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return float(t.item())


def allreduce_sum_vec(pg, xs):
    if pg is None:
        return list(xs)
    import torch

    t = torch.tensor(list(xs), dtype=torch.float64)
    pg.all_reduce(t, op=pg.ReduceOp.SUM)
    return [float(v) for v in t.tolist()]


_ROUTES = (("ipc", "send_ipc", "bytes_ipc"), ("ipc_copy", "send_ipc_copy", "bytes_ipc_copy"),
           ("oneshot", "send_oneshot", "bytes_oneshot"), ("staged", "send_staged", "bytes_staged"),
           ("device", "send_device", "bytes_device"), ("direct", "send_direct", "bytes_direct"))


def transport_block(mpi, pg, before, after, shared_gpu, what):
    """what the transport did over `what`, summed over all
    ranks -- per-route message and payload-byte counts (IPC includes IPC COPY,
    which is also counted on its own), device-object messages handed to the
    library, first-contact canaries, the IPC threshold non-blocking AUTO sends
    used and whether it came from a perf.json measured on this node. Fields
    that need ranks on separate GPUs are null with the reason."""
    import ctypes

    d = {k: after[k] - before[k] for k in after}
    keys = [k for _, m, b in _ROUTES for k in (m, b)] + ["lib_sends", "self_matched", "canary_ok", "canary_fail",
                                                         "batches", "ticket_batches"]
    tot = dict(zip(keys, (int(v) for v in allreduce_sum_vec(pg, [d.get(k, 0) for k in keys]))))
    out = {"over": what, "routes": {name: {"messages": tot[m], "bytes": tot[b]} for name, m, b in _ROUTES},
           "library_sends": tot["lib_sends"], "self_matched": tot["self_matched"], "batches": tot["batches"],
           "ticket_batches": tot["ticket_batches"]}
    if shared_gpu:
        out["canary_ok"] = out["canary_fail"] = None
        out["canary_note"] = ("shared GPU: every peer is on this rank's own GPU, so no first-contact canary (a peer "
                              "on ANOTHER GPU read back over xGMI) can run")
    else:
        out["canary_ok"], out["canary_fail"] = tot["canary_ok"], tot["canary_fail"]
    L = mpi.L
    L.tempi_ipc_threshold.restype = ctypes.c_int64
    L.tempi_ipc_threshold.argtypes = [ctypes.c_int64, ctypes.POINTER(ctypes.c_int)]
    th = {}
    fm = ctypes.c_int(0)
    for bl in (24, 512):  # the halo's x-face rows and (capped) y / z-face rows
        t = L.tempi_ipc_threshold(bl, ctypes.byref(fm))
        th[f"block_{bl}"] = None if t == (1 << 63) - 1 else int(t)  # (null: never IPC)
    out["ipc_threshold"] = dict(th, from_node_perf_json=bool(fm.value))
    buf = ctypes.create_string_buffer(4096)
    L.tempi_perf_source.argtypes = [ctypes.c_char_p, ctypes.c_int]
    loaded = L.tempi_perf_source(buf, 4096)
    src = buf.value.decode() if loaded == 1 else ""
    out["perf_json_measured_on_node"] = bool(src) and os.path.abspath(src) == os.path.abspath(
        os.path.join(tempi_cache_dir(), "perf.json"))
    if shared_gpu:
        out["perf_json_note"] = "shared GPU: a node perf.json measured here never crossed xGMI"
    return out


def make_2d(mpi, rows, pitch, block):
    t = mpi.Type_create_subarray([rows, pitch], [rows, block], [0, 0], mpi.ORDER_C, mpi.BYTE)
    return mpi.Type_commit(t)


def cpu_baseline(mpi, rows, pitch, block, seconds):
    """Host MPI (MPICH) MPI_Pack + MPI_Unpack on host buffers, one pinned core:
    the reference's CPU path (/root/reference/src/pack.cpp:51-54), on the
    headline's own object (the same subarray, the same 1 GiB packed size)."""
    import numpy as np

    t = make_2d(mpi, rows, pitch, block)
    src = np.resize(np.arange(256, dtype=np.uint8), rows * pitch)  # byte i = i & 0xFF
    packed = np.zeros(rows * block, dtype=np.uint8)
    dst = np.zeros(rows * pitch, dtype=np.uint8)
    old = os.sched_getaffinity(0)
    core = sorted(old)[0]
    os.sched_setaffinity(0, {core})
    try:
        mpi.Pack(src.ctypes.data, 1, t, packed.ctypes.data, packed.size, 0)  # warm
        n = 0
        t0 = time.perf_counter()
        while True:
            mpi.Pack(src.ctypes.data, 1, t, packed.ctypes.data, packed.size, 0)
            mpi.Unpack(packed.ctypes.data, packed.size, 0, dst.ctypes.data, 1, t)
            n += 1
            el = time.perf_counter() - t0
            if el >= seconds:
                break
    finally:
        os.sched_setaffinity(0, old)
    mpi.Type_free(t)
    alg = 4.0 * rows * block * n  # pack + unpack, each reads and writes the payload
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {
        "value": round(alg / el / 1e9, 3),
        "unit": "GB/s",
        "cores": 1,
        "kind": "reference",
        "sample": (f"MPICH 3.3.2 MPI_Pack+MPI_Unpack of the headline object ({rows * block >> 20} MiB packed) on "
                   f"host buffers, {n} pairs in {el:.1f} s, 1 pinned core of {model}"),
    }


def config1(mpi, torch, dev, iters=300):
    """BASELINE config 1 exactly: the reference's bench-mpi-pack object
    MPI_Type_vector(1024, 512, 1024, MPI_BYTE) (512 KiB packed, extent
    1 MiB), one MPI_Pack per call, trimean over `iters` calls: through the
    host MPI on host buffers (the reference's CPU path, one pinned core) and
    through libtempi on device buffers (synchronous GPU pack)."""
    import numpy as np

    t = mpi.Type_commit(mpi.Type_vector(1024, 512, 1024, mpi.BYTE))
    n = 1023 * 1024 + 512
    out = {}

    def trimean(v):
        v = sorted(v)
        q = lambda p: v[int(round(p * (len(v) - 1)))]  # noqa: E731
        return (q(0.25) + 2 * q(0.5) + q(0.75)) / 4

    try:
        src = (np.arange(n, dtype=np.int64) & 0xFF).astype(np.uint8)
        packed = np.zeros(512 * 1024, dtype=np.uint8)
        old = os.sched_getaffinity(0)
        os.sched_setaffinity(0, {sorted(old)[0]})
        try:
            # (pointers taken once, outside the timed calls, on both sides: numpy's
            # .ctypes.data costs more per access than torch's data_ptr())
            hs, hd, hn = src.ctypes.data, packed.ctypes.data, packed.size
            ts = []
            for _ in range(iters + 5):
                t0 = time.perf_counter()
                mpi.Pack(hs, 1, t, hd, hn, 0)
                ts.append(time.perf_counter() - t0)
        finally:
            os.sched_setaffinity(0, old)
        cpu = trimean(ts[5:])
        dsrc = torch.from_numpy(src).to(dev)
        dpk = torch.zeros(512 * 1024, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        ds, dd, dn = dsrc.data_ptr(), dpk.data_ptr(), dpk.numel()
        ts = []
        for _ in range(iters + 5):
            t0 = time.perf_counter()
            mpi.Pack(ds, 1, t, dd, dn, 0)
            ts.append(time.perf_counter() - t0)
        gpu = trimean(ts[5:])
        ok = bool(np.array_equal(dpk.cpu().numpy(), packed))
        out = {"workload": "BASELINE config 1: MPI_Pack of MPI_Type_vector(1024, 512, 1024, MPI_BYTE), 512 KiB packed, "
                           "API time per call (trimean)",
               "cpu_us": round(cpu * 1e6, 2), "cpu_payload_GBps": round(512 * 1024 / cpu / 1e9, 2),
               "cpu": "host MPICH 3.3.2 on host buffers, one pinned core of " + _cpu_model(),
               "gpu_us": round(gpu * 1e6, 2), "gpu_payload_GBps": round(512 * 1024 / gpu / 1e9, 2),
               "speedup": round(cpu / gpu, 2), "gpu_matches_cpu": ok}
        # the same call in C, on this box, with its phases (apps/bench_lib.cpp
        # tempi_bench_sync_phases): where a synchronous GPU MPI_Pack's time goes;
        # pinned to the core the host MPI_Pack above ran on, both sides
        try:
            import ctypes

            buf = ctypes.create_string_buffer(2048)
            L = apps_lib()
            L.tempi_bench_sync_phases.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
            os.sched_setaffinity(0, {sorted(old)[0]})
            try:
                rc = L.tempi_bench_sync_phases(iters, buf, 2048)
            finally:
                os.sched_setaffinity(0, old)
            if rc == 0 and buf.value:
                out["c_phases"] = json.loads(buf.value.decode())
                out["c_phases"]["pinned_core"] = sorted(old)[0]
        except Exception as e:  # (reported, never fatal to the line)
            out["c_phases"] = {"error": str(e)[:200]}
    finally:
        mpi.Type_free(t)
    return out


def _cpu_model():
    try:
        return [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        return "unknown"


def library_path_baselines(args):
    """CPU baselines of configs 3-5: the same apps on pageable host buffers
    with TEMPI_DISABLE=1, i.e. the host MPI's own strided Isend / Irecv /
    Send / Recv / Alltoallv (the reference's path for host memory), each a
    child MPI job of its own, bounded to a few seconds."""
    import tempi_amd

    env = {k: v for k, v in os.environ.items() if not k.startswith(("PMI_", "MPI_LOCAL", "HYDRA_"))}
    env.update({"TEMPI_DISABLE": "1", "TEMPI_BENCH_HOST": "1", "HYDRA_LAUNCHER": "fork"})
    lib = tempi_amd.LIBDIR

    def run(n, argv, timeout=240):
        r = subprocess.run(["timeout", "-k", "10", str(timeout), "/opt/conda/bin/mpiexec", "-n", str(n)] + argv,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
        for line in r.stdout.splitlines():
            if line.startswith("{"):
                return json.loads(line)
        return None

    model = _cpu_model()
    out = {}
    h = run(1, [os.path.join(lib, "halo_exchange"), "2", str(args.halo_grid)])
    if h:
        out["halo"] = {"value": h["us_per_iter"], "unit": "us/iter", "higher_is_better": False, "cores": 1,
                       "kind": "reference",
                       "sample": (f"halo_exchange {args.halo_grid}^3, 8 quantities, 1 rank, pageable host buffers, "
                                  f"TEMPI_DISABLE=1 (MPICH 3.3.2 packs the subarray types on the CPU), 2 iterations "
                                  f"after 1 warm-up, one core of {model}")}
    pp = []
    for total, bl in ((4 << 20, 512), (4 << 20, 64), (1 << 20, 8)):
        r = run(2, [os.path.join(lib, "pingpong_nd"), "20", str(total), str(bl)])
        if r:
            pp.append({"total": total, "block": bl, "oneway_us": r["oneway_us"], "GBps": r["GBps"]})
    if pp:
        out["pingpong"] = {"points": pp, "unit": "us one-way", "higher_is_better": False, "cores": 2,
                           "kind": "reference",
                           "sample": (f"pingpong_nd vector(total/bl, bl, 512) MPI_Send/MPI_Recv, 2 ranks on one host, "
                                      f"pageable host buffers, TEMPI_DISABLE=1, 20 round trips, 2 cores of {model}")}
    a = run(8, [os.path.join(lib, "alltoallv_sparse"), "20", "--scale", "100000", "--density", "1.0"])
    if a:
        out["alltoallv"] = {"value": a["min_us"], "unit": "us", "higher_is_better": False, "cores": 8,
                            "kind": "reference",
                            "sample": (f"alltoallv_sparse scale 1e5 density 1.0 (the reference's random sparse "
                                       f"matrix, seed 101), 8 ranks, pageable host buffers, TEMPI_DISABLE=1, min of 20, "
                                       f"8 cores of {model}")}
    return out


def type_commit_cost():
    """MPI_Type_commit through libtempi (commit + canonical
    descriptor) against the library's own commit (TEMPI_DISABLE=1), the
    reference's bench_type_commit shapes and constructions (apps/
    type_commit.cpp), each a one-rank child job on this host."""
    import tempi_amd

    env = {k: v for k, v in os.environ.items() if not k.startswith(("PMI_", "MPI_LOCAL", "HYDRA_"))}
    env["HYDRA_LAUNCHER"] = "fork"
    out = {}
    for name, extra in (("tempi", {}), ("library", {"TEMPI_DISABLE": "1"})):
        r = subprocess.run(["timeout", "-k", "10", "120", "/opt/conda/bin/mpiexec", "-n", "1",
                            os.path.join(tempi_amd.LIBDIR, "type_commit"), "300"], stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, env=dict(env, **extra))
        line = next((l for l in r.stdout.splitlines() if l.startswith("{")), None)
        if r.returncode != 0 or line is None:
            raise RuntimeError(f"type_commit ({name}) rc={r.returncode}: {r.stdout[-300:]}")
        d = json.loads(line)
        out[name] = {"commit_us_median": d["commit_us_median"], "commit_us_max": d["commit_us_max"],
                     "per_factory_median_us": {k: sorted(v["commit_us"])[len(v["commit_us"]) // 2]
                                               for k, v in d["factories"].items()}}
    out["workload"] = ("bench_type_commit: 24 copy extents in a 1024^3-byte allocation x 5 constructions "
                       "(subarray, byte_v_hv, byte_v1_hv_hv, byte_vn_hv_hv, subarray_v), create + commit + free "
                       "300 times each, trimean; host only, one core")
    return out


def mpi_pack_bench():
    """The reference's own headline benchmark, bench_mpi_pack
    (/root/reference/bin/bench_mpi_pack.cpp; its README chart is MPI_Pack
    speedup over the library): 2D byte objects of 1 KiB / 1 MiB / 4 MiB per
    element, count 1 and 2, rows of 1-512 B at a 512-B stride, vector /
    hvector / subarray, API-level MiB/s (MPI_Wtime per call, trimean).
    Through libtempi on device buffers (100 calls), and the library's CPU
    path on host buffers (TEMPI_DISABLE=1, 3 calls as the reference's
    no-TEMPI runs use few; subarray only, the library packs all three the
    same way), each a one-rank child job (apps/mpi_pack.cpp)."""
    import tempi_amd

    env = {k: v for k, v in os.environ.items() if not k.startswith(("PMI_", "MPI_LOCAL", "HYDRA_"))}
    env["HYDRA_LAUNCHER"] = "fork"
    exe = os.path.join(tempi_amd.LIBDIR, "mpi_pack")

    def run(argv, extra, timeout):
        r = subprocess.run(["timeout", "-k", "10", str(timeout), "/opt/conda/bin/mpiexec", "-n", "1", exe] + argv,
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=dict(env, **extra))
        recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
        if r.returncode != 0 or not recs:
            raise RuntimeError(f"mpi_pack rc={r.returncode}: {r.stdout[-300:]}")
        return recs

    gpu = run(["100"], {}, 240)
    lib = {(p["target"], p["count"], p["block"]): p
           for p in run(["3", "--host", "--factory", "subarray"], {"TEMPI_DISABLE": "1"}, 240)}
    points, speedups = [], {}
    for p in gpu:
        key = (p["target"], p["count"], p["block"])
        q = {"target": p["target"], "count": p["count"], "block": p["block"], "factory": p["factory"],
             "pack_MiBps": p["pack_MiBps"], "unpack_MiBps": p["unpack_MiBps"], "errors": p["errors"]}
        if key in lib and lib[key]["pack_us"] > 0.01 and p["pack_us"] > 0:  # (below the library's timer tick)
            s = lib[key]["pack_us"] / p["pack_us"]
            q["library_pack_MiBps"] = lib[key]["pack_MiBps"]
            q["pack_speedup"] = float(f"{s:.3g}")
            speedups.setdefault(p["target"], []).append(s)
        points.append(q)

    def gm(xs):
        return math.exp(sum(math.log(x) for x in xs) / len(xs))

    return {"workload": ("bench_mpi_pack: MPI_Pack / MPI_Unpack of 2D byte vector / hvector / subarray objects, "
                         "1 KiB / 1 MiB / 4 MiB per element, count 1-2, rows 1-512 B at stride 512, one rank; "
                         "MiB/s of packed bytes per API call (trimean)"),
            "errors": sum(p["errors"] for p in gpu),
            "pack_speedup_geomean_by_target": {str(t): float(f"{gm(v):.3g}") for t, v in sorted(speedups.items())},
            "library": "MPICH 3.3.2 MPI_Pack on pageable host buffers, TEMPI_DISABLE=1, one core of " + _cpu_model(),
            "points": points}


def run_traffic_passes(args, kernel_substr):
    """rocprofv3 PMC passes (one counter group per run, child processes),
    gfx950 correction: FETCH_SIZE reads half of a wide streaming read
    (MI355X_MICROARCH.md sec. HBM). Returns (read_bytes, write_bytes) per
    launch of kernels whose name contains kernel_substr, or None."""
    import csv
    import glob
    import shutil
    import tempfile

    if not shutil.which("rocprofv3"):
        return None
    # already under a profiler: a nested rocprofv3 would exec from a process
    # whose GPU the outer profiler's preload has initialised
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    out = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="tempi_pmc_", dir=os.path.join(ROOT, "gpurun_out") if os.path.isdir(
            os.path.join(ROOT, "gpurun_out")) else None)
        cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d,
               "-o", "pmc", "--", sys.executable, os.path.abspath(__file__), "--inner", "--steps", "3",
               "--warmup", "1", "--rows", str(args.rows), "--pitch", str(args.pitch), "--block", str(args.block),
               "--no-cpu-baseline", "--no-halo", "--no-traffic"]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            return None
        vals = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    if kernel_substr in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                        vals.append(float(row["Counter_Value"]))
        if not vals:
            return None
        out[counter] = sum(vals) / len(vals) * 1024.0  # counters are in KiB
    return out["FETCH_SIZE"] * 2.0, out["WRITE_SIZE"]


def halo_traffic(args):
    """HBM bytes per 1-rank halo iteration (rocprofv3 --pmc, one counter per
    run, over every pack / unpack / copy kernel of `halo_exchange 3 GRID`,
    which runs 1 warm-up + 3 iterations); None when it cannot be measured"""
    import csv
    import glob
    import shutil
    import tempfile

    import tempi_amd

    exe = os.path.join(tempi_amd.LIBDIR, "halo_exchange")
    if not shutil.which("rocprofv3") or not os.path.exists(exe):
        return None
    if any(k.startswith("ROCPROF") for k in os.environ) or "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None
    iters = 3
    out = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="tempi_pmc_", dir=os.path.join(ROOT, "gpurun_out") if os.path.isdir(
            os.path.join(ROOT, "gpurun_out")) else None)
        cmd = ["timeout", "-s", "KILL", "150", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d,
               "-o", "pmc", "--", exe, str(iters), str(args.halo_grid)]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            return None
        tot = 0.0
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    if row.get("Counter_Name") == counter and ("copy_batch" in name or "pack" in name):
                        tot += float(row["Counter_Value"]) * 1024.0
        out[counter] = tot / (iters + 1)
    return out["FETCH_SIZE"] * 2.0, out["WRITE_SIZE"]


def headline(args, mpi, torch, rank, world, pg, dev):
    rows, pitch, block = args.rows, args.pitch, args.block
    payload = rows * block
    t = make_2d(mpi, rows, pitch, block)
    src = (torch.arange(rows * pitch, dtype=torch.int64, device=dev) & 0xFF).to(torch.uint8)
    packed = torch.empty(payload, dtype=torch.uint8, device=dev)
    dst = torch.zeros(rows * pitch, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()

    def step():
        mpi.Pack(src.data_ptr(), 1, t, packed.data_ptr(), payload, 0)
        mpi.Unpack(packed.data_ptr(), payload, 0, dst.data_ptr(), 1, t)

    for _ in range(args.warmup):
        step()
    # parity of what is being timed (exact, via strided views)
    torch.cuda.synchronize()
    ok = torch.equal(packed.view(rows, block), src.view(rows, pitch)[:, :block]) and torch.equal(
        dst.view(rows, pitch)[:, :block], src.view(rows, pitch)[:, :block])
    if not ok:
        raise SystemExit("bench parity check failed: packed bytes differ from the strided source")

    mpi.reset_counters()
    mpi.set_kernel_profiling(True)
    barrier(pg)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    barrier(pg)
    mpi.set_kernel_profiling(False)
    kt = mpi.kernel_times()
    el_max = allreduce_max(pg, el)
    alg_step = 4.0 * payload  # pack (2P) + unpack (2P)
    total_alg = allreduce_sum(pg, alg_step * args.steps)
    value = total_alg / el_max / 1e9
    mpi.Type_free(t)

    # the box's achievable HBM rate for the same bytes: a device-to-device
    # copy of the packed size (read + write, SURVEY 8(d) "calibrated peak")
    cal = calibrate_copy(torch, packed, dst, payload)
    launches = kt["packs"] + kt["unpacks"]
    avg_ms = (kt["pack_ms"] + kt["unpack_ms"]) / max(launches, 1)
    alg_launch = 2.0 * payload
    achieved = alg_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    rec = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (byte i = i & 0xFF)",
        "config": {
            "workload": (f"config 2 point: MPI_Pack+MPI_Unpack, subarray({{{rows},{pitch}}}->{{{rows},{block}}}) "
                         f"MPI_BYTE, {payload >> 20} MiB packed, device buffers, per rank"),
            "packed_bytes": payload,
            "extent_bytes": rows * pitch,
            "block_bytes": block,
            "stride_bytes": pitch,
            "parallelism": f"replicas{world}",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": None,
            "kernel": "pack_kernel<16,1> / unpack_kernel<16,1> (libtempi_hip.so)",
            "algorithmic_bytes_per_launch": int(alg_launch),
            "avg_launch_ms": round(avg_ms, 4),
            "pack_avg_ms": round(kt["pack_ms"] / max(kt["packs"], 1), 4),
            "unpack_avg_ms": round(kt["unpack_ms"] / max(kt["unpacks"], 1), 4),
            "timed_launches": launches,
            # calibration: the guide's achievable streaming rate, and this
            # box's hipMemcpyAsync D2D of the same bytes (slower than the
            # pack kernel itself, so not a ceiling)
            "achievable_peak": HBM_ACHIEVABLE_GBS,
            "frac_achievable": round(achieved / HBM_ACHIEVABLE_GBS, 4),
            "d2d_copy_GBps": round(cal, 1),
            "calibration": ("achievable_peak: MI355X_MICROARCH.md HBM section (~6.3 TB/s streaming); d2d_copy_GBps: "
                            "torch copy_ (hipMemcpyAsync D2D) of the packed size, 10 launches, HIP events"),
        },
    }
    return rec


HBM_ACHIEVABLE_GBS = 6300.0  # MI355X_MICROARCH.md: "8 TB/s peak (spec); ~6.3 TB/s achievable"


def calibrate_copy(torch, a, scratch, n):
    """GB/s (read + write) of a plain device-to-device copy of n bytes"""
    b = scratch[:n]
    for _ in range(2):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 10
    return 2.0 * n / (ms * 1e-3) / 1e9 if ms > 0 else 0.0


XGMI_LINK_GBS = 153.0  # per direction, per link


def halo(args, mpi, world, grid=None):
    """Config 4 through libtempi_apps.so's tempi_bench_halo (every rank).
    grid: the global edge (default --halo-grid, fixed total work); the
    reference's own scripts weak-scale it instead (512, 645, 813, 1024 for 1,
    2, 4, 8 ranks: scripts/summit/bench_halo_exchange.sh:27-45)."""
    import ctypes

    import tempi_amd

    L = ctypes.CDLL(os.path.join(tempi_amd.LIBDIR, "libtempi_apps.so"), mode=ctypes.RTLD_GLOBAL)
    L.tempi_bench_halo.argtypes = [ctypes.c_int] * 9 + [ctypes.c_char_p, ctypes.c_int]
    buf = ctypes.create_string_buffer(4096)
    g = grid or args.halo_grid
    rc = L.tempi_bench_halo(args.halo_iters, g, g, g, 8, 3, 0, 0, 0, buf, 4096)
    if rc != 0:
        raise RuntimeError(f"halo exchange failed rc={rc}")
    if not buf.value:
        return None
    r = json.loads(buf.value.decode())
    t = r["us_per_iter"] * 1e-6
    out = {
        "workload": (f"{g}^3 grid, 8 quantities x 8 B, radius 3, 26 neighbours, periodic, 3 substeps/iter, "
                     f"{world} rank(s) {r['dims']} (recursive bisection), MPI_Isend/Irecv/Wait of subarray types"),
        "grid": g,
        "dims": r["dims"],
        "us_per_iter": r["us_per_iter"],
        "us_min": r["us_min"],
        "bytes_per_iter_all_ranks": r["total_bytes_per_iter"],
        "busiest_peer_bytes_per_iter": r["max_peer_bytes_per_iter"],
        "rank0_phase_us": r.get("rank0_us_per_iter"),
    }
    out["payload_GBps_all_ranks"] = round(r["total_bytes_per_iter"] / t / 1e9, 1)
    # rank 0's own share: messages to itself are one strided -> strided copy
    # (read + write each payload byte once in HBM); messages to a peer are a
    # pack (read + write) here and a scatter on the peer that pulls the
    # packed bytes over xGMI (read there + write there)
    if world == 1:
        hbm_bytes = 2.0 * r["total_bytes_per_iter"]
        lb = hbm_bytes / (HBM_PEAK_GBS * 1e9)
        out["roofline"] = {"bound": "hbm", "algorithmic_bytes_per_iter": int(hbm_bytes),
                           "lower_bound_us": round(lb * 1e6, 1), "achieved_GBps": round(hbm_bytes / t / 1e9, 1),
                           "peak_GBps": HBM_PEAK_GBS, "frac": round(lb / t, 4),
                           "note": ("all 26 neighbours are this rank: every message is one strided->strided "
                                    "copy (2 x payload bytes algorithmic); the HBM bytes actually moved "
                                    "(traffic_per_iter, when measured) are ~1.9x that, because each 24-byte "
                                    "x-face row costs a whole-line read and 32-byte sector writes")}
        # an empirical floor for the GPU's share of an iteration, per substep:
        # the x faces as their bare access pattern timed on this box (the
        # packer's paired copy runs at or below it) + the other 24
        # regions' read + write at the achievable streaming rate
        # (apps/bench_lib.cpp tempi_bench_halo_floor)
        try:
            L.tempi_bench_halo_floor.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                                 ctypes.c_int]
            fb = ctypes.create_string_buffer(1024)
            if L.tempi_bench_halo_floor(g, 8, 10, fb, 1024) == 0 and fb.value:
                f = json.loads(fb.value.decode())
                rest_us = 2.0 * f["rest_payload_bytes"] / (HBM_ACHIEVABLE_GBS * 1e9) * 1e6
                floor_us = 3 * (f["x_faces_us"] + rest_us)
                out["floor"] = {"us_per_iter": round(floor_us, 1), "frac": round(floor_us / r["us_per_iter"], 4),
                                "x_faces_bare_us_per_substep": f["x_faces_us"],
                                "rest_streaming_us_per_substep": round(rest_us, 1),
                                "what": ("3 substeps x (x faces moved by a bare kernel, both faces of a row per "
                                         "lane, timed here + the other 24 regions' 2 x payload at "
                                         f"{HBM_ACHIEVABLE_GBS:.0f} GB/s)")}
        except Exception as e:  # (evidence beside the metric, never fatal)
            out["floor"] = {"error": str(e)[:200]}
        # the iteration split by TEMPI's own account (counters.ns_gpu_inflight:
        # a transport batch launched and not yet seen complete): GPU work, and
        # host-only time -- the send burst (every MPI_Isend of a substep is
        # posted before any receive exists, so nothing can run) and the rest
        # (first receives and launch, the waits' tail); DESIGN §6
        ph = r.get("rank0_us_per_iter") or {}
        if ph.get("gpu_inflight", -1) > 0:
            busy = ph["gpu_inflight"]
            out["split_us_per_iter"] = {"gpu_inflight": round(busy, 1),
                                        "host_only": round(r["us_per_iter"] - busy, 1),
                                        "send_burst": round(ph.get("isend", 0.0), 1)}
            fl = out.get("floor") or {}
            if "us_per_iter" in fl:
                fl["frac_of_gpu_inflight"] = round(fl["us_per_iter"] / busy, 4)
    else:
        # xGMI: the busiest point-to-point link carries max_peer bytes per iteration
        lb = r["max_peer_bytes_per_iter"] / (XGMI_LINK_GBS * 1e9)
        out["roofline"] = {"bound": "xgmi", "busiest_link_GBps": round(r["busiest_link_GBps"], 2),
                           "link_peak_GBps": XGMI_LINK_GBS, "frac": round(r["busiest_link_GBps"] / XGMI_LINK_GBS, 4),
                           "lower_bound_us": round(lb * 1e6, 1)}
        links = r.get("links_used") or 0
        if links:
            # sum of peer bytes / t / (directed links used x link peak)
            agg = r["remote_bytes_per_iter"] / t / 1e9
            out["roofline"].update({"remote_bytes_per_iter": int(r["remote_bytes_per_iter"]),
                                    "links_used": int(links), "aggregate_xgmi_GBps": round(agg, 1),
                                    "aggregate_frac": round(agg / (links * XGMI_LINK_GBS), 4)})
    return out


def tempi_cache_dir():
    """TEMPI_CACHE_DIR as libtempi resolves it (tempi_amd/csrc/core/env.cpp)"""
    if os.environ.get("TEMPI_CACHE_DIR"):
        return os.environ["TEMPI_CACHE_DIR"]
    if os.environ.get("XDG_CACHE_HOME"):
        return os.path.join(os.environ["XDG_CACHE_HOME"], "tempi")
    if os.environ.get("HOME"):
        return os.path.join(os.environ["HOME"], ".tempi")
    return "/var/tmp"


def node_perf_model(args, mpi, pg, rank, world, shared_gpu):
    """AUTO's model on this node: when TEMPI_CACHE_DIR/perf.json is missing,
    rank 0 measures it with apps/measure_system --quick (a 2-rank MPI job of
    its own, a child process: ranks 0 and 1 of the node, GPUs 0 and 1), then
    every rank re-reads the model. Reports which file AUTO uses."""
    import ctypes

    import tempi_amd

    path = os.path.join(tempi_cache_dir(), "perf.json")
    info = {"perf_json": path, "measured_here": False}
    if rank == 0 and not os.path.exists(path) and not args.no_measure_system:
        # (a failure here must not skip the barrier below: every rank waits there)
        try:
            os.makedirs(os.path.dirname(path), exist_ok=True)
            env = {k: v for k, v in os.environ.items() if not k.startswith(("PMI_", "MPI_LOCAL", "HYDRA_"))}
            env["HYDRA_LAUNCHER"] = "fork"
            exe = os.path.join(tempi_amd.LIBDIR, "measure_system")
            t0 = time.perf_counter()
            r = subprocess.run(["timeout", "-k", "10", "120", "/opt/conda/bin/mpiexec", "-n", "2", exe, "--quick",
                                "--out", path], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env)
            info["measure_seconds"] = round(time.perf_counter() - t0, 1)
            info["measured_here"] = r.returncode == 0 and os.path.exists(path)
            if not info["measured_here"]:
                info["measure_error"] = (r.stdout or "")[-400:]
        except Exception as e:
            info["measure_error"] = f"{type(e).__name__}: {e}"
    barrier(pg)
    mpi.L.tempi_perf_reload()
    buf = ctypes.create_string_buffer(4096)
    mpi.L.tempi_perf_source.argtypes = [ctypes.c_char_p, ctypes.c_int]
    loaded = mpi.L.tempi_perf_source(buf, 4096)
    info["auto_model"] = buf.value.decode() if loaded == 1 else "built-in policy (no perf.json)"
    if shared_gpu:
        info["note"] = ("shared GPU: the ranks share this box's MI355X, so a curve measured here is not an "
                        "xGMI curve")
    return info


def _smi_bytes(v):
    """an amd-smi metric value ({'value': x, 'unit': 'KB'} or 'N/A') in bytes"""
    if isinstance(v, dict) and isinstance(v.get("value"), (int, float)):
        unit = str(v.get("unit", "B")).upper()
        return float(v["value"]) * {"B": 1, "KB": 1024, "KIB": 1024, "MB": 1 << 20, "MIB": 1 << 20,
                                    "GB": 1 << 30, "GIB": 1 << 30}.get(unit, 1)
    if isinstance(v, (int, float)):
        return float(v)
    return None


def xgmi_snapshot():
    """amd-smi xgmi -m: {(gpu, peer): (read_bytes, write_bytes)} of the xGMI
    links that report data counters, or None when the tool or the counters
    are unavailable (a one-GPU box reports only its SELF link, 'N/A')"""
    import shutil

    if not shutil.which("amd-smi"):
        return None
    try:
        r = subprocess.run(["amd-smi", "xgmi", "-m", "--json"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, timeout=30)
        data = json.loads(r.stdout)
    except Exception:
        return None
    out = {}
    groups = data.get("xgmi_metric", []) if isinstance(data, dict) else data
    for grp in groups:
        for g in (grp if isinstance(grp, list) else [grp]):
            for i, link in enumerate((g.get("link_metrics") or {}).get("links", [])):
                rd, wr = _smi_bytes(link.get("read")), _smi_bytes(link.get("write"))
                if rd is None and wr is None:
                    continue
                out[(g.get("gpu"), link.get("gpu", i))] = (rd or 0.0, wr or 0.0)
    return out or None


def xgmi_delta(before, after, units_of_work, algorithmic_bytes, seconds):
    """counter-based xGMI bytes between two snapshots, per unit of work, next
    to the algorithmic bytes the app computed"""
    if before is None or after is None:
        return {"available": False,
                "note": "amd-smi reports no xGMI data counters on this node (one GPU: only its SELF link)"}
    rd = sum(max(0.0, after[k][0] - before[k][0]) for k in after if k in before)
    wr = sum(max(0.0, after[k][1] - before[k][1]) for k in after if k in before)
    moved = max(rd, wr)
    return {"available": True, "source": "amd-smi xgmi -m (per-link accumulated read / write data, all GPUs)",
            "read_bytes": int(rd), "write_bytes": int(wr), "per_unit_bytes": int(moved / max(units_of_work, 1)),
            "algorithmic_per_unit_bytes": int(algorithmic_bytes),
            "counter_GBps": round(moved / seconds / 1e9, 1) if seconds > 0 else None,
            "links_reporting": len(after)}


def apps_lib():
    import ctypes

    import tempi_amd

    L = ctypes.CDLL(os.path.join(tempi_amd.LIBDIR, "libtempi_apps.so"), mode=ctypes.RTLD_GLOBAL)
    L.tempi_bench_pingpong.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_long, ctypes.c_long, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.tempi_bench_alltoallv.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    L.tempi_bench_pingpong_1d.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_char_p,
                                          ctypes.c_int]
    L.tempi_bench_nbr_alltoallv.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    return L


def pingpong(args, world):
    """Config 3 between ranks 0 and 1 (every rank calls; others only barrier):
    strided vector(total/bl, bl, 512) MPI_Send/MPI_Recv of device buffers,
    AUTO method (IPC between co-located GPUs), one-way time."""
    import ctypes

    L = apps_lib()
    out = []
    for total, bl in ((4 << 20, 512), (4 << 20, 64), (1 << 20, 8), (1024, 8)):
        buf = ctypes.create_string_buffer(1024)
        rc = L.tempi_bench_pingpong(args.pp_iters, total, bl, 512, 0, 0, buf, 1024)
        if rc != 0:
            raise RuntimeError(f"pingpong failed rc={rc}")
        if buf.value:
            r = json.loads(buf.value.decode())
            r["xgmi_frac"] = round(r["GBps"] / XGMI_LINK_GBS, 4)
            out.append(r)
    return {"workload": ("config 3: MPI_Type_vector(total/bl, bl, 512, MPI_BYTE) MPI_Send/MPI_Recv ping-pong "
                         "rank 0 <-> 1, device buffers, one-way = trimean(round trip)/2"),
            "link_peak_GBps": XGMI_LINK_GBS, "points": out}


def pingpong_1d(args, world):
    """The reference's bench_mpi_pingpong_1d (contiguous
    senders): MPI_BYTE count = 2 MiB and 16 MiB of device buffers, ranks r and
    r + N/2 paired, all pairs at once, one-way = trimean(max over ranks of the
    round trip) / 2; aggregate = the pairs' bytes in flight per one-way time."""
    import ctypes

    L = apps_lib()
    out = []
    for total in (1 << 21, 1 << 24):
        buf = ctypes.create_string_buffer(1024)
        rc = L.tempi_bench_pingpong_1d(args.pp_iters, total, 0, 0, buf, 1024)
        if rc != 0:
            raise RuntimeError(f"pingpong_1d failed rc={rc}")
        if buf.value:
            r = json.loads(buf.value.decode())
            r["xgmi_frac"] = round(r["pair_GBps"] / XGMI_LINK_GBS, 4)
            out.append(r)
    return {"workload": ("bench_mpi_pingpong_1d: MPI_BYTE MPI_Send/MPI_Recv of device buffers, ranks r <-> r + N/2, "
                         "all pairs at once"), "link_peak_GBps": XGMI_LINK_GBS, "points": out}


def alltoallv(args, world):
    """Config 5: MPI_BYTE MPI_Alltoallv of device buffers with the
    reference's random sparse count matrix (seed 101), min over iterations
    of the max over ranks."""
    import ctypes

    L = apps_lib()
    out = []
    for scale, density in ((100000, 1.0), (100000, 0.5), (1000, 1.0)):
        buf = ctypes.create_string_buffer(1024)
        rc = L.tempi_bench_alltoallv(args.a2av_iters, scale, density, 101, 0, 0, buf, 1024)
        if rc != 0:
            raise RuntimeError(f"alltoallv failed rc={rc}")
        if buf.value:
            r = json.loads(buf.value.decode())
            # every GPU pair has its own xGMI link: the largest pairwise
            # message bounds the exchange
            lb = r["max_pairwise_bytes"] / (XGMI_LINK_GBS * 1e9)
            r["lower_bound_us"] = round(lb * 1e6, 2)
            r["xgmi_frac"] = round(lb / (r["min_us"] * 1e-6), 4) if r["min_us"] > 0 else None
            out.append(r)
    return {"workload": ("config 5: bench-mpi-random-alltoallv, SquareMat::make_random_sparse(size, "
                         "round(density*size), 1, 10, scale, 101) byte counts, device buffers"),
            "points": out}


def _line_classes(bl, st, n, first):
    """Per 128-B line of the strided side of n rows of bl bytes at stride st
    (first row at byte `first`): (lines touched, lines with a partly written
    64-B sector, lines written whole, lines with one whole sector and one
    untouched). Counted exactly on a sample of whole periods of the row
    pattern (>= 64 KiB of address span) and scaled to n rows."""
    import numpy as np

    p = 128 // math.gcd(st, 128)  # rows after which the pattern repeats modulo a line
    m = min(n, max(p, -(-65536 // st)))
    m = min(n, -(-m // p) * p)
    lo = first - first % 128
    span = (m - 1) * st + bl + (first - lo)
    cov = np.zeros(-(-span // 128) * 128, dtype=np.uint8)
    starts = first - lo + np.arange(m, dtype=np.int64) * st
    for b in range(bl):  # bl <= 4096; vectorised over rows
        cov[starts + b] = 1
    sec = cov.reshape(-1, 2, 64).sum(axis=2)  # bytes covered per sector
    touched = (sec > 0).any(axis=1)
    partial = ((sec > 0) & (sec < 64)).any(axis=1)
    whole = (sec == 64).all(axis=1)
    half = touched & ~partial & ~whole
    s = n / m
    return touched.sum() * s, partial.sum() * s, whole.sum() * s, half.sum() * s


# Write cost per line, in bytes of full-line streaming, from the box's
# calibration (profiles/r02/counter_calibration.txt: whole lines 5.6-5.7 TB/s,
# one whole sector per line 7.5-7.6 TB/s of lines, lines with a partly
# written sector 2.3-2.7 TB/s of lines: a DRAM read-modify-write)
LINE_WRITE_WHOLE, LINE_WRITE_HALF, LINE_WRITE_PARTIAL = 128.0, 96.0, 292.0
# A line with one whole 64-B sector written and the other untouched costs more
# as such lines get sparser (fewer written sectors per DRAM page): the bare
# pattern (tools/calib.hip sect_copy, 64-B rows at stride S, the kernel's tile
# order) runs 5.25 / 4.63 / 4.27 / 4.00 / 3.96 TB/s (read + write) at S = 128
# / 256 / 512 / 1024 / 4096 (round 3, profiles/r03/sect3_s4.jsonl), i.e.
# 90 / 110 / 125 / 138 / 140 bytes-equivalent per line at 6.3 TB/s
HALF_LINE_COST = ((128, 90.0), (256, 110.0), (512, 125.0), (1024, 138.0), (4096, 140.0))


def half_line_cost(stride):
    """bytes-equivalent of a line written in one whole sector, rows `stride`
    bytes apart (log-linear between the calibrated strides, clamped)"""
    pts = HALF_LINE_COST
    if stride <= pts[0][0]:
        return pts[0][1]
    for (s0, c0), (s1, c1) in zip(pts, pts[1:]):
        if stride <= s1:
            f = (math.log(stride) - math.log(s0)) / (math.log(s1) - math.log(s0))
            return c0 + f * (c1 - c0)
    return pts[-1][1]


def touched_model(bl, st, nplanes, rows, plane_stride, first):
    """Bytes-equivalent one pack and one unpack of this config-2 shape must
    move at the memory side, to be divided by the achievable streaming rate:
    pack = every 128-B line the strided side touches (a read fetches whole
    lines, any load flavour) + the packed bytes written whole; unpack = the
    packed bytes read + each strided-side line at its calibrated write cost
    (whole, one whole sector, or a partly written sector). Planes of a 3D
    shape are counted at the first plane's alignment (their offsets differ by
    less than a line per plane)."""
    payload = nplanes * rows * bl
    touched, partial, whole, half = _line_classes(bl, st, rows, first)
    return {"pack_bytes": nplanes * touched * 128.0 + payload,
            "unpack_bytes": payload + nplanes * (whole * LINE_WRITE_WHOLE + half * half_line_cost(st) +
                                                 partial * LINE_WRITE_PARTIAL)}


def nbr_alltoallv(args, world):
    """Config 5's neighbourhood form (bench_nbr_alltoallv_random_sparse.cpp):
    the same matrices as a distributed graph created with reorder = 1 (the
    reference's KaHIP remapping is a no-op on one node, F12), then MPI_BYTE
    MPI_Neighbor_alltoallv of device buffers; min over iterations of the max
    over ranks."""
    import ctypes

    L = apps_lib()
    out = []
    for scale, density in ((100000, 1.0), (100000, 0.5), (1000, 1.0)):
        buf = ctypes.create_string_buffer(2048)
        rc = L.tempi_bench_nbr_alltoallv(args.a2av_iters, scale, density, 101, 1, 0, 0, buf, 2048)
        if rc != 0:
            raise RuntimeError(f"neighbor alltoallv failed rc={rc}")
        if buf.value:
            r = json.loads(buf.value.decode())
            lb = r["max_pairwise_bytes"] / (XGMI_LINK_GBS * 1e9)
            r["lower_bound_us"] = round(lb * 1e6, 2)
            r["xgmi_frac"] = round(lb / (r["min_us"] * 1e-6), 4) if r["min_us"] > 0 else None
            out.append(r)
    return {"workload": ("config 5, neighbourhood form: bench-nbr-alltoallv-random-sparse, the same matrices as "
                         "MPI_Dist_graph_create_adjacent(reorder = 1) + MPI_Neighbor_alltoallv, device buffers"),
            "points": out}


def sweep_shape(mpi, bl, st, dims, packed_target):
    """One config-2 sweep shape: (uncommitted type, extent, label, planes,
    payload). planes = (planes, rows per plane, plane stride, first byte) for
    touched_model."""
    rows = packed_target // bl
    if dims == 2:
        t = mpi.Type_create_subarray([rows, st], [rows, bl], [0, 0], mpi.ORDER_C, mpi.BYTE)
        extent = rows * st
        shape = f"2d rows={rows} stride={st}"
        planes = (1, rows, 0, 0)
    else:
        y = max(1, int(rows ** 0.5))
        z = max(1, rows // y)
        rows = y * z
        Y = y + 3
        t = mpi.Type_create_subarray([z + 2, Y, st], [z, y, bl], [1, 2, 0], mpi.ORDER_C, mpi.BYTE)
        extent = (z + 2) * Y * st
        shape = f"3d {z}x{y} rows pitch={st} ypad=3"
        planes = (z, y, Y * st, Y * st + 2 * st)
    return t, extent, shape, planes, rows * bl


def sweep(args, mpi, torch, dev, path, sizes=(1 << 20, 16 << 20, 256 << 20, 1 << 30), quiet=False):
    """Config-2 sweep: 2D subarray and 3D subarray, block 1 B - 4 KiB.
    Returns the records (also written to `path` when given)."""
    recs = []
    blocks = [1, 2, 3, 4, 8, 12, 16, 24, 32, 64, 128, 256, 512, 1024, 2048, 4096]
    for packed_target in sizes:
        for bl in blocks:
            strides = sorted({2 * bl, bl + 16} | ({512} if bl <= 256 else set()))
            for st in strides:
                for dims in (2, 3):
                    t, extent, shape, planes, payload = sweep_shape(mpi, bl, st, dims, packed_target)
                    if extent > (12 << 30):
                        mpi.Type_free(t)
                        continue
                    t = mpi.Type_commit(t)
                    src = torch.empty(extent, dtype=torch.uint8, device=dev)
                    pk = torch.empty(payload, dtype=torch.uint8, device=dev)
                    torch.cuda.synchronize()
                    reps = max(30, min(50, int(2e9 / max(payload, 1))))  # (>= 30 iterations)
                    mpi.Pack(src.data_ptr(), 1, t, pk.data_ptr(), payload, 0)
                    mpi.Unpack(pk.data_ptr(), payload, 0, src.data_ptr(), 1, t)
                    mpi.reset_counters()
                    mpi.set_kernel_profiling(True)
                    t0 = time.perf_counter()
                    for _ in range(reps):
                        mpi.Pack(src.data_ptr(), 1, t, pk.data_ptr(), payload, 0)
                    t1 = time.perf_counter()
                    for _ in range(reps):
                        mpi.Unpack(pk.data_ptr(), payload, 0, src.data_ptr(), 1, t)
                    t2 = time.perf_counter()
                    mpi.set_kernel_profiling(False)
                    kt = mpi.kernel_times()
                    pk_ms = kt["pack_ms"] / reps
                    up_ms = kt["unpack_ms"] / reps
                    rec = {"shape": shape, "block": bl, "stride": st, "packed": payload, "extent": extent,
                           "pack_kernel_ms": pk_ms, "unpack_kernel_ms": up_ms,
                           "pack_api_ms": (t1 - t0) / reps * 1e3, "unpack_api_ms": (t2 - t1) / reps * 1e3,
                           "pack_alg_gbs": 2 * payload / (pk_ms * 1e-3) / 1e9,
                           "unpack_alg_gbs": 2 * payload / (up_ms * 1e-3) / 1e9}
                    tb = touched_model(bl, st, *planes)
                    rec.update({"pack_touched_bytes": tb["pack_bytes"], "unpack_touched_bytes": tb["unpack_bytes"],
                                "pack_frac_touched": tb["pack_bytes"] / (HBM_ACHIEVABLE_GBS * 1e9) / (pk_ms * 1e-3),
                                "unpack_frac_touched": tb["unpack_bytes"] / (HBM_ACHIEVABLE_GBS * 1e9) / (up_ms * 1e-3)})
                    recs.append(rec)
                    if not quiet:
                        print(json.dumps(rec), flush=True)
                    mpi.Type_free(t)
                    del src, pk
    if path:
        with open(path, "w") as f:
            json.dump(recs, f, indent=1)
    return recs


def sweep_traffic(specs):
    """FETCH_SIZE / WRITE_SIZE counted per sweep shape against the touched
    model's raw bytes (tools/sweep_pmc.py): model / counted ratios, and the
    shapes re-scored where the model over-predicts by more than 10 %"""
    import shutil

    if not shutil.which("rocprofv3") or any(k.startswith("ROCPROF") for k in os.environ) or \
            "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None  # (no profiler, or already under one: see run_traffic_passes)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import sweep_pmc

    outdir = os.path.join(ROOT, "gpurun_out") if os.path.isdir(os.path.join(ROOT, "gpurun_out")) else None
    recs = sweep_pmc.run(specs, outdir, echo=False)  # (stdout carries the bench line only)
    keep = ("spec", "shape", "pack_model_over_counted", "unpack_model32_over_counted", "pack_frac_touched",
            "unpack_frac_touched", "pack_frac_counted", "unpack_frac_counted", "pack_rescored_frac_touched",
            "unpack_rescored_frac_touched", "counted", "model")
    return [{k: r[k] for k in keep if k in r} for r in recs]


def sweep_geomean(args, mpi, torch, dev):
    """The config-2 sweep's 1 GiB points (2D and 3D subarrays, block 1 B -
    4 KiB, strides 2*bl / bl+16 / 512): geometric mean of algorithmic GB/s
    (kernel time, HIP events), and how many reach 70 % of the 8 TB/s spec."""
    recs = sweep(args, mpi, torch, dev, None, sizes=(1 << 30,), quiet=True)
    if not recs:
        return None

    def gm(xs):
        return math.exp(sum(math.log(x) for x in xs) / len(xs))

    pk = [r["pack_alg_gbs"] for r in recs]
    up = [r["unpack_alg_gbs"] for r in recs]
    pkt = [r["pack_frac_touched"] for r in recs]
    upt = [r["unpack_frac_touched"] for r in recs]
    worst = sorted(recs, key=lambda r: min(r["pack_alg_gbs"], r["unpack_alg_gbs"]))[:3]
    worst_t = sorted(recs, key=lambda r: min(r["pack_frac_touched"], r["unpack_frac_touched"]))[:3]
    return {"points": len(recs), "packed_bytes": 1 << 30,
            "pack_GBps": round(gm(pk), 1), "unpack_GBps": round(gm(up), 1),
            "pack_frac": round(gm(pk) / HBM_PEAK_GBS, 4), "unpack_frac": round(gm(up) / HBM_PEAK_GBS, 4),
            "pack_ge_0.7": sum(x >= 0.7 * HBM_PEAK_GBS for x in pk),
            "unpack_ge_0.7": sum(x >= 0.7 * HBM_PEAK_GBS for x in up),
            "worst": [{"shape": r["shape"], "block": r["block"], "stride": r["stride"],
                       "pack_GBps": round(r["pack_alg_gbs"], 1), "unpack_GBps": round(r["unpack_alg_gbs"], 1)}
                      for r in worst],
            # the same points against the bytes the memory side must move
            # (touched_model: whole lines read, partial sectors read-modify-
            # written) at the 6.3 TB/s achievable rate
            "pack_frac_touched": round(gm(pkt), 4), "unpack_frac_touched": round(gm(upt), 4),
            "worst_touched": [{"shape": r["shape"], "block": r["block"], "stride": r["stride"],
                               "pack_frac_touched": round(r["pack_frac_touched"], 3),
                               "unpack_frac_touched": round(r["unpack_frac_touched"], 3)} for r in worst_t],
            "touched_model": ("pack: 128-B lines touched on the strided side + packed bytes; unpack: packed bytes + "
                              "each strided-side line at its calibrated write cost (whole 128, one whole sector 90-140 "
                              "by row stride, a partly written sector 292 bytes-equivalent: DRAM read-modify-write), "
                              "all at 6.3 TB/s; profiles/r02/counter_calibration.txt, profiles/r03/sect3_s4.jsonl"),
            "workload": "config 2 at 1 GiB packed: MPI_Type_create_subarray 2D {rows, S} and 3D {z+2, y+3, S}, "
                        "block 1 B - 4 KiB, S in {2*bl, bl+16, 512 (bl <= 256)}; kernel time per MPI_Pack / "
                        "MPI_Unpack from HIP events on TEMPI's stream"}


SHARED_GPU_NOTE = ("ranks share one GPU: no byte crosses xGMI, so xGMI fractions are null (the algorithmic bytes "
                   "never left HBM)")


def null_shared_gpu_fractions(rec):
    """With ranks sharing one GPU an 'xGMI' fraction is physically
    meaningless (it exceeds the link peak): null every one of them"""
    for name in ("halo", "halo_weak"):
        r = (rec.get(name) or {}).get("roofline")
        if r and r.get("bound") == "xgmi":
            for k in ("frac", "aggregate_frac", "busiest_link_GBps", "aggregate_xgmi_GBps"):
                if k in r:
                    r[k] = None
            r["note"] = SHARED_GPU_NOTE
    for name in ("pingpong", "pingpong_1d", "alltoallv", "nbr_alltoallv"):
        p = rec.get(name)
        if isinstance(p, dict) and "points" in p:
            for q in p["points"]:
                q["xgmi_frac"] = None
            p["note"] = SHARED_GPU_NOTE


LINE_LIMIT = 3800  # bytes of the final stdout line; the driver keeps ~8 KB of stdout tail


def _sig(x, digits=4):
    """a float rounded to `digits` significant digits (ints and None pass)"""
    if isinstance(x, float) and x != 0 and math.isfinite(x):
        return float(f"{x:.{digits}g}")
    return x


def _err(sec):
    return {"error": str(sec["error"])[:160]} if isinstance(sec, dict) and "error" in sec else None


def _compact_sections(rec, shared_gpu):
    """{name: compact summary} of every section after the headline; each
    one's full record stays in the detail file"""
    out = {}
    s = rec.get("sweep_geomean")
    if s:
        out["sweep"] = _err(s) or {
            "points": s["points"], "pack_GBps": s["pack_GBps"], "unpack_GBps": s["unpack_GBps"],
            "pack_frac": s["pack_frac"], "unpack_frac": s["unpack_frac"], "pack_ge_0.7": s["pack_ge_0.7"],
            "unpack_ge_0.7": s["unpack_ge_0.7"], "pack_frac_touched": s["pack_frac_touched"],
            "unpack_frac_touched": s["unpack_frac_touched"],
            "worst_touched": [f"{w['shape'].split()[0]} {w['block']}:{w['stride']} p{w['pack_frac_touched']:.3f} "
                              f"u{w['unpack_frac_touched']:.3f}" for w in s.get("worst_touched", [])]}
    for name in ("halo", "halo_weak"):
        h = rec.get(name)
        if not h:
            continue
        e = _err(h)
        if e:
            out[name] = e
            continue
        r = h.get("roofline") or {}
        c = {"grid": h.get("grid"), "dims": h.get("dims"), "us_per_iter": h["us_per_iter"], "us_min": h["us_min"],
             "bound": r.get("bound"), "frac": r.get("frac")}
        if r.get("bound") == "hbm":
            c.update({"alg_bytes_per_iter": r.get("algorithmic_bytes_per_iter"),
                      "traffic_per_iter": r.get("traffic_per_iter"), "frac_touched": r.get("frac_touched")})
        else:
            c.update({"busiest_link_GBps": r.get("busiest_link_GBps"), "aggregate_frac": r.get("aggregate_frac"),
                      "remote_bytes_per_iter": r.get("remote_bytes_per_iter")})
            x = h.get("xgmi_counters") or {}
            c["xgmi_counter_bytes_per_iter"] = x.get("per_unit_bytes") if x.get("available") else None
        fl = h.get("floor") or {}
        if "frac" in fl:
            c["floor_us_per_iter"], c["frac_floor"] = fl["us_per_iter"], fl["frac"]
            if "frac_of_gpu_inflight" in fl:
                c["frac_floor_of_gpu_inflight"] = fl["frac_of_gpu_inflight"]
        if h.get("split_us_per_iter"):
            c["split_us_per_iter"] = h["split_us_per_iter"]
        if h.get("rank0_phase_us"):
            c["rank0_phase_us"] = h["rank0_phase_us"]
        cb = h.get("cpu_baseline")
        if cb and "value" in cb:
            c["cpu_us_per_iter"] = _sig(cb["value"])
        out[name] = c
    if rec.get("config1"):
        c = rec["config1"]
        out["config1"] = _err(c) or {k: c.get(k) for k in ("cpu_us", "gpu_us", "speedup", "gpu_matches_cpu")}
        cp = c.get("c_phases") or {}
        if "phases_us" in cp and isinstance(out["config1"], dict):
            out["config1"]["c"] = {"gpu_us": cp.get("mpi_pack_device_us"), "mpich_us": cp.get("mpich_host_us"),
                                   "speedup": cp.get("c_speedup"), "phases_us": cp["phases_us"]}
    if rec.get("type_commit"):
        c = rec["type_commit"]
        out["type_commit"] = _err(c) or {"tempi_us": c["tempi"]["commit_us_median"],
                                         "library_us": c["library"]["commit_us_median"]}
    if rec.get("mpi_pack"):
        c = rec["mpi_pack"]
        out["mpi_pack"] = _err(c) or {"errors": c["errors"], "points": len(c.get("points", [])),
                                      "pack_speedup_geomean_by_target": c["pack_speedup_geomean_by_target"]}
    lb = rec.get("cpu_baselines_configs_3_5")
    if lb:
        c = _err(lb) or {}
        if not c:
            if "halo" in lb:
                c["halo_us_per_iter"] = _sig(lb["halo"]["value"])
            if "pingpong" in lb:
                c["pingpong_oneway_us"] = [[p["total"], p["block"], _sig(p["oneway_us"])] for p in lb["pingpong"]["points"]]
            if "alltoallv" in lb:
                c["alltoallv_us"] = _sig(lb["alltoallv"]["value"])
            c["cores"] = "halo 1, pingpong 2, alltoallv 8 (MPICH, TEMPI_DISABLE=1, host buffers)"
        out["cpu_baselines_configs_3_5"] = c
    for name, cols in (("pingpong", ("total", "block", "oneway_us", "GBps", "xgmi_frac")),
                       ("pingpong_1d", ("total", "pairs", "oneway_us", "aggregate_GBps", "xgmi_frac")),
                       ("alltoallv", ("scale", "density", "min_us", "max_pairwise_bytes", "xgmi_frac")),
                       ("nbr_alltoallv", ("scale", "density", "min_us", "max_pairwise_bytes", "xgmi_frac"))):
        p = rec.get(name)
        if not p:
            continue
        out[name] = _err(p) or {"cols": list(cols), "points": [[_sig(q.get(k)) for k in cols] for q in p["points"]],
                                "errors": sum(q.get("errors", 0) for q in p["points"])}
    t = rec.get("transport")
    if t:
        out["transport"] = _err(t) or {
            "routes": {k: [v["messages"], v["bytes"]] for k, v in t["routes"].items() if v["messages"]},
            "library_sends": t["library_sends"], "canary_ok": t["canary_ok"], "canary_fail": t["canary_fail"],
            "ipc_threshold": t["ipc_threshold"], "perf_json_measured_on_node": t["perf_json_measured_on_node"]}
        if t.get("canary_note"):
            out["transport"]["null_because"] = "shared GPU"
    if rec.get("perf_model"):
        pm = rec["perf_model"]
        out["perf_model"] = _err(pm) or {"measured_here": pm.get("measured_here"),
                                         "auto_model": os.path.basename(str(pm.get("auto_model", ""))) or None}
    return out


# sections dropped, in this order, if the line is still over LINE_LIMIT
_DROP_ORDER = ("mpi_pack", "type_commit", "perf_model", "cpu_baselines_configs_3_5", "halo_weak", "transport",
               "nbr_alltoallv",
               "pingpong_1d", "alltoallv", "pingpong", "config1", "sweep")


def compact_line(rec, shared_gpu=False, detail=None, limit=LINE_LIMIT):
    """The driver's one JSON line: the contract's keys, the headline's
    roofline and cpu_baseline, and a bounded summary of every other section
    (the full record goes to the detail file). Guaranteed <= limit bytes."""
    line = {k: rec[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config") if k in rec}
    ro = rec.get("roofline")
    if ro:
        line["roofline"] = {k: ro[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "traffic_read",
                                               "traffic_write", "kernel", "algorithmic_bytes_per_launch",
                                               "avg_launch_ms", "pack_avg_ms", "unpack_avg_ms", "timed_launches",
                                               "achievable_peak", "frac_achievable", "d2d_copy_GBps",
                                               "traffic_error") if k in ro}
    cb = rec.get("cpu_baseline")
    if cb:
        line["cpu_baseline"] = _err(cb) or {k: cb[k] for k in ("value", "unit", "cores", "kind", "sample") if k in cb}
    if rec.get("incomplete"):
        line["incomplete"] = rec["incomplete"]
    line["shared_gpu"] = bool(shared_gpu)
    secs = _compact_sections(rec, shared_gpu)
    line.update(secs)
    if detail:
        line["detail"] = detail
    dropped = []
    for name in _DROP_ORDER:
        if len(json.dumps(line)) <= limit:
            break
        if name in line:
            del line[name]
            dropped.append(name)
    if dropped:
        line["dropped"] = dropped
    while len(json.dumps(line)) > limit:  # last resort: never hand the driver an unparseable tail
        extra = [k for k in line if k not in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                              "higher_is_better", "scaling", "vs_baseline", "dtype", "data",
                                              "config", "roofline", "cpu_baseline")]
        if not extra:
            line["config"] = {"workload": str(line.get("config", {}).get("workload", ""))[:120]}
            line.get("cpu_baseline", {}).pop("sample", None)
            break
        del line[extra[-1]]
    return line


DETAIL_NAME = None  # --detail-name


def write_detail(rec, world):
    """the full record, next to the line (gpurun_out/ is merged back from a
    builder's GPU session); returns the path relative to the repo for the
    line's "detail" key only when --detail-name named it: the driver's own
    run does not retrieve gpurun_out/, so its line names no file it cannot
    read"""
    d = os.path.join(ROOT, "gpurun_out")
    path = os.path.join(d, os.path.basename(DETAIL_NAME or f"bench_detail_n{world}.json"))
    try:
        os.makedirs(d, exist_ok=True)
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
        return os.path.relpath(path, ROOT) if DETAIL_NAME else None
    except OSError:
        return None


class Sections:
    """The sections after the headline (sweep, halo, configs 3 and 5,
    traffic, CPU baselines) are evidence beside the metric, not the metric:
    one that raises is recorded as {"error": ...} in its field, and one that
    has not finished `deadline` seconds after the headline (a hang on a node
    this pool never ran, e.g. the first cross-GPU IPC) ends the run with the
    line so far, its "incomplete" field naming the section."""

    def __init__(self, rec, rank, deadline, world=1, shared_gpu=False):
        import threading

        self.rec, self.rank, self.current = rec, rank, "start"
        self.world, self.shared_gpu = world, shared_gpu
        self.timer = threading.Timer(deadline, self._expire, args=(deadline,))
        self.timer.daemon = True
        self.timer.start()

    def _expire(self, deadline):
        if self.rank == 0:
            line = dict(self.rec)
            line["incomplete"] = {"section": self.current, "deadline_s": deadline}
            try:
                if self.shared_gpu:
                    null_shared_gpu_fractions(line)
                print(json.dumps(compact_line(line, self.shared_gpu, write_detail(line, self.world))), flush=True)
            except Exception as e:  # a section was mutating the record
                print(json.dumps({k: line[k] for k in ("metric", "value", "unit", "n_gpus") if k in line} |
                                 {"incomplete": {"section": self.current, "deadline_s": deadline,
                                                 "print_error": str(e)[:200]}}), flush=True)
        sys.stdout.flush()
        os._exit(0)

    def run(self, name, fn, *a, **kw):
        self.current = name
        t0 = time.perf_counter()
        try:
            return fn(*a, **kw)
        except Exception as e:
            return {"error": f"{type(e).__name__}: {e}"}
        finally:  # progress on stderr (a long multi-rank run is never silent for minutes)
            if self.rank == 0:
                print(f"[bench] {name}: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)

    def done(self):
        self.timer.cancel()


def main():
    global DETAIL_NAME
    args = parse()
    DETAIL_NAME = args.detail_name
    rank, world, local, pg, keep = dist_setup(args)
    import torch

    import tempi_amd

    dev = torch.device("cuda", local % max(torch.cuda.device_count(), 1))  # ranks may share a GPU when testing
    torch.cuda.set_device(dev)
    mpi = tempi_amd.get_mpi()
    mpi.Init()
    try:
        assert mpi.gpu_available(), "libtempi.so found no GPU"
        if args.sweep:
            if args.sweep_sizes:
                sweep(args, mpi, torch, dev, args.sweep, sizes=tuple(int(x) for x in args.sweep_sizes.split(",")))
            else:
                sweep(args, mpi, torch, dev, args.sweep)
            return
        rec = headline(args, mpi, torch, rank, world, pg, dev)
        if args.inner:
            return
        torch.cuda.empty_cache()
        shared_gpu = world > max(torch.cuda.device_count(), 1)
        sec = Sections(rec, rank, args.extras_deadline, world, shared_gpu)
        if world == 1 and not args.no_sweep_geomean:
            rec["sweep_geomean"] = sec.run("sweep_geomean", sweep_geomean, args, mpi, torch, dev)
            torch.cuda.empty_cache()
        if world > 1:
            pm = sec.run("perf_model", node_perf_model, args, mpi, pg, rank, world, shared_gpu)
            if rank == 0:
                rec["perf_model"] = pm
        c_start = mpi.counters() if world > 1 else None
        if not args.no_halo:
            barrier(pg)
            snap0 = xgmi_snapshot() if world > 1 and rank == 0 else None
            c_halo0 = mpi.counters() if world > 1 else None
            t0 = time.perf_counter()
            h = sec.run("halo", halo, args, mpi, world)
            barrier(pg)
            el = time.perf_counter() - t0
            if world > 1:
                tb = sec.run("transport", transport_block, mpi, pg, c_halo0, mpi.counters(), shared_gpu,
                             "the halo section (config 4), all ranks")
                if rank == 0 and h and "error" not in h:
                    h["transport"] = tb
            if rank == 0:
                rec["halo"] = h
                if world > 1 and h and "error" not in h:
                    iters = args.halo_iters + 1  # the app's warm-up iteration moves the same bytes
                    x = xgmi_delta(snap0, xgmi_snapshot(), iters,
                                   (h.get("roofline") or {}).get("remote_bytes_per_iter", 0), el)
                    if shared_gpu:
                        x["note"] = ("shared GPU: the ranks share this box's MI355X, no byte crosses xGMI; "
                                     "the algorithmic fractions above only say the bytes never left HBM")
                    h["xgmi_counters"] = x
            if world > 1:  # the reference scripts' weak scaling: 512 * N^(1/3) per edge
                hw = sec.run("halo_weak", halo, args, mpi, world,
                             grid=int(round(args.halo_grid * world ** (1.0 / 3.0))))
                if rank == 0:
                    rec["halo_weak"] = hw
        if world > 1 and not args.no_p2p:
            barrier(pg)
            pp = sec.run("pingpong", pingpong, args, world)
            barrier(pg)
            p1 = sec.run("pingpong_1d", pingpong_1d, args, world)
            barrier(pg)
            a2 = sec.run("alltoallv", alltoallv, args, world)
            barrier(pg)
            na = sec.run("nbr_alltoallv", nbr_alltoallv, args, world)
            if rank == 0:
                rec["pingpong"] = pp
                rec["pingpong_1d"] = p1
                rec["alltoallv"] = a2
                rec["nbr_alltoallv"] = na
        if world > 1:
            barrier(pg)
            tr = sec.run("transport", transport_block, mpi, pg, c_start, mpi.counters(), shared_gpu,
                         "every N > 1 section (halo, halo_weak, pingpong, pingpong_1d, alltoallv, nbr_alltoallv), "
                         "all ranks")
            if rank == 0:
                rec["transport"] = tr
        if rank == 0 and world == 1:
            if not args.no_traffic:
                tr = sec.run("traffic", run_traffic_passes, args, "pack_kernel")
                if isinstance(tr, dict):
                    rec["roofline"]["traffic_error"] = tr["error"]
                elif tr:
                    rec["roofline"]["traffic"] = int(tr[0] + tr[1])
                    rec["roofline"]["traffic_read"] = int(tr[0])
                    rec["roofline"]["traffic_write"] = int(tr[1])
                    rec["roofline"]["traffic_source"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes, "
                                                         "per launch of pack_kernel/unpack_kernel, FETCH_SIZE x2 "
                                                         "(gfx950)")
                if args.sweep_traffic not in (None, "", "none") and isinstance(rec.get("sweep_geomean"), dict):
                    tc = sec.run("sweep_traffic", sweep_traffic, args.sweep_traffic.split(","))
                    rec["sweep_geomean"]["traffic_checked"] = tc
                if rec.get("halo") and "error" not in rec["halo"]:
                    ht = sec.run("halo_traffic", halo_traffic, args)
                    if isinstance(ht, dict):
                        rec["halo"]["roofline"]["traffic_error"] = ht["error"]
                    elif ht:
                        hr = rec["halo"]["roofline"]
                        tr_iter = ht[0] + ht[1]
                        lb = tr_iter / (HBM_ACHIEVABLE_GBS * 1e9)
                        hr["traffic_per_iter"] = int(tr_iter)
                        hr["traffic_read_per_iter"] = int(ht[0])
                        hr["traffic_write_per_iter"] = int(ht[1])
                        hr["touched_lower_bound_us"] = round(lb * 1e6, 1)
                        hr["frac_touched"] = round(lb / (rec["halo"]["us_per_iter"] * 1e-6), 4)
                        hr["traffic_source"] = ("rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate runs) over the "
                                                "copy kernels of halo_exchange 3 GRID, per iteration, FETCH_SIZE x2; "
                                                "bound at the 6.3 TB/s achievable rate")
            if not args.no_cpu_baseline:
                rec["cpu_baseline"] = sec.run("cpu_baseline", cpu_baseline, mpi, args.rows, args.pitch, args.block,
                                              args.cpu_seconds)
                rec["config1"] = sec.run("config1", config1, mpi, torch, dev)
                rec["type_commit"] = sec.run("type_commit", type_commit_cost)
                rec["mpi_pack"] = sec.run("mpi_pack", mpi_pack_bench)
                lb = sec.run("cpu_baselines_configs_3_5", library_path_baselines, args)
                if lb:
                    rec["cpu_baselines_configs_3_5"] = lb
                    if "halo" in lb and rec.get("halo") and "error" not in rec["halo"]:
                        rec["halo"]["cpu_baseline"] = lb["halo"]
        sec.done()
        if rank == 0:
            if shared_gpu:
                null_shared_gpu_fractions(rec)
            print(json.dumps(compact_line(rec, shared_gpu, write_detail(rec, world))), flush=True)
    finally:
        mpi.Finalize()
        if pg is not None:
            pg.destroy_process_group()


if __name__ == "__main__":
    main()
