"""Counter check of the config-2 sweep's traffic model.

bench.py scores each 1 GiB sweep shape against `touched_model`: the bytes the
memory side must move (pack: every 128-B line the strided side touches is
fetched whole + the packed bytes written; unpack: the packed bytes read + the
strided side's lines written, weighted by their calibrated write cost). This
tool measures those bytes: per shape, one process runs 1 + 5 MPI_Pack and
1 + 5 MPI_Unpack of the shape under `rocprofv3 --pmc FETCH_SIZE`, another
under `--pmc WRITE_SIZE` (one counter per pass), and the per-launch averages
of the pack and unpack kernels (FETCH_SIZE x 2, the gfx950 correction of
MI355X_MICROARCH.md) are set beside the model's raw-byte prediction:
  pack    read  = lines touched x 128        write = payload
  unpack  read  = payload                    write = 32-B chunks touched x 32
                                                     (and 64-B sectors x 64)
The ratio model / counter > 1.10 means the model over-predicts the traffic:
that shape's frac_touched is then re-scored with the counted bytes
(`rescored_frac_touched`, the counted bytes at 6.3 TB/s over the kernel
time of a third run of the same child without a profiler: counter
collection serialises and slows the dispatches it counts).

usage (GPU box): python3 tools/sweep_pmc.py OUT.json DIMS:BLOCK:STRIDE ...
       python3 tools/sweep_pmc.py --one DIMS:BLOCK:STRIDE   (the profiled child)"""
import csv
import glob
import json
import math
import os
import subprocess
import sys
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)

PACKED = 1 << 30
REPS = 5


def chunks_touched(bl, st, n, first, size):
    """size-byte chunks of the strided side touched by n rows of bl bytes at
    stride st from byte `first` (exact on whole periods, scaled)"""
    import numpy as np

    p = 128 // math.gcd(st, 128)
    m = min(n, max(p, -(-65536 // st)))
    m = min(n, -(-m // p) * p)
    lo = first - first % 128
    span = (m - 1) * st + bl + (first - lo)
    cov = np.zeros(-(-span // 128) * 128, dtype=np.uint8)
    starts = first - lo + np.arange(m, dtype=np.int64) * st
    for b in range(bl):
        cov[starts + b] = 1
    return float((cov.reshape(-1, size).sum(axis=1) > 0).sum()) * n / m


def model(bl, st, planes):
    import bench

    nplanes, rows, _, first = planes
    payload = nplanes * rows * bl
    touched, _, _, _ = bench._line_classes(bl, st, rows, first)
    tm = bench.touched_model(bl, st, *planes)
    return {"pack_read": nplanes * touched * 128.0, "pack_write": float(payload),
            "unpack_read": float(payload),
            "unpack_write_32": nplanes * chunks_touched(bl, st, rows, first, 32) * 32.0,
            "unpack_write_64": nplanes * chunks_touched(bl, st, rows, first, 64) * 64.0,
            "pack_equiv": tm["pack_bytes"], "unpack_equiv": tm["unpack_bytes"], "payload": payload}


def one(spec):
    """the profiled child: 1 + REPS packs, then 1 + REPS unpacks of one shape"""
    import torch

    import bench
    import tempi_amd

    dims, bl, st = (int(x) for x in spec.split(":"))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mpi = tempi_amd.get_mpi()
    mpi.Init()
    t, extent, shape, planes, payload = bench.sweep_shape(mpi, bl, st, dims, PACKED)
    t = mpi.Type_commit(t)
    src = torch.zeros(extent, dtype=torch.uint8, device=dev)
    pk = torch.zeros(payload, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    mpi.Pack(src.data_ptr(), 1, t, pk.data_ptr(), payload, 0)
    mpi.reset_counters()
    mpi.set_kernel_profiling(True)
    for _ in range(REPS):
        mpi.Pack(src.data_ptr(), 1, t, pk.data_ptr(), payload, 0)
    mpi.Unpack(pk.data_ptr(), payload, 0, src.data_ptr(), 1, t)
    for _ in range(REPS):
        mpi.Unpack(pk.data_ptr(), payload, 0, src.data_ptr(), 1, t)
    mpi.set_kernel_profiling(False)
    kt = mpi.kernel_times()
    print(json.dumps({"spec": spec, "shape": shape, "planes": list(planes), "payload": payload,
                      "pack_ms": kt["pack_ms"] / REPS, "unpack_ms": kt["unpack_ms"] / (REPS + 1)}), flush=True)
    mpi.Type_free(t)
    mpi.Finalize()


def family(name):
    import re

    m = re.search(r"::(\w+)[<(]", name)
    n = m.group(1) if m else ""
    if "ticket" in n:
        return None
    if "unpack" in n:
        return "unpack"
    if "pack" in n:
        return "pack"
    return None


def profile(spec, counter, outdir):
    d = tempfile.mkdtemp(prefix=f"sweep_{counter}_", dir=outdir)
    cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--pmc", counter, "--output-format", "csv", "-d", d,
           "-o", "pmc", "--", sys.executable, os.path.abspath(__file__), "--one", spec]
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{spec} {counter}: rc {r.returncode}\n{r.stdout[-2000:]}")
    info = json.loads(next(l for l in r.stdout.splitlines() if l.startswith("{")))
    vals = {"pack": [], "unpack": []}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            fam = family(row.get("Kernel_Name", ""))
            if fam and row.get("Counter_Name") == counter:
                vals[fam].append(float(row["Counter_Value"]) * 1024.0)  # KiB
    # the first launch of each is the warm-up
    return info, {k: (sum(v[1:]) / len(v[1:]) if len(v) > 1 else None) for k, v in vals.items()}


def timed(spec):
    """the same child without a profiler: its kernel times (counter
    collection serialises and slows the dispatches it counts)"""
    r = subprocess.run(["timeout", "-s", "KILL", "120", sys.executable, os.path.abspath(__file__), "--one", spec],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"{spec} timing run: rc {r.returncode}\n{r.stdout[-2000:]}")
    return json.loads(next(l for l in r.stdout.splitlines() if l.startswith("{")))


def run(specs, outdir, echo=True):
    """echo: one JSON line per spec on stdout (the command line); bench.py
    passes False, its stdout carries exactly one line"""
    import bench

    recs = []
    for spec in specs:
        _, fetch = profile(spec, "FETCH_SIZE", outdir)
        _, write = profile(spec, "WRITE_SIZE", outdir)
        info = timed(spec)
        dims, bl, st = (int(x) for x in spec.split(":"))
        m = model(bl, st, tuple(info["planes"]))
        got = {"pack_read": 2.0 * fetch["pack"], "pack_write": write["pack"],
               "unpack_read": 2.0 * fetch["unpack"], "unpack_write": write["unpack"]}
        rec = {"spec": spec, "shape": info["shape"], "block": bl, "stride": st, "payload": info["payload"],
               "pack_ms": round(info["pack_ms"], 4), "unpack_ms": round(info["unpack_ms"], 4),
               "counted": {k: int(v) for k, v in got.items()},
               "model": {k: int(v) for k, v in m.items()}}
        pm = m["pack_read"] + m["pack_write"]
        pc = got["pack_read"] + got["pack_write"]
        um = m["unpack_read"] + m["unpack_write_32"]
        uc = got["unpack_read"] + got["unpack_write"]
        rec["pack_model_over_counted"] = round(pm / pc, 3)
        rec["unpack_model32_over_counted"] = round(um / uc, 3)
        rec["unpack_model64_over_counted"] = round((m["unpack_read"] + m["unpack_write_64"]) / uc, 3)
        ach = bench.HBM_ACHIEVABLE_GBS * 1e9
        rec["pack_frac_touched"] = round(m["pack_equiv"] / ach / (info["pack_ms"] * 1e-3), 3)
        rec["unpack_frac_touched"] = round(m["unpack_equiv"] / ach / (info["unpack_ms"] * 1e-3), 3)
        rec["pack_frac_counted"] = round(pc / ach / (info["pack_ms"] * 1e-3), 3)
        rec["unpack_frac_counted"] = round(uc / ach / (info["unpack_ms"] * 1e-3), 3)
        if rec["pack_model_over_counted"] > 1.10:
            rec["pack_rescored_frac_touched"] = rec["pack_frac_counted"]
        if rec["unpack_model32_over_counted"] > 1.10:
            rec["unpack_rescored_frac_touched"] = rec["unpack_frac_counted"]
        recs.append(rec)
        if echo:
            print(json.dumps(rec), flush=True)
    return recs


if __name__ == "__main__":
    if sys.argv[1] == "--one":
        one(sys.argv[2])
    else:
        out = sys.argv[1]
        recs = run(sys.argv[2:], os.path.dirname(os.path.abspath(out)))
        json.dump(recs, open(out, "w"), indent=1)
