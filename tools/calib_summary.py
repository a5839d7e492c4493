"""Summarise tools/calib.sh: per calibration case, time-derived GB/s and the
memory-side counters per KNOWN byte (the case's algorithmic bytes and the
128-B lines it touches).
usage: python tools/calib_summary.py gpurun_out/calib > profiles/r02/counter_calibration.txt"""
import csv
import json
import os
import sys

d = sys.argv[1]
cases = [json.loads(l) for l in open(os.path.join(d, "time.jsonl"))]


def per_dispatch(sub):
    """counter -> list of values in dispatch order (calib kernels only)"""
    rows = {}
    path = os.path.join(d, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        if r["Kernel_Name"].startswith("__amd"):
            continue
        rows.setdefault(r["Counter_Name"], {})[int(r["Dispatch_Id"])] = float(r["Counter_Value"])
    return {c: [v[k] for k in sorted(v)] for c, v in rows.items()}


counters = {}
for sub in ("fetch", "write", "rdreq", "wrreq"):
    counters.update(per_dispatch(sub))
# tools/calib 1: each case is one warm-up dispatch and one timed dispatch
print("MI355X memory-counter calibration (tools/calib.hip, tools/calib.sh): 4 GiB buffer (16x the")
print("Infinity Cache), known byte counts. Columns: time-derived algorithmic and touched-line rates;")
print("counters of the case's second dispatch divided by its algorithmic bytes (alg) and by its")
print("128-B lines x 128 (line). FETCH_SIZE / WRITE_SIZE in KiB as rocprofv3 reports them; RDREQ /")
print("WRREQ are TCC_EA0 request counts, scaled here by 64 B (RDREQ, WRREQ) or 32 B (RDREQ_32B) /")
print("64 B (WRREQ_64B) per request.\n")
hdr = f"{'case':22s} {'ms':>7s} {'algGB/s':>8s} {'lineGB/s':>8s}"
names = [("FETCH_SIZE", 1024), ("WRITE_SIZE", 1024), ("TCC_EA0_RDREQ_sum", 64), ("TCC_EA0_RDREQ_32B_sum", 32),
         ("TCC_EA0_WRREQ_sum", 64), ("TCC_EA0_WRREQ_64B_sum", 64)]
for n, _ in names:
    short = n.replace("TCC_EA0_", "").replace("_sum", "")
    hdr += f" {short + '/alg':>14s} {short + '/line':>14s}"
print(hdr)
for i, c in enumerate(cases):
    line = f"{c['case']:22s} {c['ms']:7.3f} {c['alg_GBps']:8.1f} {c['line_GBps']:8.1f}"
    for n, scale in names:
        v = counters.get(n)
        if not v or 2 * i + 1 >= len(v):
            line += f" {'-':>14s} {'-':>14s}"
            continue
        b = v[2 * i + 1] * scale
        line += f" {b / c['alg_bytes']:14.3f} {b / c['line_bytes']:14.3f}"
    print(line)
