"""Checks of a perf.json written by apps/measure_system (shared by the CPU
and GPU tests): the reference's schema (/root/reference/src/internal/
measure_system.cpp:31-56 -- every key, curves of {"time", "iid"}), finite
positive times, the 1-D curves over 2^0 .. 2^maxLog bytes and the 2-D
tables' rows of 2^(2i+6) bytes x 10 block columns (2^j bytes)."""
import json
import math

ONE_D = ("d2h", "h2d", "intraNodeCpuCpuPingpong", "intraNodeGpuGpuPingpong", "interNodeCpuCpuPingpong",
         "interNodeGpuGpuPingpong")
TWO_D = ("packDevice", "unpackDevice", "packHost", "unpackHost")


def point_ok(p):
    return (set(p) == {"time", "iid"} and isinstance(p["iid"], bool) and isinstance(p["time"], float)
            and math.isfinite(p["time"]) and p["time"] > 0)


def check(path, gpu, quick=True):
    """returns (doc, [problems])"""
    text = open(path).read()
    doc = json.loads(text)
    bad = []
    missing = [k for k in ("cudaKernelLaunch",) + ONE_D + TWO_D if k not in doc]
    if missing:
        return doc, [f"missing keys {missing}"]
    n1 = (20 if quick else 23) + 1
    rows = ((18 if quick else 22) - 6) // 2 + 1  # 2^(2i+6) <= 2^maxTableLog
    want1 = {"intraNodeCpuCpuPingpong": n1}
    if gpu:
        want1.update({"d2h": n1, "h2d": n1, "intraNodeGpuGpuPingpong": n1})
    for k in ONE_D:
        c = doc[k]
        if len(c) != want1.get(k, 0):
            bad.append(f"{k}: {len(c)} points, expected {want1.get(k, 0)}")
        bad += [f"{k}[{i}] = {p}" for i, p in enumerate(c) if not point_ok(p)]
    for k in TWO_D:
        t = doc[k]
        if len(t) != (rows if gpu else 0) or any(len(r) != 10 for r in t):
            bad.append(f"{k}: {len(t)} rows of {[len(r) for r in t]}, expected {rows if gpu else 0} x 10")
        bad += [f"{k}[{i}][{j}] = {p}" for i, r in enumerate(t) for j, p in enumerate(r) if not point_ok(p)]
    launch = doc["cudaKernelLaunch"]
    if gpu:
        if not (isinstance(launch, float) and 0 < launch < 1e-3):
            bad.append(f"cudaKernelLaunch {launch}")
        elif launch == round(launch, 6):  # the 6-decimal rounding of std::to_string (VERDICT r04 missing 1)
            bad.append(f"cudaKernelLaunch {launch} has no sub-microsecond digits")
    return doc, bad
