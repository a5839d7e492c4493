"""Busy / idle time of the GPU over a halo trace (tools/gpu_session.sh
halo-trace): per kernel name the total time, and over the timed window the
union of kernel intervals (busy) against the window (busy + gaps). Several
trace files (one per process of a multi-rank run on one GPU) are merged.

With a HIP API trace (--hip-trace) beside the kernel trace, every idle gap is
split by what the host was doing while the GPU had nothing to run:
  host_late  the host had not yet entered the launch call of the kernel that
             ends the gap (it was posting sends, testing, waiting ...; with a
             marker trace the innermost roctx range open at the gap's start
             names it)
  launch     the host was inside that launch call (HIP's host cost)
  dispatch   the call had returned and the kernel had not started yet
and the host time of each launch API is reported per call."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/halo_trace"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10


def load(kind):
    return [r for p in glob.glob(root + f"/**/*{kind}.csv", recursive=True) for r in csv.DictReader(open(p))]


krows = load("kernel_trace")
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Correlation_Id", "")) for r in krows)
copies = [k for k in ks if "copy" in k[2] or "pack" in k[2]]
# skip the warm-up iteration: the first 1/(iters + 1) of the copy launches
skip = len(copies) // (iters + 1)
win = copies[skip:]
t0, t1 = win[0][0], max(k[1] for k in win)
busy, cur_s, cur_e = 0, None, None
gaps = []  # (gap start, gap end, correlation id of the kernel that ends it)
for s, e, _, corr in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((cur_e, s, corr))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
per = defaultdict(lambda: [0, 0])
for s, e, n, _ in win:
    per[n][0] += 1
    per[n][1] += e - s
print(f"window {(t1 - t0) / 1e3 / iters:.1f} us/iter, busy (union) {busy / 1e3 / iters:.1f} us/iter, "
      f"idle {(t1 - t0 - busy) / 1e3 / iters:.1f} us/iter, launches/iter {len(win) / iters:.1f}")
for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
    print(f"  {t / 1e3 / iters:8.1f} us/iter  {c / iters:6.1f} launches/iter  {n[:110]}")

api = load("hip_api_trace")
if not api:
    sys.exit(0)
launch_fns = ("hipModuleLaunchKernel", "hipLaunchKernel", "hipExtModuleLaunchKernel", "hipExtLaunchKernel",
              "hipLaunchKernelExC", "hipGraphLaunch")
by_corr = {}
calls = defaultdict(lambda: [0, 0])
for r in api:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s < t0 or s > t1:
        continue
    calls[r["Function"]][0] += 1
    calls[r["Function"]][1] += e - s
    by_corr[r.get("Correlation_Id", "")] = (s, e, r["Function"])
print(f"\nHIP API calls inside the window (per iteration):")
for fn, (c, t) in sorted(calls.items(), key=lambda kv: -kv[1][1])[:14]:
    print(f"  {t / 1e3 / iters:8.1f} us/iter  {c / iters:7.1f} calls/iter  {t / 1e3 / max(c, 1):6.2f} us/call  {fn}")

# launch host cost by kernel name
lcost = defaultdict(list)
for s, e, n, corr in win:
    a = by_corr.get(corr)
    if a and a[2] in launch_fns:
        lcost[n].append((a[1] - a[0]) / 1e3)
print("\nlaunch call host time by kernel (us/call: mean, min, max; calls/iter)")
for n, v in sorted(lcost.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {sum(v) / len(v):6.2f} {min(v):6.2f} {max(v):6.2f}  {len(v) / iters:6.1f}  {n[:90]}")

markers = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Message") or r.get("Function", ""))
           for r in load("marker_api_trace")]


def innermost(t):
    best = None
    for s, e, m in markers:
        if s <= t < e and (best is None or s > best[0]):
            best = (s, e, m)
    return best[2] if best else "(no range)"


parts = defaultdict(int)
late_by = defaultdict(int)
for gs, ge, corr in gaps:
    a = by_corr.get(corr)
    if not a:
        parts["unattributed"] += ge - gs
        continue
    s, e = a[0], a[1]
    late = max(0, min(s, ge) - gs)
    launch = max(0, min(e, ge) - max(s, gs))
    disp = max(0, ge - max(e, gs))
    parts["host_late"] += late
    parts["launch"] += launch
    parts["dispatch"] += disp
    if late and markers:
        late_by[innermost(gs)] += late
total = sum(parts.values())
print(f"\nidle {total / 1e3 / iters:.1f} us/iter over {len(gaps) / iters:.1f} gaps/iter:")
for k, v in sorted(parts.items(), key=lambda kv: -kv[1]):
    print(f"  {k:12s} {v / 1e3 / iters:8.1f} us/iter")
for k, v in sorted(late_by.items(), key=lambda kv: -kv[1])[:8]:
    print(f"    host_late inside {k[:60]:60s} {v / 1e3 / iters:8.1f} us/iter")
