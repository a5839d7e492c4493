"""Busy / idle time of the GPU over a halo kernel trace (tools/gpu_halo_trace.sh):
per kernel name the total time, and over the timed window the union of
kernel intervals (busy) against the window (busy + gaps). Several trace
files (one per process of a multi-rank run on one GPU) are merged."""
import csv
import glob
import sys
from collections import defaultdict

paths = glob.glob((sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/halo_trace") + "/**/*kernel_trace.csv",
                  recursive=True)
rows = [r for p in paths for r in csv.DictReader(open(p))]
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
copies = [k for k in ks if "copy" in k[2] or "pack" in k[2]]
# skip the warm-up iteration: the first 1/11 of the copy launches
skip = len(copies) // 11
win = copies[skip:]
t0, t1 = win[0][0], max(e for _, e, _ in win)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
per = defaultdict(lambda: [0, 0])
for s, e, n in win:
    per[n][0] += 1
    per[n][1] += e - s
it = 10
print(f"window {(t1 - t0) / 1e3 / it:.1f} us/iter, busy (union) {busy / 1e3 / it:.1f} us/iter, "
      f"idle {(t1 - t0 - busy) / 1e3 / it:.1f} us/iter, launches/iter {len(win) / it:.1f}")
for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
    print(f"  {t / 1e3 / it:8.1f} us/iter  {c / it:6.1f} launches/iter  {n[:110]}")
