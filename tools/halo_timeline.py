"""Where the 1-rank halo's GPU idle time goes, per substep.

Inputs: the host timeline TEMPI writes under TEMPI_TIMELINE=PREFIX
(PREFIX.r0.csv: CLOCK_BOOTTIME ns of the MPI entry points' and the batched
launches' begin / end, and of each batch observed complete) and a rocprofv3
--kernel-trace of the same run (the same clock; no HIP API tracing, so the
host runs nearly as fast as untraced).

A substep runs from its first MPI_Isend to its last MPI_Wait (the barrier
between substeps is outside, as in halo_exchange's own timing). Each GPU-idle
interval inside it is split by what the host was doing:
  send burst    posting the substep's MPI_Isends (no receive exists yet, so
                nothing can run: the application's own order)
  recv posting  posting MPI_Irecvs, no launch in progress
  launch        inside a batched launch (tempi::launch ...)
  dispatch      the launch returned, its kernel has not started
  tail          after the substep's last kernel: completion observed,
                requests completed, MPI_Wait returns
  wait          in MPI_Wait with the GPU idle before that

Without a kernel trace (KERNEL_TRACE_DIR "-"), the GPU is taken as idle while
no batch is in flight by the host's own account: from a batched launch's end
to that batch observed complete (its ticket or event). This needs no
profiler at all -- rocprofv3, even with --kernel-trace alone, triples the
host's per-call cost here (MPI_Isend phase 315 against 89 us per iteration,
profiles/r05/halo_timeline_s3.txt) -- so it is the attribution of an
untraced run; it counts the dispatch latency as busy and the observation
latency as busy too.
usage: halo_timeline.py TIMELINE.csv KERNEL_TRACE_DIR|- [skip_substeps]"""
import csv
import glob
import sys
from collections import defaultdict

tl_path, kdir = sys.argv[1], sys.argv[2]
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 3

marks = [(int(r["ns"]), int(r["phase"]), r["name"]) for r in csv.DictReader(open(tl_path))]
marks.sort()
kern = [] if kdir == "-" else sorted(
    (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    for p in glob.glob(kdir + "/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(p)))

# substeps: [first MPI_Isend begin, last MPI_Wait end] between barriers
subs = []
cur = None
for ns, ph, name in marks:
    if name == "MPI_Barrier" and ph == 0:
        if cur and cur.get("end"):
            subs.append(cur)
        cur = None
    elif name == "MPI_Isend" and ph == 0 and cur is None:
        cur = {"start": ns, "irecv": None, "irecv_end": None, "end": None, "flushes": [], "done": []}
    elif cur is not None:
        if name == "MPI_Irecv" and ph == 0 and cur["irecv"] is None:
            cur["irecv"] = ns
        if name == "MPI_Irecv" and ph == 1:
            cur["irecv_end"] = ns
        if name == "MPI_Wait" and ph == 1:
            cur["end"] = ns
        if name.startswith("tempi::launch") and ph == 0:
            cur["flushes"].append([ns, None])
        if name.startswith("tempi::launch") and ph == 1 and cur["flushes"]:
            cur["flushes"][-1][1] = ns
        if name.startswith("batch done"):
            cur["done"].append(ns)
if cur and cur.get("end"):
    subs.append(cur)
subs = subs[skip:]


def busy_from_host(sb, a, b):
    """[launch end, observed complete] of the substep's batches, merged"""
    ev = sorted([(f[1], +1) for f in sb["flushes"] if f[1] is not None] + [(t, -1) for t in sb["done"]])
    out, depth, start = [], 0, None
    for t, d in ev:
        if d > 0 and depth == 0:
            start = t
        depth = max(0, depth + d)
        if depth == 0 and start is not None:
            out.append([max(start, a), min(t, b)])
            start = None
    if start is not None:
        out.append([max(start, a), b])
    return [iv for iv in out if iv[1] > iv[0]]


def busy_intervals(sb, a, b):
    if not kern:
        return busy_from_host(sb, a, b)
    out = []
    for s, e in kern:
        if e <= a or s >= b:
            continue
        s, e = max(s, a), min(e, b)
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


tot = defaultdict(float)
walls, busys = [], []
for sb in subs:
    a, b = sb["start"], sb["end"]
    busy = busy_intervals(sb, a, b)
    walls.append(b - a)
    busys.append(sum(e - s for s, e in busy))
    # idle intervals
    idle, t = [], a
    for s, e in busy:
        if s > t:
            idle.append((t, s))
        t = max(t, e)
    if t < b:
        idle.append((t, b))
    fl = [f for f in sb["flushes"] if f[1] is not None]
    last_kernel_end = busy[-1][1] if busy else a

    def host_state(x):
        for fb, fe in fl:
            if fb <= x < fe:
                return "launch"
        if x >= last_kernel_end and x >= (sb["irecv_end"] or b):
            return "tail"
        if sb["irecv"] is None or x < sb["irecv"]:
            return "send burst"
        done = [f for f in fl if f[1] <= x]
        if done:
            fe = max(f[1] for f in done)
            if not any(fe <= ks <= x for ks, _ in busy):  # launched; its kernel has not started
                return "dispatch"
        if x < (sb["irecv_end"] or b):
            return "recv posting"
        return "wait"

    # integrate by 200 ns steps (idle intervals are tens of us)
    for s, e in idle:
        x = s
        while x < e:
            st = e if e - x < 200 else x + 200
            tot[host_state(x)] += st - x
            x = st

n = len(subs)
if not n:
    sys.exit("no substeps found")
wall = sum(walls) / n / 1e3
busy = sum(busys) / n / 1e3
print(("kernel trace" if kern else "host account of batches in flight (no profiler)") + ":")
print(f"{n} substeps: wall {wall:.1f} us, GPU busy (union) {busy:.1f} us, idle {wall - busy:.1f} us per substep "
      f"(x3 = {3 * wall:.1f} / {3 * busy:.1f} / {3 * (wall - busy):.1f} us per iteration)")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"  {k:14s} {v / n / 1e3:7.1f} us per substep  {3 * v / n / 1e3:7.1f} us per iteration")
