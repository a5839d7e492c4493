"""Summarise tools/gpu_kbench_pmc.sh: per shape and kernel kind, HBM bytes
touched per launch (FETCH_SIZE x2 on gfx950, + WRITE_SIZE; both in KiB) against
the algorithmic 2 x payload.  usage: python tools/kbench_pmc_summary.py DIR"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kind(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                kind = "unpack" if "unpack" in name else "pack" if "pack" in name else None
                if kind:
                    vals[kind].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sorted(v)[len(v) // 2] for k, v in vals.items()}


def main(root):
    i = 1
    print("shape | kind | payload B | read B | write B | touched / algorithmic | kernel GB/s (alg)")
    while os.path.exists(os.path.join(root, f"k{i}.json")):
        rec = None
        with open(os.path.join(root, f"k{i}.json")) as fh:
            for line in fh:
                if line.startswith("{"):
                    rec = json.loads(line)
        f = per_kind(os.path.join(root, f"p{i}_FETCH_SIZE"), "FETCH_SIZE")
        w = per_kind(os.path.join(root, f"p{i}_WRITE_SIZE"), "WRITE_SIZE")
        if rec:
            p = rec["payload"]
            for kind in ("pack", "unpack"):
                if kind in f and kind in w:
                    rd, wr = 2.0 * f[kind], w[kind]
                    print(f"{rec['shape']} | {kind} | {p} | {rd:.0f} | {wr:.0f} | {(rd + wr) / (2.0 * p):.2f} | "
                          f"{rec[kind + '_gbs']}")
        i += 1


if __name__ == "__main__":
    main(sys.argv[1])
