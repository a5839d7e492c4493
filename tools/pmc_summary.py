"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes per kernel
(gfx950: FETCH_SIZE counts half of a wide streaming read -> x2; values in KiB).
usage: python tools/pmc_summary.py DIR_FETCH DIR_WRITE [kernel-substring ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") == counter:
                    vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def main():
    fd, wd = sys.argv[1], sys.argv[2]
    subs = sys.argv[3:] or ["pack_kernel", "copy"]
    print("rocprofv3 --pmc <C> (one counter per run); FETCH_SIZE/WRITE_SIZE in KiB; gfx950: FETCH_SIZE x2")
    for counter, d, mult in (("FETCH_SIZE", fd, 2.0), ("WRITE_SIZE", wd, 1.0)):
        for k, v in sorted(load(d, counter).items()):
            if not any(s in k for s in subs):
                continue
            avg = sum(v) / len(v)
            print(f"{counter:10s}  {k[:70]:70s} launches={len(v)} avg={avg:.1f} KiB -> "
                  f"{avg * 1024 * mult / 1e9:.4f} GB per launch (corrected)")


if __name__ == "__main__":
    main()
