"""Per-kernel averages of every counter in rocprofv3 --pmc output directories
(raw values as rocprofv3 reports them: FETCH_SIZE / WRITE_SIZE in KiB, the
TCC_EA0_* request counts as counts; no gfx950 correction applied here).
usage: python tools/pmc_kernels.py DIR [DIR ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    vals = defaultdict(list)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    vals[(row["Counter_Name"], row["Kernel_Name"])].append(float(row["Counter_Value"]))
    for (c, k), v in sorted(vals.items()):
        print(f"{c:22s} {k[:90]:90s} launches={len(v):4d} avg={sum(v) / len(v):.1f}")


if __name__ == "__main__":
    main()
