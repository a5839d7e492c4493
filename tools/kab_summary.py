"""Summarise a tools/kab.sh JSONL: per shape, each variant's pack / unpack
algorithmic GB/s over the rounds (round by round, best last).
usage: python tools/kab_summary.py gpurun_out/FILE.jsonl"""
import collections
import json
import sys

d = collections.defaultdict(list)
shapes, variants = [], []
for line in open(sys.argv[1]):
    r = json.loads(line)
    d[(r["shape"], r["variant"])].append((r["pack_gbs"], r["unpack_gbs"]))
    if r["shape"] not in shapes:
        shapes.append(r["shape"])
    if r["variant"] not in variants:
        variants.append(r["variant"])
for s in shapes:
    cells = []
    for v in variants:
        xs = d[(s, v)]
        cells.append(f"{v} pack {'/'.join(f'{x[0]:.0f}' for x in xs):11s} unpack {'/'.join(f'{x[1]:.0f}' for x in xs):11s}")
    print(f"{s:26s} " + " | ".join(cells))
