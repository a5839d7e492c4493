#!/usr/bin/env python3
"""Regenerate tests/golden/mpich_golden.json from tests/golden/cases.txt.

For every case, runs oracle/_build/gen_golden (linked against the host MPI,
MPICH 3.3.2 in /opt/conda) and stores what the LIBRARY's MPI_Pack/MPI_Unpack
produced: size / lb / extent / pack size / final position, and the packed
bytes (hex when <= 64 KiB, else SHA-256 plus the first and last 64 bytes) and
the SHA-256 of MPI_Unpack of those bytes into a zeroed buffer.

Run in the build container (needs /opt/conda MPICH):  python tools/make_golden.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
GEN = os.path.join(ROOT, "oracle", "_build", "gen_golden")
CASES = os.path.join(ROOT, "tests", "golden", "cases.txt")
OUT = os.path.join(ROOT, "tests", "golden", "mpich_golden.json")
FULL_LIMIT = 64 * 1024


def read_cases(path=CASES):
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            name, count, recipe = [p.strip() for p in line.split("|")]
            out.append((name, int(count), recipe))
    return out


def main():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "golden"])
    records = []
    with tempfile.TemporaryDirectory() as td:
        pb, ub = os.path.join(td, "p.bin"), os.path.join(td, "u.bin")
        for name, count, recipe in read_cases():
            meta = json.loads(subprocess.check_output([GEN, recipe, str(count), pb, ub]))
            packed = open(pb, "rb").read()
            unpacked = open(ub, "rb").read()
            rec = {"name": name, "count": count, "recipe": recipe}
            rec.update(meta)
            rec["packed_sha256"] = hashlib.sha256(packed).hexdigest()
            rec["unpacked_sha256"] = hashlib.sha256(unpacked).hexdigest()
            if len(packed) <= FULL_LIMIT:
                rec["packed_hex"] = packed.hex()
            else:
                rec["packed_head_hex"] = packed[:64].hex()
                rec["packed_tail_hex"] = packed[-64:].hex()
            records.append(rec)
    doc = {
        "generator": "oracle/gen_golden.c via tools/make_golden.py",
        "library": records[0]["library"] if records else "",
        "input_convention": "buffer byte i (from allocation start) = i & 0xFF; MPI buffer = alloc + origin",
        "cases": records,
    }
    with open(OUT, "w") as f:
        json.dump(doc, f, indent=1)
        f.write("\n")
    print(f"wrote {len(records)} golden records to {OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
