#!/bin/bash
# Kernel A/B on one GPU box: every tools/_variants/libtempi_hip_*.so, in
# alternation, ROUNDS times, on the same shapes (tools/kbench.cpp SHAPE
# syntax: block:count:stride[:count:stride], outermost dimension first).
# One JSON line per (variant, shape) into gpurun_out/$OUT.
# usage: tools/kab.sh OUT ROUNDS REPS SHAPE...
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/$1; ROUNDS=$2; REPS=$3; shift 3
V=${KAB_DIR:-tools/_variants}  # (tools/bin/v travels to the box: tools/_variants is gpurun-ignored)
rm -f $OUT
for r in $(seq $ROUNDS); do
  for lib in $V/libtempi_hip_*.so; do
    v=$(basename $lib .so); v=${v#libtempi_hip_}
    timeout -k 10 300 $V/kbench $lib $REPS "$@" | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $OUT || exit 5
  done
done
echo "wrote $(wc -l < $OUT) lines to $OUT"
