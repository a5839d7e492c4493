#!/bin/bash
# TEMPI_BLOCK=64 (one wave; built on the CPU with that -D on
# tools/build_variants.sh's hipcc line) against the shipped 128, on one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/block64_ab.jsonl
SHAPES="512:2097152:1024 4096:262144:4160 64:16777216:128 8:67108864:16 24:512:2386944:512:4608 1:268435456:2 1:134217728:8"
for rep in 1 2; do
  for v in cur bs64; do
    timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/block64_ab.jsonl || exit 5
  done
done
