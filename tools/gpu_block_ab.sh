#!/bin/bash
# Workgroup-size A/B on one box: TEMPI_BLOCK 128/512/1024 variants (built on the
# CPU with that -D on tools/build_variants.sh's hipcc line) against the shipped
# 256, over the kbench shapes and the halo regions, interleaved twice.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/block_ab.jsonl
SHAPES="512:2097152:1024 4096:262144:4160 64:16777216:128 8:67108864:16 24:512:2386944:512:4608 1:268435456:2 1:134217728:8"
for rep in 1 2; do
  for v in cur bs128 bs512 bs1024; do
    timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/block_ab.jsonl || exit 5
    timeout -k 10 120 tools/_variants/hbench tools/_variants/libtempi_hip_$v.so 20 >> $O/block_ab.jsonl || exit 6
  done
done
