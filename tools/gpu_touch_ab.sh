#!/bin/bash
# Unpack A/B on one box: TEMPI_UNPACK_TOUCH (load the destination line of
# sub-sector rows before the scatter writes it) against the shipped kernel.
# Variants (built on the CPU first): cur = tools/build_variants.sh; touch = the same
# hipcc line with -DTEMPI_UNPACK_TOUCH=1 on the build this A/B measured
# (reverted).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/touch_ab.jsonl
SHAPES="24:512:2386944:512:4608 8:67108864:16 1:268435456:2 3:89478485:7 1:134217728:8 4:67108864:16 64:16777216:128 512:2097152:1024"
for rep in 1 2; do
  for v in cur touch; do
    timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/touch_ab.jsonl || exit 5
    HBENCH_ONLY=x_faces timeout -k 10 120 tools/_variants/hbench tools/_variants/libtempi_hip_$v.so 20 >> $O/touch_ab.jsonl || exit 6
  done
done
