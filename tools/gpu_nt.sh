#!/bin/bash
# A/B of the strided-side cache policy on one box: cur (nontemporal strided
# side for 16-byte words) vs nt1 (plain strided side), over aligned and
# misaligned-stride (bl+16) shapes. Build nt1 first:
#   hipcc ... -DTEMPI_NT=1 -o tools/_variants/libtempi_hip_nt1.so (see build_variants.sh)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
SHAPES="512:2097152:1024 128:8388608:256 128:8388608:144 256:4194304:272 512:2097152:528 64:16777216:80 32:33554432:48 1024:1048576:1040 2048:524288:2064 4096:262144:4112"
rm -f $O/nt.jsonl
for rep in 1 2; do
  for v in cur nt1; do
    timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/nt.jsonl || exit 5
  done
done
