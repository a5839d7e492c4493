#!/bin/bash
# A/B of the XCD-aware workgroup -> tile map for partial-sector scatters
# (kXcdRange, pack_kernels.hip) over the headline, the config-2 sweep's 2D/3D
# twins, the gapped shapes and the halo's 24-B rows (those also time the
# strided -> strided copy); then the 512^3 halo at 1 and 2 ranks with the map
# off (TEMPI_NO_XCD_MAP=1) and on.
# usage: tools/gpu_xcd_ab.sh OUT ROUNDS   (after tools/build_ab.sh nomap:-DTEMPI_XCD_MAP=0)
set -o pipefail
cd "$(dirname "$0")/.."
KBENCH_NO_COPY=1 tools/kab.sh "$1.a" "$2" 10 \
  512:2097152:1024 \
  1:1073741824:2 1:32768:65542:32768:2 \
  4:268435456:8 4:16384:131096:16384:8 \
  16:67108864:32 16:8192:262240:8192:32 \
  64:16777216:128 64:4096:524672:4096:128 \
  2:536870912:18 2:23170:417114:23170:18 \
  128:8388608:144 256:4194304:272 64:16777216:512 && \
tools/kab.sh "$1.b" "$2" 20 24:512:2386944:512:4608 8:134217728:24 8:11585:278112:11585:24 && \
cat gpurun_out/$1.a gpurun_out/$1.b > gpurun_out/$1 && rm gpurun_out/$1.a gpurun_out/$1.b && \
tools/gpu_halo_ab.sh TEMPI_NO_XCD_MAP=1 "1 2"
