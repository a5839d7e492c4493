#!/bin/bash
# XCD map A/B, second pass: long gapped rows (where the map's row limit
# TEMPI_XCD_MAX_BLOCK falls), a few narrow shapes, then the 512^3 halo at 1
# and 2 ranks with the map off (TEMPI_NO_XCD_MAP=1) and on.
# usage: tools/gpu_xcd_ab2.sh OUT ROUNDS   (after tools/build_ab.sh nomap:-DTEMPI_XCD_MAP=0 big:-DTEMPI_XCD_MAX_BLOCK=65536)
set -o pipefail
cd "$(dirname "$0")/.."
KBENCH_NO_COPY=1 tools/kab.sh "$1" "$2" 10 \
  512:2097152:1024 512:2097152:528 1024:1048576:1040 4096:262144:4112 \
  256:4194304:272 1:32768:65542:32768:2 4:268435456:8 16:67108864:32 && \
tools/gpu_halo_ab.sh TEMPI_NO_XCD_MAP=1 "1 2"
