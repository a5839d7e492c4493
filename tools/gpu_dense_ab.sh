#!/bin/bash
# The dense-window gather (pack_kernels.hip pack_dense_kernel) at wider
# stride : block ratios (TEMPI_DENSE_RATIO 4 = tree, 9, 16, 24) on the narrow
# misaligned rows the config-2 sweep reports worst (2 B rows at stride 18 in
# 2D and 3D with a 3-row pad, 3 B at 19, 1 B at 17) and controls (1 B : 2,
# 4-byte words, 8-byte rows). Two alternations, gpurun_out/dense_ab.jsonl.
# Build the variants first, on the CPU side:
#   tools/build_ab.sh "r9:-DTEMPI_DENSE_RATIO=9" "r16:-DTEMPI_DENSE_RATIO=16" "r24:-DTEMPI_DENSE_RATIO=24"
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SHAPES="2:536870912:18 2:23170:417114:23170:18 3:357913941:19 1:1073741824:17 1:32768:65542:32768:2 4:268435456:20 6:178956970:22 8:134217728:24"
bash tools/kab.sh dense_ab.jsonl 2 10 $SHAPES || exit 4
