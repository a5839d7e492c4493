#!/bin/bash
# 2D vs 3D twins of the config-2 sweep's narrow unpacks, plus 3D objects of
# two planes (the 3D decode with almost no plane crossings): kernel GB/s per
# variant in tools/_variants (tools/build_ab.sh), ROUNDS alternations.
# usage: tools/gpu_3d_unpack.sh OUT ROUNDS
set -o pipefail
cd "$(dirname "$0")/.."
KBENCH_NO_COPY=1 tools/kab.sh "$1" "$2" 10 \
  1:1073741824:2 1:32768:65542:32768:2 1:2:1073741830:536870912:2 \
  4:268435456:8 4:16384:131096:16384:8 4:2:1073741848:134217728:8 \
  16:67108864:32 16:8192:262240:8192:32 \
  64:16777216:128 64:4096:524672:4096:128 64:2:1073742208:8388608:128
