#!/bin/bash
# the sector-scatter pattern alone (tools/calib
# sect_copy: no packer index math; rows of B bytes every S bytes; 1 or 4
# chunks per lane; dealt or XCD-range order) next to the packer's own kernels
# on the same shapes (tools/gpu_gap_ab.sh: variants from tools/build_ab.sh, and
# the write-request counters). Output under gpurun_out/.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 tools/calib 10 --only sc_ > $O/sect.jsonl || exit 3
timeout -k 10 120 tools/calib 10 --only ga_ >> $O/sect.jsonl || exit 3
echo "sect cases: $(wc -l < $O/sect.jsonl)"
bash tools/gpu_gap_ab.sh
