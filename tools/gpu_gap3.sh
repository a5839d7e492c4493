#!/bin/bash
# which whole-sector gapped scatters gain from the
# XCD-range tile order. The pattern alone (tools/calib sect_copy, dealt vs
# XCD-range, 20 (block, stride) pairs) and the packer's kernels on the same
# shapes at 1 GiB, dealt ("cur") vs XCD-range ("gap", TEMPI_XCD_GAPPED=1),
# two alternations. Output: gpurun_out/sect3.jsonl, gap3_ab.jsonl.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
timeout -k 10 300 tools/calib 10 --only sc_ > $O/sect3.jsonl || exit 3
echo "sect cases: $(wc -l < $O/sect3.jsonl)"
SHAPES="64:16777216:512 64:8388608:4096 128:8388608:256 128:8388608:512 256:4194304:512 256:4194304:1024 256:4194304:4096 512:2097152:1024 512:2097152:2048 512:2097152:4096 1024:1048576:2048 1024:1048576:4096 1024:1048576:8192 2048:524288:4096 2048:524288:8192 2048:724:2977792:724:4096 1024:1024:2359296:1024:2048 4096:131072:8192 4096:131072:16384"
bash tools/kab.sh gap3_ab.jsonl 2 10 $SHAPES || exit 4
