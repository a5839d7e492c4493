#!/bin/bash
# The partial-page XCD-range rule (pack_kernels.hip partial_pages): the tree
# ("cur": scatters), the rule off ("old"), and the rule for gathers too
# ("packxr"), on the shapes it covers and on controls; two alternations.
# gpurun_out/gap4_ab.jsonl.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
SHAPES="64:16777216:512 64:8388608:4096 256:4194304:4096 512:2097152:4096 1024:1048576:4096 1024:1048576:8192 2048:524288:4096 2048:524288:8192 2048:724:2977792:724:4096 512:2097152:1024 4096:131072:8192 128:8388608:256 1024:1048576:2048"
bash tools/kab.sh gap4_ab.jsonl 2 10 $SHAPES || exit 4
