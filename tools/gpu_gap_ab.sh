#!/bin/bash
# the gapped whole-sector unpacks (64 : 512, 1 024 : 4 096,
# 3D 2 048 : 4 096) against their touched bound, with the headline and two
# whole-line shapes as controls. Kernel A/B of the scatter's store policy and
# tile order (tools/build_ab.sh variants), then the memory-side write
# requests of the current kernels (one rocprofv3 --pmc pass per group).
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
SHAPES="64:16777216:512 1024:1048576:4096 2048:724:2977792:724:4096 2048:524288:4096 512:2097152:1024 256:4194304:512 4096:131072:8192"
bash tools/kab.sh gap_ab.jsonl 2 20 $SHAPES || exit 4
for g in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "WRITE_SIZE" "FETCH_SIZE"; do
  n=$(echo $g | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d $O/gap_pmc_$n -o run -- \
    tools/_variants/kbench tools/_variants/libtempi_hip_cur.so 3 $SHAPES > $O/gap_pmc_$n.log 2>&1 || exit 5
  echo "pmc $n ok"
done
