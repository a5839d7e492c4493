#!/bin/bash
# 1-rank halo A/B: tools/_variants/old vs the tree's build, alternating,
# with the rank-0 phase times
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/ab1.txt
for rep in 1 2 3 4; do
  for v in old new; do
    LP=; [ $v = old ] && LP=$PWD/tools/_variants/old
    LD_LIBRARY_PATH=$LP timeout -k 10 200 tempi_amd/lib/halo_exchange 10 512 > $O/ab1_one.txt 2>&1 || exit 3
    echo "$v $(grep -o '"us_per_iter": [0-9.]*' $O/ab1_one.txt) $(grep -o 'rank0_us_per_iter.*' $O/ab1_one.txt)" | tee -a $O/ab1.txt
  done
done
