#!/bin/bash
# 1-rank halo: size of the first scatter batch of a burst (TEMPI_FIRST_FLUSH)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/first.txt
for rep in 1 2 3; do
  for f in 32 4 8 16; do
    TEMPI_FIRST_FLUSH=$f timeout -k 10 200 tempi_amd/lib/halo_exchange 10 512 > $O/first_one.txt 2>&1 || exit 3
    echo "first=$f $(grep -o '"us_per_iter": [0-9.]*' $O/first_one.txt) $(grep -o 'rank0_us_per_iter.*' $O/first_one.txt)" | tee -a $O/first.txt
  done
done
