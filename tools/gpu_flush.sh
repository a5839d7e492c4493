#!/bin/bash
# 1-rank halo: early-flush sizes with the stream lanes, counters printed
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/flush.txt
for rep in 1 2; do
  for f in 8 16 32 64; do
    TEMPI_PRINT_COUNTERS=1 TEMPI_EARLY_FLUSH=$f timeout -k 10 200 tempi_amd/lib/halo_exchange 10 512 > $O/flush_one.txt 2>&1 || exit 3
    echo "flush=$f $(grep -o '"us_per_iter": [0-9.]*' $O/flush_one.txt) $(grep -o 'rank0_us_per_iter.*' $O/flush_one.txt) $(grep -o 'batches=.*' $O/flush_one.txt)" | tee -a $O/flush.txt
  done
done
