#!/bin/bash
# 1-rank halo in MPI_Neighbor_alltoallw mode: stream lanes / first flush A/B
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/nbr.txt
for rep in 1 2; do
  for cfg in "TEMPI_STREAMS=3" "TEMPI_STREAMS=1" "TEMPI_FIRST_FLUSH=32" "TEMPI_STREAMS=1 TEMPI_FIRST_FLUSH=32"; do
    env $cfg TEMPI_PRINT_COUNTERS=1 timeout -k 10 200 tempi_amd/lib/halo_exchange 10 512 --neighbor > $O/nbr_one.txt 2>&1 || exit 3
    echo "$cfg $(grep -o '"us_per_iter": [0-9.]*' $O/nbr_one.txt) $(grep -o 'batches=[0-9]* items=[0-9]*' $O/nbr_one.txt)" | tee -a $O/nbr.txt
  done
done
