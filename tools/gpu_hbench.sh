#!/bin/bash
# halo-region kernel bench over the libtempi_hip variants + host-time counters
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/hbench.jsonl
for v in $(ls tools/_variants/ | sed -n 's/^libtempi_hip_\(.*\)\.so$/\1/p'); do
  timeout -k 10 120 tools/_variants/hbench tools/_variants/libtempi_hip_$v.so 20 >> $O/hbench.jsonl || exit 5
done
cat $O/hbench.jsonl | cut -c 1-400
TEMPI_PRINT_COUNTERS=1 timeout -k 10 120 tempi_amd/lib/halo_exchange 10 512 > $O/halo_counters.txt 2>&1 || exit 6
cat $O/halo_counters.txt
