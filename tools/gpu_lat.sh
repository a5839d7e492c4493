#!/bin/bash
# small-message latency: kernel launch->completion floor, then the 1 KiB
# ping-pong per method with TEMPI's host-time counters
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
timeout -k 10 60 tools/_variants/latbench > $O/lat.jsonl || exit 3
for m in ${LAT_METHODS:-TEMPI_DATATYPE_IPC TEMPI_DATATYPE_ONESHOT}; do
  env $m=1 TEMPI_PRINT_COUNTERS=1 timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 1000 1024 8 >> $O/lat.jsonl 2>> $O/lat.err || exit 4
done
