#!/bin/bash
# config 3 matrix: vector(total/bl, bl, 512) byte, total {1 KiB, 1 MiB, 4 MiB},
# bl 1..512 (powers of 2), methods IPC / ONESHOT / STAGED / AUTO; 2 ranks
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/pp_full.jsonl
for m in TEMPI_DATATYPE_IPC TEMPI_DATATYPE_ONESHOT TEMPI_DATATYPE_STAGED TEMPI_DATATYPE_AUTO; do
  for t in 1024 1048576 4194304; do
    for b in 1 2 4 8 16 32 64 128 256 512; do
      echo "{\"method_env\": \"$m\"}" >> $O/pp_full.jsonl
      env $m=1 timeout -k 10 60 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 100 $t $b >> $O/pp_full.jsonl 2>> $O/pp_full.err || exit 4
    done
  done
done
