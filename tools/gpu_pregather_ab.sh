#!/bin/bash
# Pre-gather of narrow-row direct sends during the send burst
# (TEMPI_PREGATHER_BYTES; p2p_internal.hpp): the 512^3 halo (Isend form) at 1
# and 2 ranks, default vs 32 MiB and 128 MiB budgets, two alternations, with
# the counters (direct_pregathers). gpurun_out/pregather_ab.jsonl.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; OUT=$O/pregather_ab.jsonl; : > $OUT
for rep in 1 2; do
  for n in 1 2; do
    for B in 0 33554432 134217728; do
      r=$(TEMPI_PREGATHER_BYTES=$B TEMPI_PRINT_COUNTERS=1 timeout -k 10 200 /opt/conda/bin/mpiexec -n $n \
          tempi_amd/lib/halo_exchange 10 512 2> $O/pregather_cnt.txt | grep '^{') || { echo "failed n=$n B=$B"; exit 3; }
      pg=$(grep -o 'pregather[a-z_]*=[0-9]*' $O/pregather_cnt.txt | head -1)
      echo "{\"pregather_bytes\": $B, \"ranks\": $n, \"rep\": $rep, \"counters\": \"$pg\", \"r\": $r}" >> $OUT
      echo "n=$n B=$B $(echo "$r" | grep -o '"us_per_iter": [0-9.]*') $pg"
    done
  done
done
