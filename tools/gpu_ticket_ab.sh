#!/bin/bash
# A/B of batch tickets in the transport (TEMPI_BATCH_TICKETS=1, a trial build:
# DESIGN §9, profiles/r02/ticket_ab_s14.jsonl) against event queries alone: the reference's 1D ping-pong at 2 ranks (small to 1 MiB,
# every byte checked) and the 512^3 halo at 1 and 2 ranks, alternating.
# usage: tools/gpu_ticket_ab.sh OUT
set -o pipefail
cd "$(dirname "$0")/.."
export HYDRA_LAUNCHER=fork
O=gpurun_out/$1; rm -f $O
for r in 1 2; do
  for v in default tickets; do
    E=; [ $v = tickets ] && E="TEMPI_BATCH_TICKETS=1"
    env $E timeout -k 10 200 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_1d 200 1 64 4096 65536 1048576 --check \
      | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, \"app\": \"pingpong_1d\", /" >> $O || exit 4
    for n in 1 2; do
      env $E timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 \
        | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, \"app\": \"halo\", /" >> $O || exit 5
    done
  done
done
echo "wrote $(wc -l < $O) lines"
