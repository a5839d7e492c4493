#!/bin/bash
# 1-rank (or $RANKS) 512^3 halo under several environment settings, rotated
# REPS times on one box: bash tools/gpu_halo_knobs.sh "A=1" "B=2 C=3" ...
# ("-" = the defaults). Summary lines on stdout, JSON in gpurun_out/halo_knobs.jsonl.
cd "$(dirname "$0")/.."
export HYDRA_LAUNCHER=fork
O=gpurun_out/halo_knobs.jsonl
: > $O
for rep in $(seq ${REPS:-3}); do
  for v in "$@"; do
    E=; [ "$v" != "-" ] && E="$v"
    r=$(env $E timeout -k 10 120 /opt/conda/bin/mpiexec -n ${RANKS:-1} tempi_amd/lib/halo_exchange 10 512 | grep '^{') || exit 3
    echo "{\"variant\": \"$v\", \"rep\": $rep, \"r\": $r}" >> $O
    echo "[$v] $(echo "$r" | grep -o '"us_per_iter": [0-9.]*') $(echo "$r" | grep -o '"rank0_us_per_iter": {[^}]*}')"
  done
done
