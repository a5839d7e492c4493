#!/bin/bash
# Halo A/B on one box: the default build vs the same with the environment
# assignment given as $1 (e.g. TEMPI_NO_SELF_CHANNEL=1), alternating, at the
# rank counts in $2 (default "1 2 4"; 512^3, 8 quantities, 10 iterations).
# JSON lines to gpurun_out/halo_ab.jsonl; one summary line per run.
cd "$(dirname "$0")/.."
export HYDRA_LAUNCHER=fork
A=$1
RANKS=${2:-1 2 4}
O=gpurun_out/halo_ab.jsonl
rm -f $O
for rep in 1 2; do
  for n in $RANKS; do
    for v in default alt; do
      E=; [ $v = alt ] && E="$A"
      r=$(env $E TEMPI_PRINT_COUNTERS=1 timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2> gpurun_out/halo_ab_cnt.txt | grep '^{') || exit 3
      echo "{\"variant\": \"$([ $v = alt ] && echo "$A" || echo default)\", \"rep\": $rep, \"r\": $r}" >> $O
      echo "$v n=$n $(echo "$r" | grep -o '"us_per_iter": [0-9.]*') $(grep -o 'testsome=[0-9.]*' gpurun_out/halo_ab_cnt.txt | head -1)"
    done
  done
done
