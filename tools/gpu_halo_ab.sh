#!/bin/bash
# Halo A/B on one box: the environment variable given as $1 unset vs set,
# alternating, at 1/2/4 ranks (512^3, 8 quantities); JSON lines to
# gpurun_out/halo_ab.jsonl
cd "$(dirname "$0")/.."
export HYDRA_LAUNCHER=fork
V=$1
O=gpurun_out/halo_ab.jsonl
rm -f $O
for rep in 1 2; do
  for n in 1 2 4; do
    for v in on off; do
      E=; [ $v = off ] && E="$V=1"
      r=$(env $E timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 | grep '^{') || exit 3
      echo "{\"variant\": \"$V=$([ $v = off ] && echo 1 || echo unset)\", \"rep\": $rep, \"r\": $r}" >> $O
      echo "$v n=$n $(echo "$r" | grep -o '"us_per_iter": [0-9.]*')"
    done
  done
done
