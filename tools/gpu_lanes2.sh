#!/bin/bash
# why do extra stream lanes hurt when ranks share the GPU? n=2 halo with
# TEMPI_STREAMS=1/2/3 under AUTO (IPC) and forced ONESHOT, then two
# independent 1-rank halos side by side on the one GPU
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/lanes2.txt
j() { python3 -c "import sys,json; r=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][0]); print(r['us_per_iter'], r['us_min'])"; }
for rep in 1 2; do
  for S in 1 2 3; do
    for m in AUTO ONESHOT; do
      E=; [ $m = ONESHOT ] && E=TEMPI_DATATYPE_ONESHOT=1
      r=$(env $E TEMPI_STREAMS=$S timeout -k 10 200 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/halo_exchange 10 512 2>&1 | j) || exit 3
      echo "n=2 S=$S $m $r" | tee -a $O/lanes2.txt
    done
    # two independent single-rank jobs on the same GPU at once
    TEMPI_STREAMS=$S timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 10 512 > $O/pair_a.txt 2>&1 &
    pa=$!
    TEMPI_STREAMS=$S timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 10 512 > $O/pair_b.txt 2>&1 &
    pb=$!
    wait $pa || exit 4
    wait $pb || exit 4
    echo "pair S=$S $(j < $O/pair_a.txt) | $(j < $O/pair_b.txt)" | tee -a $O/lanes2.txt
  done
done
