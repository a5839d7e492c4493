#!/bin/bash
# two independent 1-rank halo jobs on the one GPU at once (long enough to
# overlap), TEMPI_STREAMS=1 vs 3: does sharing the GPU alone make lanes hurt?
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/lanes4.txt
j() { python3 -c "import sys,json; r=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][0]); print(r['us_per_iter'], r['us_min'])"; }
for rep in 1 2; do
  for S in 1 3; do
    TEMPI_STREAMS=$S timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 800 512 > $O/pair_a.txt 2>&1 &
    pa=$!
    TEMPI_STREAMS=$S timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 800 512 > $O/pair_b.txt 2>&1 &
    pb=$!
    wait $pa || exit 4
    wait $pb || exit 4
    echo "pair S=$S $(j < $O/pair_a.txt) | $(j < $O/pair_b.txt)" | tee -a $O/lanes4.txt
    r=$(TEMPI_STREAMS=$S timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 800 512 2>&1 | j) || exit 3
    echo "solo S=$S $r" | tee -a $O/lanes4.txt
  done
done
