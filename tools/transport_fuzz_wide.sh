#!/bin/bash
# A widened run of the transport fuzz (tests/mpi_progs/fuzz.py) on the GPU box:
# SEEDS seeds x 1-4 ranks x ROUNDS rounds, plain and --modes, with the
# transport switches rotated over the seeds (none, no self channel, three
# stream lanes, no IPC COPY, no DIRECT). One line per run into
# gpurun_out/transport_fuzz_wide.txt; stops at the first failing run.
# usage: bash tools/transport_fuzz_wide.sh [SEEDS] [ROUNDS]
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O
OUT=$O/transport_fuzz_wide.txt; : > $OUT
SEEDS=${1:-10}; ROUNDS=${2:-20}
ENVS=("" "TEMPI_NO_SELF_CHANNEL=1" "TEMPI_STREAMS=3" "TEMPI_NO_IPC_COPY=1" "TEMPI_NO_DIRECT=1")
for s in $(seq 1 $SEEDS); do
  seed=$((1000 + s)); e=${ENVS[$((s % ${#ENVS[@]}))]}
  for n in 1 2 3 4; do
    for modes in "" "--modes"; do
      log=$O/tfw.log
      env $e timeout -k 10 300 /opt/conda/bin/mpiexec -n $n python -u tests/mpi_progs/fuzz.py $ROUNDS $seed $modes > $log 2>&1
      rc=$?
      res=$(grep -o "RESULT errors=[0-9]*" $log | sort | uniq -c | tr '\n' ' ')
      echo "seed=$seed n=$n rounds=$ROUNDS modes=${modes:-none} env=${e:-none} rc=$rc $res" | tee -a $OUT
      if [ $rc -ne 0 ] || grep -q "errors=[1-9]" $log; then
        tail -30 $log >> $OUT
        exit 1
      fi
    done
  done
done
echo "all $(wc -l < $OUT) runs clean" | tee -a $OUT
