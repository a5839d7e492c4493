#!/bin/bash
# anyrecv at 1 rank with TEMPI_NO_DIRECT under knob variants, 60 s each:
# the last case each reached (a hang shows where).
cd "$(dirname "$0")/.."
export HYDRA_LAUNCHER=fork
for v in "-" "TEMPI_NO_SHM_ACKS=1" "TEMPI_EAGER_FLUSH=1"; do E=; [ "$v" != "-" ] && E="$v"
  env $E TEMPI_NO_DIRECT=1 timeout -k 5 60 /opt/conda/bin/mpiexec -n 1 python -u tests/mpi_progs/anyrecv.py > gpurun_out/anyrecv_$$.log 2>&1
  echo "[$v] rc=$? last: $(grep -E '^case|RESULT' gpurun_out/anyrecv_$$.log | tail -1)"
done
