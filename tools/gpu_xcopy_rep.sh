#!/bin/bash
# IPC COPY data check, repeated: system-scope source loads vs plain loads
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/xrep.txt
export TEMPI_DATATYPE_IPC=1 TEMPI_IPC_COPY_MIN_BYTES=1 TEMPI_IPC_COPY_MIN_BLOCK=1
for rep in 1 2 3 4 5; do
  for v in sys plain; do
    E=; [ $v = plain ] && E=TEMPI_IPC_PLAIN_LOADS=1
    env $E timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 python -u tests/mpi_progs/xcopy.py > $O/xrep_one.txt 2>&1
    echo "$v rep=$rep rc=$? $(grep -h 'differ' $O/xrep_one.txt | tr '\n' ' ')" | tee -a $O/xrep.txt
  done
done
