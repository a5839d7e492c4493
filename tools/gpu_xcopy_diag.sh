#!/bin/bash
# the xcopy receiver program (tests/mpi_progs/xcopy.py) repeated under the
# COPY and unmapped (forced NACK -> host) settings, to characterise the
# intermittent 'realloc' mismatch; no GPU fault is involved (a data check)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/xdiag.log
for rep in $(seq 1 ${REPS:-4}); do
  for v in "TEMPI_FAULT_IPC_OPEN=1" "TEMPI_X=1"; do
    echo "== rep $rep $v" >> $O/xdiag.log
    env TEMPI_DATATYPE_IPC=1 TEMPI_IPC_COPY_MIN_BLOCK=1 TEMPI_IPC_COPY_MIN_BYTES=1 $v HYDRA_LAUNCHER=fork \
      timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 python -u tests/mpi_progs/xcopy.py >> $O/xdiag.log 2>&1
    rc=$?
    echo "rc=$rc" >> $O/xdiag.log
    [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  done
done
