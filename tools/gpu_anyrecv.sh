export HYDRA_LAUNCHER=fork
for cfg in "2:" "1:" "2:TEMPI_DATATYPE_IPC=1 TEMPI_FAULT_IPC_OPEN=1" "1:TEMPI_NO_DIRECT=1" "2:TEMPI_DATATYPE_IPC=1 TEMPI_IPC_COPY_MIN_BYTES=1 TEMPI_IPC_COPY_MIN_BLOCK=1"; do
  n=${cfg%%:*}; e=${cfg#*:}
  echo "=== n=$n env=$e"
  env $e timeout -k 5 90 /opt/conda/bin/mpiexec -n $n python -u tests/mpi_progs/anyrecv.py > gpurun_out/ar.log 2>&1; rc=$?
  echo "rc=$rc"; grep -v "^case" gpurun_out/ar.log | tail -n 8; grep "^case" gpurun_out/ar.log | tail -n 1
  [ $rc -eq 124 ] || [ $rc -eq 137 ] && break
done
exit 0
