#!/bin/bash
# where a synchronous small MPI_Pack's time goes.
# tools/syncbench (C ABI, per phase) with and without folded tickets, then
# BASELINE config 1 exactly through MPI_Pack in C (apps/mpi_pack --shape):
# TEMPI on device buffers (ticket, folded or not; hipStreamSynchronize) and
# MPICH on host buffers, pinned to one core; three alternations.
# JSON lines in gpurun_out/sync2.jsonl.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; OUT=$O/sync2.jsonl; : > $OUT
for r in 1 2 3; do
  timeout -k 10 60 tools/_variants/syncbench tempi_amd/lib/libtempi_hip.so 2000 | sed "s/^{/{\"round\": $r, \"bench\": \"syncbench\", /" >> $OUT || exit 3
  TEMPI_FOLD_MAX_BLOCKS=0 timeout -k 10 60 tools/_variants/syncbench tempi_amd/lib/libtempi_hip.so 2000 | sed "s/^{/{\"round\": $r, \"bench\": \"syncbench\", /" >> $OUT || exit 3
  for v in fold nofold stream host; do
    E="TEMPI_X=1"; A=""
    [ $v = nofold ] && E="TEMPI_FOLD_MAX_BLOCKS=0"
    [ $v = stream ] && E="TEMPI_STREAM_SYNC=1"
    [ $v = host ] && E="TEMPI_DISABLE=1" && A="--host"
    env $E timeout -k 10 60 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/mpi_pack 1000 $A --shape 1024:512:1024 --pin \
      | sed "s/^{/{\"round\": $r, \"bench\": \"config1\", \"variant\": \"$v\", /" >> $OUT || exit 4
    env $E timeout -k 10 60 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/mpi_pack 1000 $A --shape 2:512:1024 --pin \
      | sed "s/^{/{\"round\": $r, \"bench\": \"1KiB\", \"variant\": \"$v\", /" >> $OUT || exit 4
  done
done
echo "sync2 lines: $(wc -l < $OUT)"
