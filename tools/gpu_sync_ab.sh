#!/bin/bash
# A/B of how synchronous MPI_Pack / MPI_Unpack wait, on bench_mpi_pack's
# vector points up to 1 MiB, alternating: the default (a ticket stored by a
# kernel queued behind the work, tempi_hip_stream_signal_wait) against
# hipStreamSynchronize (TEMPI_STREAM_SYNC=1). JSON lines to gpurun_out/$1.
# usage: tools/gpu_sync_ab.sh OUT ROUNDS
set -o pipefail
cd "$(dirname "$0")/.."
export HYDRA_LAUNCHER=fork
O=gpurun_out/$1; rm -f $O
for r in $(seq $2); do
  for v in ticket stream; do
    E=; [ $v = stream ] && E="TEMPI_STREAM_SYNC=1"
    env $E timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/mpi_pack 300 --factory vector \
      --max-target 1048576 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O || exit 4
  done
done
echo "wrote $(wc -l < $O) lines"
