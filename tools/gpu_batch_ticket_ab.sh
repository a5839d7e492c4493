#!/bin/bash
# Transport batches completing by a ticket their last launch stores (default)
# against HIP events (TEMPI_NO_BATCH_TICKET=1): ping-pong latency (contiguous
# and strided), the halo at 1 / 2 ranks (Isend and neighbourhood forms) and a
# small-message alltoallv; two alternations. gpurun_out/batch_ticket_ab.jsonl.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; OUT=$O/batch_ticket_ab.jsonl; : > $OUT
L=tempi_amd/lib
run() { # label n argv...
  local label=$1 n=$2; shift 2
  timeout -k 10 120 /opt/conda/bin/mpiexec -n $n "$@" 2>> $O/batch_ticket_ab.err | grep '^{' \
    | sed "s/^{/{\"label\": \"$label\", \"variant\": \"$V\", /" >> $OUT || { echo "failed: $label $V"; exit 3; }
}
for rep in 1 2; do
  for V in ticket event; do
    if [ $V = event ]; then export TEMPI_NO_BATCH_TICKET=1; else unset TEMPI_NO_BATCH_TICKET; fi
    run pp1d 2 $L/pingpong_1d 200 1024 65536 1048576 --check
    run ppnd_1k 2 $L/pingpong_nd 200 1024 8 --check
    run ppnd_64k 2 $L/pingpong_nd 200 65536 64 --check
    run halo_n1 1 $L/halo_exchange 10 512
    run halo_n2 2 $L/halo_exchange 10 512
    run halo_n2_nbr 2 $L/halo_exchange 10 512 --neighbor
    run a2av_1e3 8 $L/alltoallv_sparse 50 --scale 1000 --density 1.0 --check
  done
done
echo "lines: $(wc -l < $OUT)"
