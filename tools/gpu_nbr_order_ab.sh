#!/bin/bash
# MPI_Neighbor_alltoallw: the peers' gathers launched before the self edges'
# copies (default) against copies first (TEMPI_NBR_COPIES_FIRST=1): the
# neighbourhood halo at 1 / 2 / 4 ranks and config 5's neighbourhood form at
# 8 ranks; two alternations. gpurun_out/nbr_order_ab.jsonl.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; OUT=$O/nbr_order_ab.jsonl; : > $OUT
L=tempi_amd/lib
run() { # label n argv...
  local label=$1 n=$2; shift 2
  timeout -k 10 120 /opt/conda/bin/mpiexec -n $n "$@" 2>> $O/nbr_order_ab.err | grep '^{' \
    | sed "s/^{/{\"label\": \"$label\", \"variant\": \"$V\", /" >> $OUT || { echo "failed: $label $V"; exit 3; }
}
for rep in 1 2; do
  for V in gathers_first copies_first; do
    if [ $V = copies_first ]; then export TEMPI_NBR_COPIES_FIRST=1; else unset TEMPI_NBR_COPIES_FIRST; fi
    run nbr_n1 1 $L/halo_exchange 10 512 --neighbor
    run nbr_n2 2 $L/halo_exchange 10 512 --neighbor
    run nbr_n4 4 $L/halo_exchange 10 512 --neighbor
    run nbr_a2av_n8 8 $L/alltoallv_sparse 30 --scale 100000 --density 1.0 --neighbor --check
  done
done
echo "lines: $(wc -l < $OUT)"
