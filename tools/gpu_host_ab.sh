#!/bin/bash
# host-buffer traffic with TEMPI active against the library
# alone (TEMPI_DISABLE=1), the same apps bench.py's CPU baselines run
# (TEMPI_BENCH_HOST=1: pageable host buffers): halo 1 rank, ping-pong 2 ranks,
# alltoallv and its neighbourhood form at 8 ranks; two alternations.
# One JSON line per run in gpurun_out/host_ab.jsonl.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork TEMPI_BENCH_HOST=1
O=gpurun_out; mkdir -p $O
OUT=$O/host_ab.jsonl; : > $OUT
L=tempi_amd/lib
run() { # label n argv...
  local label=$1 n=$2; shift 2
  for mode in tempi disabled; do
    if [ $mode = disabled ]; then e="TEMPI_DISABLE=1"; else e="TEMPI_HOST_AB=1"; fi
    line=$(env $e timeout -k 10 120 /opt/conda/bin/mpiexec -n $n "$@" 2>>$O/host_ab.err | grep '^{' | tail -1)
    [ -n "$line" ] || { echo "no line: $label $mode"; exit 3; }
    echo "{\"case\": \"$label\", \"mode\": \"$mode\", \"r\": $line}" >> $OUT
  done
}
for rep in 1 2; do
  run halo512_n1 1 $L/halo_exchange 2 512
  run pp_4MiB_512 2 $L/pingpong_nd 20 4194304 512
  run pp_1MiB_8 2 $L/pingpong_nd 20 1048576 8
  run a2av_1e5_n8 8 $L/alltoallv_sparse 20 --scale 100000 --density 1.0
  run nbr_1e5_n8 8 $L/alltoallv_sparse 20 --scale 100000 --density 1.0 --neighbor
done
echo "host_ab lines: $(wc -l < $OUT)"
