#!/bin/bash
# ping-pong (config 3) with and without IPC COPY, 2 ranks on the one GPU
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/pp_ab.txt
for rep in 1 2; do
  for v in copy slab; do
    for tb in "4194304 512" "4194304 256" "4194304 64" "1048576 512" "65536 512"; do
      E=TEMPI_DATATYPE_IPC=1; [ $v = slab ] && E="$E TEMPI_NO_IPC_COPY=1"
      r=$(env $E timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 200 $tb 2>&1 | grep '^{') || exit 3
      echo "$v $tb $r" | tee -a $O/pp_ab.txt
    done
  done
done
