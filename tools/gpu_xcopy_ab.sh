#!/bin/bash
# IPC COPY A/B on one box: halo at 2 / 4 ranks (strong and weak) with and
# without (TEMPI_NO_IPC_COPY), alternating, counters of rank 0
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/xcopy_ab.txt
for rep in 1 2 3; do
  for v in copy slab; do
    for n in 2 4; do
      E=TEMPI_PRINT_COUNTERS=1; [ $v = slab ] && E="$E TEMPI_NO_IPC_COPY=1"
      env $E timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 > $O/xab_one.txt 2>&1 || exit 3
      echo "$v n=$n $(grep -o '"us_per_iter": [0-9.]*' $O/xab_one.txt) $(grep -o 'rank0_us_per_iter.*' $O/xab_one.txt) $(grep 'tempi r0' $O/xab_one.txt | grep -o 'ipc=[0-9]*')" | tee -a $O/xcopy_ab.txt
    done
  done
done
