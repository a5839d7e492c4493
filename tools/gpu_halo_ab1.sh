#!/bin/bash
# 1- and 2-rank halo, old build (tools/_variants/old: libtempi + libtempi_hip
# via LD_LIBRARY_PATH) vs new, alternating on one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/halo_ab1.txt
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then LP=$PWD/tools/_variants/old; else LP=; fi
    for n in 1 2; do
      r=$(LD_LIBRARY_PATH=$LP timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>&1 | grep '^{' | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['us_per_iter'], r['us_min'])") || exit 3
      echo "$v n=$n $r" | tee -a $O/halo_ab1.txt
    done
  done
done
