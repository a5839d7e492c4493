#!/bin/bash
# A/B of libtempi builds on the same box: halo at 1/2/4 ranks, alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/ab.txt
for rep in 1 2; do
  for v in old new; do
    for n in 2 4; do
      if [ $v = old ]; then LP=$PWD/tools/_variants/old; else LP=; fi
      r=$(LD_LIBRARY_PATH=$LP timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>&1 | grep '^{' | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['us_per_iter'], r['us_min'])") || exit 3
      echo "$v n=$n $r" | tee -a $O/ab.txt
    done
  done
done
