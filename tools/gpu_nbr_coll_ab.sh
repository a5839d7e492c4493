#!/bin/bash
# neighbourhood-collective halo (--neighbor) at 2 and 4 ranks: IPC COPY at
# every size inside the collective (default) vs TEMPI_NO_COLL_COPY=1
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/nbr_coll_ab.txt
for rep in 1 2; do
  for v in TEMPI_X=1 TEMPI_NO_COLL_COPY=1; do
    for n in 2 4; do
      r=$(env $v timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 --neighbor 2>&1 | grep '^{' | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['us_per_iter'], r['us_min'])") || exit 3
      echo "$v n=$n $r" | tee -a $O/nbr_coll_ab.txt
    done
  done
done
