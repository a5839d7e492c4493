#!/bin/bash
# neighbour-collective tests, then the 1/2/4-rank halo in MPI_Neighbor_alltoallw
# mode: tools/_variants/old vs the tree's build, alternating
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_p2p_gpu.py -k "neighbor or halo" -x -q --timeout 150 --timeout-method thread > $O/nbr_tests.log 2>&1
rc=$?; tail -3 $O/nbr_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f $O/nbr_ab.txt
for rep in 1 2; do
  for v in old new; do
    for n in 1 2 4; do
      LP=; [ $v = old ] && LP=$PWD/tools/_variants/old
      r=$(LD_LIBRARY_PATH=$LP timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 --neighbor 2>&1 | grep '^{' | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['us_per_iter'], r['us_min'])") || exit 3
      echo "$v n=$n $r" | tee -a $O/nbr_ab.txt
    done
  done
done
