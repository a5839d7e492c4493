#!/bin/bash
# send-order gate: the order / p2p / direct GPU tests, then an A/B of the
# halo (1, 2, 4 ranks) against tools/_variants/old on the same box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py tests/test_direct_gpu.py -x -q --timeout 120 --timeout-method thread > $O/order_tests.log 2>&1
rc=$?; tail -3 $O/order_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f $O/ab.txt
for rep in 1 2; do
  for v in old new; do
    for n in 1 2 4; do
      if [ $v = old ]; then LP=$PWD/tools/_variants/old; else LP=; fi
      r=$(LD_LIBRARY_PATH=$LP timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>&1 | grep '^{' | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['us_per_iter'], r['us_min'])") || exit 3
      echo "$v n=$n $r" | tee -a $O/ab.txt
    done
  done
done
