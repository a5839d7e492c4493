#!/bin/bash
# p2p GPU tests, then an A/B of libtempi builds on the same box (halo at 2/4
# ranks, alternating): old = tools/_variants/old (LD_LIBRARY_PATH beats RUNPATH)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py -x -q --timeout 120 --timeout-method thread > $O/p2p_tests.log 2>&1
  rc=$?; tail -2 $O/p2p_tests.log; [ $rc -eq 0 ] || exit $rc
fi
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
