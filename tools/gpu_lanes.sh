#!/bin/bash
# stream lanes: the p2p / direct GPU tests, then the halo (1, 2, 4 ranks) for
# the old build (tools/_variants/old) and the new one at TEMPI_STREAMS=1..4,
# alternating, all on one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
if [ "$1" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py tests/test_direct_gpu.py -x -q --timeout 120 --timeout-method thread > $O/lanes_tests.log 2>&1
  rc=$?; tail -3 $O/lanes_tests.log; [ $rc -eq 0 ] || exit $rc
fi
rm -f $O/lanes.txt
for rep in 1 2; do
  for v in old s1 s2 s3 s4; do
    for n in 1 2 4; do
      LP=; S=3
      case $v in old) LP=$PWD/tools/_variants/old ;; s*) S=${v#s} ;; esac
      r=$(LD_LIBRARY_PATH=$LP TEMPI_STREAMS=$S timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>&1 | grep '^{' | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['us_per_iter'], r['us_min'])") || exit 3
      echo "$v n=$n $r" | tee -a $O/lanes.txt
    done
  done
done
rm -rf $O/halo_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/halo_prof -o run -- tempi_amd/lib/halo_exchange 10 512 > $O/halo_prof.log 2>&1 || exit 4
