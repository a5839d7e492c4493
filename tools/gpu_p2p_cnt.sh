#!/bin/bash
# p2p GPU tests, then host counters of the 2- and 4-rank halo
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py tests/test_direct_gpu.py -x -q --timeout 120 --timeout-method thread > $O/p2p_tests.log 2>&1
rc=$?; tail -2 $O/p2p_tests.log; [ $rc -eq 0 ] || exit $rc
for n in 1 2 4; do
  TEMPI_PRINT_COUNTERS=1 timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 > $O/halo_cnt_$n.txt 2>&1 || exit 3
  cut -c 1-200 $O/halo_cnt_$n.txt | head -3
done
