#!/bin/bash
# quick GPU iteration: chosen pytest files, then the 1-rank halo (+ profile)
# usage: tools/gpu_quick.sh "tests/test_a.py tests/test_b.py"
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest $1 -x -v --timeout 100 --timeout-method thread > $O/quick_tests.log 2>&1
  rc=$?; tail -5 $O/quick_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for mode in "" "--neighbor"; do
  TEMPI_PRINT_COUNTERS=1 timeout -k 10 120 tempi_amd/lib/halo_exchange 10 512 $mode > $O/halo_1.json 2>&1 || exit 3
  cat $O/halo_1.json
done
TEMPI_NO_DIRECT=1 timeout -k 10 120 tempi_amd/lib/halo_exchange 10 512 > $O/halo_1_nodirect.json 2>&1 || exit 3
cat $O/halo_1_nodirect.json
rm -rf $O/halo_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/halo_prof -o run -- tempi_amd/lib/halo_exchange 10 512 > $O/halo_prof.log 2>&1 || exit 4
cut -d, -f1-4 $O/halo_prof/run_kernel_stats.csv
