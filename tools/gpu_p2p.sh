#!/bin/bash
# the p2p / direct GPU tests, then the halo at 1, 2, 4 ranks (defaults)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py tests/test_direct_gpu.py -x -q --timeout 120 --timeout-method thread > $O/p2p_tests.log 2>&1
rc=$?; tail -3 $O/p2p_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for n in 1 2 4; do
    timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>&1 | grep '^{' || exit 3
  done
done
