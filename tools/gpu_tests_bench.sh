#!/bin/bash
# GPU session: the whole -m gpu suite (FOCUS="pytest -k expr" runs those tests
# first), then the driver's N=1 bench line (tools/gpu_bench_n1.sh).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O
if [ -n "$FOCUS" ]; then
  echo "== focused tests: $FOCUS"
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "$FOCUS" \
    > $O/gpu_focus.log 2>&1
  rc=$?; tail -n 3 $O/gpu_focus.log; [ $rc -eq 0 ] || exit $rc
fi
echo "== all gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
bash tools/gpu_bench_n1.sh
