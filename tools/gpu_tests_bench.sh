#!/bin/bash
# GPU session: the tests touched by this change first, then the whole -m gpu
# suite, then the driver's N=1 bench line (tools/gpu_bench_n1.sh).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O
echo "== focused tests"
timeout -k 10 300 python -u -m pytest tests/test_pack_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "ticket or pinned or golden" > $O/gpu_focus.log 2>&1
rc=$?; tail -n 3 $O/gpu_focus.log; [ $rc -eq 0 ] || exit $rc
echo "== focused p2p tests"
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "probe or neighbor or halo_exchange_content" > $O/gpu_focus_p2p.log 2>&1
rc=$?; tail -n 3 $O/gpu_focus_p2p.log; [ $rc -eq 0 ] || exit $rc
echo "== all gpu tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
bash tools/gpu_bench_n1.sh
