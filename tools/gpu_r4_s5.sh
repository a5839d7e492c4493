#!/bin/bash
# Round 4, evidence session: the whole -m gpu suite in the driver's form
# (one process, -x), the N=1 bench line, rocprof kernel-trace stats and the
# FETCH_SIZE / WRITE_SIZE passes of the headline (tools/gpu_prof.sh), and the
# driver's torchrun command at N=2 (two ranks sharing this box's GPU).
# Stops at the first failing step.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out
mkdir -p $O
echo "== all gpu tests (-x)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench N=1"
bash tools/gpu_bench_n1.sh || exit 5
echo "== rocprof"
bash tools/gpu_prof.sh || exit 6
python3 tools/pmc_summary.py $O/prof_FETCH_SIZE $O/prof_WRITE_SIZE pack_kernel > $O/bench_pmc_summary.txt
cat $O/bench_pmc_summary.txt
echo "== torchrun N=2"
NS=2 bash tools/gpu_torchrun.sh || exit 7
