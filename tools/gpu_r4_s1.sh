#!/bin/bash
# Round 4, first session: the whole -m gpu suite under -x (the driver's form),
# then the kernel A/B that bisects the 3D 2:18 pack regression (round-3
# kernels before/after ab92370 and 3d55e7d against the working tree; build
# them with tools/build_ab.sh ab92370^ ab92370 3d55e7d), then the N=1 bench
# line. Stops at the first failing step.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out
mkdir -p $O
echo "== tests"
# (TESTS=path limits the run, e.g. tests/test_round3_gpu.py)
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== kab 2:18"
# 3D 2:18 of the sweep: 23170 planes x 23170 rows, pitch 18, plane 23173*18;
# its 2D twin; the headline
bash tools/kab.sh kab_218_r4s1.jsonl 2 20 2:23170:417114:23170:18 2:536870912:18 512:2097152:1024 || exit 5
echo "== bench"
bash tools/gpu_bench_n1.sh
