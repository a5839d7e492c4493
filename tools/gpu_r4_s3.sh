#!/bin/bash
# Round 4, third session:
#  1. the hot path's parity suites (oracle, pack, dense, direct) and the
#     round-3 transport tests, after the WTC kernel split and the AQL /
#     pre-gather removal;
#  2. kernel A/B (tools/build_ab.sh ab92370^ "r9:-DTEMPI_DENSE_RATIO=9"
#     "r16:-DTEMPI_DENSE_RATIO=16"): the 3D / 2D 2:18 shapes and the headline,
#     and the 512^3 halo's face shapes as strided -> strided copies (x face:
#     24-B rows at pitch 4608; y and z faces: 4 KiB rows);
#  3. the 1-rank 512^3 halo with TEMPI_PRINT_COUNTERS (host time split);
#  4. the N=1 bench line.
# Stops at the first failing step.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out
mkdir -p $O
echo "== parity + round-3 tests"
timeout -k 10 600 python -u -m pytest tests/test_oracle.py tests/test_pack_gpu.py tests/test_dense_gpu.py \
  tests/test_direct_gpu.py tests/test_round3_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread \
  > $O/gpu_tests_s3.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests_s3.log; [ $rc -eq 0 ] || exit $rc
echo "== kab"
# pitch 4608, 518 rows per plane: plane stride 2386944
bash tools/kab.sh kab_r4s3.jsonl 2 20 2:23170:417114:23170:18 2:536870912:18 512:2097152:1024 \
  24:512:2386944:512:4608 4096:512:2386944:3:4608 4096:3:2386944:512:4608 || exit 5
echo "== hbench: the halo's regions as batches (copy GB/s per class, host time per batch)"
for v in cur ab92370_; do
  timeout -k 10 200 tools/_variants/hbench tools/_variants/libtempi_hip_$v.so 10 > $O/hbench_$v.jsonl || exit 7
  cut -c1-400 $O/hbench_$v.jsonl
done
echo "== halo 1 rank, counters"
: > $O/halo1_counters.txt
for rep in 1 2; do
  TEMPI_PRINT_COUNTERS=1 timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 10 512 \
    > $O/halo1.out 2> $O/halo1.err || exit 6
  grep '^{' $O/halo1.out | cut -c1-200
  grep '^{' $O/halo1.out >> $O/halo1_counters.txt
  grep '^\[tempi' $O/halo1.err | tee -a $O/halo1_counters.txt
done
echo "== bench"
bash tools/gpu_bench_n1.sh
