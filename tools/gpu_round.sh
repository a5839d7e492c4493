#!/bin/bash
# One GPU session: tests, kernel variants, bench, rocprof (trace + PMC), apps.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
step() { echo "== $*"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
step kbench
SHAPES="512:2097152:1024 4096:262144:4160 64:16777216:128 8:67108864:16 24:512:2386944:512:4608 1:268435456:2 3:89478485:7 2:134217728:4 1:134217728:8 4:67108864:16 1073741824"
rm -f $O/kbench.jsonl $O/pingpong.jsonl
for v in $(ls tools/_variants/ | sed -n 's/^libtempi_hip_\(.*\)\.so$/\1/p'); do
  timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/kbench.jsonl || exit 5
done
step bench
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 6
tail -c 600 $O/bench.json
step rocprof-trace
rm -rf $O/prof_trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic > $O/prof_trace.log 2>&1 || exit 7
for c in FETCH_SIZE WRITE_SIZE; do
  step rocprof-pmc $c
  rm -rf $O/prof_$c
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/prof_$c -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-halo > $O/prof_$c.log 2>&1 || exit 8
done
step halo
rm -f $O/halo.jsonl
for n in 1 2 4; do
  for mode in "" "--neighbor"; do
    timeout -k 10 300 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 $mode >> $O/halo.jsonl 2>> $O/halo.err || exit 9
  done
done
step hbench
rm -f $O/hbench.jsonl
timeout -k 10 120 tools/_variants/hbench tools/_variants/libtempi_hip_cur.so 20 >> $O/hbench.jsonl || exit 11
step halo-prof
rm -rf $O/halo_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/halo_prof -o run -- tempi_amd/lib/halo_exchange 10 512 > $O/halo_prof.log 2>&1 || exit 12
step pingpong
for m in TEMPI_DATATYPE_IPC TEMPI_DATATYPE_ONESHOT TEMPI_DATATYPE_STAGED; do
  for t in 1024 1048576 4194304; do
    for b in 1 8 64 512; do
      env $m=1 timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 50 $t $b >> $O/pingpong.jsonl 2>> $O/pingpong.err || exit 10
    done
  done
done
step done
