#!/bin/bash
# One parameterised GPU session (replaces the per-session gpu_r4_s*.sh
# scripts of round 4). Usage, on the GPU box:
#   bash tools/gpu_session.sh STEP [STEP ...]
# Steps (run in the order given; the session stops at the first failure, so a
# GPU fault, abort or time limit never has a second GPU step behind it):
#   tests        the whole -m gpu suite in the driver's form (-x, one process)
#   focus        only the tests FOCUS (a pytest -k expression) selects
#   bench        the driver's N=1 bench line (tools/gpu_bench_n1.sh)
#   prof         rocprofv3 kernel-trace stats + FETCH_SIZE / WRITE_SIZE passes
#                of the headline (tools/gpu_prof.sh)
#   halo         halo_exchange 10 512 at RANKS (default "1 2") ranks, both forms
#   halo-trace   kernel + HIP API trace of the 1-rank halo (tools/halo_trace_summary.py)
#   halo-timeline  TEMPI's host timeline (TEMPI_TIMELINE) beside a kernel-only
#                trace of the 1-rank halo: idle attribution (tools/halo_timeline.py)
#   sweep-pmc    FETCH_SIZE / WRITE_SIZE passes over the sweep shapes SHAPES
#                (DIMS:BLOCK:STRIDE ...; tools/sweep_pmc.py)
#   measure      measure_system --quick at 2 ranks into gpurun_out/perf_quick.json
#   torchrun     the driver's torchrun command at NS (default "2") ranks
#   n8           the driver's torchrun command at 8 ranks (tools/gpu_n8.sh)
#   kab          kernel A/B: tools/kab.sh $KAB_OUT $KAB_ROUNDS $KAB_ITERS $KAB_SHAPES
#   koff         tools/bin/kbench on the in-tree library, KBENCH_OFFSET in turn
#                each of $KOFF_OFFSETS (default "24 32"), $KOFF_ROUNDS rotations,
#                shapes $KOFF_SHAPES -> gpurun_out/koff.jsonl
#   launchsplit  tools/bin/launchsplit: dispatch / execution / visibility of
#                the config-1 synchronous call -> gpurun_out/launchsplit.jsonl
#   halo-ab      halo_exchange $HALO_ITERS (default 30) 512 at $HALO_RANKS (default 1) under each
#                environment of $HALO_AB ("A=1,B=2 A=0" style, "-" for none),
#                $HALO_ROUNDS rotations -> gpurun_out/halo_ab.jsonl
#   ls-ab        launchsplit under each environment of $LS_AB (as HALO_AB), $LS_ROUNDS rotations
#   launch-check the GPU tests LC_FOCUS selects with TEMPI_LAUNCH_CHECK=1 (every
#                TEMPI launch synchronised and checked)
#   kpmc         rocprofv3 --pmc passes ($KPMC_PASSES, ';'-separated counter
#                lists, one run each) over tools/bin/kbench (pack / unpack /
#                memcpy, no copies) of $KPMC_SHAPES -> gpurun_out/kpmc.txt
#   diag-hostmalloc  tools/diag_hostmalloc.py (both HIP runtimes in one
#                process; may end in a HIP error: run it LAST)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
MPIEXEC=/opt/conda/bin/mpiexec
for step in "$@"; do
  echo "== $step $(date +%T)"
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread --durations=25 \
      > $O/gpu_tests.log 2>&1
    rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
  focus)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "$FOCUS" \
      > $O/gpu_focus.log 2>&1
    rc=$?; tail -n 15 $O/gpu_focus.log; [ $rc -eq 0 ] || exit $rc ;;
  bench)
    bash tools/gpu_bench_n1.sh || exit 5 ;;
  prof)
    bash tools/gpu_prof.sh || exit 7 ;;
  halo)
    rm -f $O/halo.jsonl
    for n in ${RANKS:-1 2}; do
      for mode in "" "--neighbor"; do
        timeout -k 10 300 $MPIEXEC -n $n tempi_amd/lib/halo_exchange 10 512 $mode >> $O/halo.jsonl 2>> $O/halo.err || exit 9
      done
    done
    cat $O/halo.jsonl ;;
  halo-trace)
    rm -rf $O/halo_trace
    timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d $O/halo_trace -o run \
      -- tempi_amd/lib/halo_exchange 10 512 $HALO_ARGS > $O/halo_trace.log 2>&1 || exit 10
    grep '^{' $O/halo_trace.log
    python3 tools/halo_trace_summary.py $O/halo_trace > $O/halo_trace_summary.txt 2>&1 || exit 11
    cat $O/halo_trace_summary.txt ;;
  halo-timeline)
    rm -rf $O/halo_tl $O/halo_tl.r0.csv
    TEMPI_TIMELINE=$O/halo_tl timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/halo_tl -o run \
      -- tempi_amd/lib/halo_exchange 10 512 $HALO_ARGS > $O/halo_tl.log 2>&1 || exit 17
    grep '^{' $O/halo_tl.log
    python3 tools/halo_timeline.py $O/halo_tl.r0.csv $O/halo_tl > $O/halo_timeline.txt 2>&1 || exit 18
    cat $O/halo_timeline.txt ;;
  sweep-pmc)
    timeout -k 10 900 python3 tools/sweep_pmc.py $O/sweep_pmc.json ${SHAPES:-2:2:18 3:2:18 3:1:2 3:2:4 3:3:19 2:24:40 3:64:128 2:8:512} \
      > $O/sweep_pmc.log 2>&1 || exit 12
    cat $O/sweep_pmc.log ;;
  measure)
    rm -f $O/perf_quick.json
    timeout -k 10 400 $MPIEXEC -n 2 tempi_amd/lib/measure_system --quick --out $O/perf_quick.json \
      > $O/measure.log 2>&1 || exit 13
    tail -n 2 $O/measure.log ;;
  torchrun)
    bash tools/gpu_torchrun.sh || exit 14 ;;
  n8)
    bash tools/gpu_n8.sh || exit 15 ;;
  kab)
    bash tools/kab.sh $KAB_OUT ${KAB_ROUNDS:-3} ${KAB_ITERS:-20} $KAB_SHAPES || exit 16
    python3 tools/kab_summary.py $O/$KAB_OUT 2>&1 | tail -40 ;;
  koff)
    rm -f $O/koff.jsonl
    for r in $(seq ${KOFF_ROUNDS:-3}); do
      for off in ${KOFF_OFFSETS:-24 32}; do
        KBENCH_OFFSET=$off timeout -k 10 300 tools/bin/kbench tempi_amd/lib/libtempi_hip.so ${KOFF_ITERS:-20} $KOFF_SHAPES \
          | sed "s/^{/{\"round\": $r, /" >> $O/koff.jsonl || exit 19
      done
    done
    cat $O/koff.jsonl ;;
  launchsplit)
    timeout -k 10 120 tools/bin/launchsplit ${LS_REPS:-2000} > $O/launchsplit.jsonl 2>&1 || exit 20
    cat $O/launchsplit.jsonl ;;
  halo-ab)
    rm -f $O/halo_ab.jsonl
    for r in $(seq ${HALO_ROUNDS:-3}); do
      for v in $HALO_AB; do
        envs=$([ "$v" = "-" ] && echo "" || echo "$v" | tr ',' ' ')
        env $envs timeout -k 10 300 $MPIEXEC -n ${HALO_RANKS:-1} tempi_amd/lib/halo_exchange ${HALO_ITERS:-30} 512 2>> $O/halo_ab.err \
          | grep '^{' | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/halo_ab.jsonl || exit 21
      done
    done
    python3 -c "
import json,collections
d=collections.defaultdict(list)
for l in open('$O/halo_ab.jsonl'): j=json.loads(l); d[j['variant']].append(round(j['us_per_iter'],1))
for k,v in d.items(): print(k, v)" ;;
  ls-ab)
    rm -f $O/launchsplit_ab.jsonl
    for r in $(seq ${LS_ROUNDS:-3}); do
      for v in ${LS_AB:--}; do
        envs=$([ "$v" = "-" ] && echo "" || echo "$v" | tr ',' ' ')
        env $envs timeout -k 10 120 tools/bin/launchsplit ${LS_REPS:-2000} 2>&1 \
          | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/launchsplit_ab.jsonl || exit 22
      done
    done
    cat $O/launchsplit_ab.jsonl ;;
  launch-check)
    TEMPI_LAUNCH_CHECK=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      -k "$LC_FOCUS" > $O/launch_check.log 2>&1
    rc=$?; tail -n 15 $O/launch_check.log; [ $rc -eq 0 ] || exit $rc ;;
  kpmc)
    rm -rf $O/kpmc_*; rm -f $O/kpmc.txt
    IFS=';' read -ra passes <<< "$KPMC_PASSES"
    for shape in $KPMC_SHAPES; do
      i=0
      for pass in "${passes[@]}"; do
        i=$((i+1)); d=$O/kpmc_${shape//:/_}_$i
        KBENCH_NO_COPY=1 timeout -s KILL 120 rocprofv3 --pmc $pass -d $d -o run --output-format csv \
          -- tools/bin/kbench tempi_amd/lib/libtempi_hip.so ${KPMC_ITERS:-3} $shape > $d.log 2>&1 || exit 23
      done
      echo "== $shape (KBENCH_OFFSET=${KBENCH_OFFSET:-0})" >> $O/kpmc.txt
      python3 tools/pmc_kernels.py $O/kpmc_${shape//:/_}_* >> $O/kpmc.txt 2>&1 || exit 24
    done
    cat $O/kpmc.txt ;;
  diag-hostmalloc)
    timeout -k 10 300 python3 -u tools/diag_hostmalloc.py > $O/diag_hostmalloc.jsonl 2>&1
    rc=$?; tail -n 40 $O/diag_hostmalloc.jsonl; exit $rc ;;
  *)
    echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done $(date +%T)"
