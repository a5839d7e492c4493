#!/bin/bash
# Round 4, second session:
#  1. round 3's unexecuted opt-in paths: the AQL session (probe, syncbench,
#     its GPU test, config-1 A/B in C, persistent tests) and the pre-gather
#     A/B of the 512^3 halo;
#  2. kernel traces of the 1-rank 512^3 halo with the default lanes and with
#     TEMPI_STREAMS=1 (busy vs wall, tools/halo_trace_summary.py);
#  3. the 2-rank halo, Isend form vs neighbourhood form, with
#     TEMPI_PRINT_COUNTERS (the neighbourhood calls' post / wait split), next
#     to the small-message ping-pong latency.
# Stops at the first failing step.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out
mkdir -p $O
echo "== aql"
bash tools/gpu_aql_session.sh > $O/aql_session.log 2>&1
rc=$?; tail -n 30 $O/aql_session.log; [ $rc -eq 0 ] || exit $rc
echo "== pregather"
bash tools/gpu_pregather_ab.sh || exit 6
echo "== halo traces"
for lanes in default 1; do
  E="TEMPI_X=1"; [ $lanes = 1 ] && E="TEMPI_STREAMS=1"
  rm -rf $O/halo_trace_$lanes
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/halo_trace_$lanes \
    -- tempi_amd/lib/halo_exchange 10 512 > $O/halo_trace_$lanes.log 2>&1 || exit 7
  grep '^{' $O/halo_trace_$lanes.log
  python3 tools/halo_trace_summary.py $O/halo_trace_$lanes > $O/halo_trace_$lanes.txt || exit 8
  head -n 8 $O/halo_trace_$lanes.txt
done
echo "== 2-rank halo: Isend vs neighbourhood, counters"
: > $O/nbr_split.jsonl
for rep in 1 2; do
  for mode in "" "--neighbor"; do
    r=$(TEMPI_PRINT_COUNTERS=1 timeout -k 10 200 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/halo_exchange 10 512 $mode \
        2> $O/nbr_cnt.txt | grep '^{') || exit 9
    echo "{\"rep\": $rep, \"mode\": \"${mode:-isend}\", \"r\": $r}" >> $O/nbr_split.jsonl
    echo "mode=${mode:-isend} $(echo "$r" | grep -o '"us_per_iter": [0-9.]*')"
    grep '^\[tempi' $O/nbr_cnt.txt | sed "s/^/  /" | tee -a $O/nbr_split_counters.txt
  done
done
echo "== 2-rank ping-pong latency (small messages)"
: > $O/pingpong_small.jsonl
for total in 4096 65536 1048576; do
  timeout -k 10 100 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 300 $total 512 1024 > $O/pp.out 2>&1 || exit 10
  grep '^{' $O/pp.out >> $O/pingpong_small.jsonl
done
cut -c1-300 $O/pingpong_small.jsonl
