#!/bin/bash
# why the torchrun-launched 2-rank halo is bimodal.
# bench.py at N > 1 measures this node's perf.json (measure_system --quick)
# BEFORE its halo, and AUTO then picks each message's method from that model;
# the mpiexec-launched app ran without one. So the same halo under each
# launcher, without a perf.json and then with the one bench.py would measure,
# with the methods each run chose (TEMPI_PRINT_COUNTERS: ipc / oneshot /
# staged), plus bench.py's own torchrun line. Output: gpurun_out/n2_variants.jsonl,
# n2_counters.txt, n2_perf.json. Stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork TEMPI_PRINT_COUNTERS=1
O=gpurun_out; mkdir -p $O
OUT=$O/n2_variants.jsonl; : > $OUT; : > $O/n2_counters.txt
PERF=$HOME/.tempi/perf.json
P=29700
trun() { P=$((P + 1)); timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
         --master-addr 127.0.0.1 --master-port $P "$@"; }
run() { # label cmd...
  local label=$1; shift
  echo "== $label"
  "$@" > $O/n2_run.out 2> $O/n2_run.err || { tail -5 $O/n2_run.err; exit 3; }
  grep '^{' $O/n2_run.out | tail -1 | sed "s/^{/{\"label\": \"$label\", /" >> $OUT
  echo "$label: $(grep -h '\[tempi r' $O/n2_run.err | paste -sd ' ')" >> $O/n2_counters.txt
  tail -n 1 $OUT | cut -c1-300
}
rm -f $PERF
for rep in $(seq ${REPS:-2}); do
  run "mpiexec-app-nomodel" timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/halo_exchange 10 512
  run "torchrun-plain-nomodel" trun tools/halo_variant.py --mode plain
  [ -n "$SHORT" ] || run "torchrun-headline-nomodel" trun tools/halo_variant.py --mode headline
done
mkdir -p $(dirname $PERF)
echo "== measure_system --quick (as bench.py does at N > 1)"
timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/measure_system --quick --out $PERF > $O/n2_measure.log 2>&1 || exit 5
cp $PERF $O/n2_perf.json
for rep in $(seq ${REPS:-2}); do
  run "mpiexec-app-model" timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/halo_exchange 10 512
  run "torchrun-plain-model" trun tools/halo_variant.py --mode plain
done
echo "== bench torchrun N=2 (halo sections only, with the model)"
P=$((P + 1))
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port $P bench.py --gpus 2 --steps 3 --warmup 1 --no-p2p > $O/n2_bench.json 2> $O/n2_bench.err || exit 4
tail -c 1500 $O/n2_bench.json
grep -h '\[tempi r' $O/n2_bench.err | sed 's/^/bench: /' >> $O/n2_counters.txt
rm -f $PERF
