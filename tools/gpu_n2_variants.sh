#!/bin/bash
# The 2-rank halo under each launch mode on one box (tools/halo_variant.py),
# against the C app under mpiexec and bench.py's own torchrun line.
# Output: gpurun_out/n2_variants.jsonl (+ .err). Stops at the first failure.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O
OUT=$O/n2_variants.jsonl; : > $OUT
P=29700
tr() { P=$((P + 1)); timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
         --master-addr 127.0.0.1 --master-port $P "$@"; }
run() { echo "== $*"; "$@" 2>> $O/n2_variants.err | grep '^{' >> $OUT || exit 3; tail -n 1 $OUT; }
for rep in 1 2; do
  run timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/halo_exchange 10 512
  run tr tools/halo_variant.py --mode plain
  run tr tools/halo_variant.py --mode cuda
  run tr tools/halo_variant.py --mode headline
  run timeout -k 10 240 /opt/conda/bin/mpiexec -n 2 python tools/halo_variant.py --mode headline
done
echo "== bench torchrun N=2 (halo sections only)"
P=$((P + 1))
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port $P bench.py --gpus 2 --steps 3 --warmup 1 --no-p2p --no-measure-system > $O/n2_bench.json 2>> $O/n2_variants.err || exit 4
tail -c 1500 $O/n2_bench.json
