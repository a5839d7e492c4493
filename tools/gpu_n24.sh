#!/bin/bash
# bench.py at N=2 then N=4 through torchrun on the box's one GPU (ranks share it),
# the driver's multi-rank launch line
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
for n in 2 4; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2952$n bench.py --gpus $n --steps 10 --warmup 2 > $O/bench_n$n.json 2> $O/bench_n$n.err || exit 6
  tail -c 400 $O/bench_n$n.json
done
