#!/bin/bash
# bench.py at N=1 (no PMC passes, no CPU baseline) and N=2 through torchrun
# on the box's one GPU (ranks share it)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline > $O/bench_n1.json 2> $O/bench_n1.err || exit 5
tail -c 1500 $O/bench_n1.json
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err || exit 6
python3 -c "import json; r=json.loads(open('$O/bench_n2.json').read().splitlines()[-1]); print(json.dumps({k: r.get(k) for k in ('value','halo','halo_weak')})[:3000])"
