#!/bin/bash
# bench.py at N=4 through torchrun on the box's one GPU (ranks share it)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 4 --steps 10 --warmup 2 > $O/bench_n4.json 2> $O/bench_n4.err || exit 6
python3 -c "import json; r=json.loads(open('$O/bench_n4.json').read().splitlines()[-1]); print(json.dumps({k: r.get(k) for k in ('value','n_gpus','halo','halo_weak')})[:3000]); print([ (p['total_bytes'] if 'total_bytes' in p else p.get('total'), p.get('us_oneway', p.get('oneway_us'))) for p in r['pingpong']['points']]); print([(p.get('scale'), p.get('min_us')) for p in r['alltoallv']['points']])"
