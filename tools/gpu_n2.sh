#!/bin/bash
# N=2 bench through torchrun on the box's one GPU (ranks share it) + new app tests
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_p2p_gpu.py -k "alltoallv_sparse or pingpong" -x -q --timeout 200 --timeout-method thread > $O/n2_tests.log 2>&1
rc=$?; tail -3 $O/n2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 > $O/bench_n2.json 2> $O/bench_n2.err || exit 6
tail -c 3000 $O/bench_n2.json
