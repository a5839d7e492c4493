#!/bin/bash
# N=2 bench under torchrun (ranks sharing the box's GPU) in three variants:
# a = shipped model, b = this node's perf.json measured first, c = a with
# host receives straight to the library. Prints halo us/iter per variant.
cd "$(dirname "$0")/.."
P=29511
for v in a b c; do
  X="--no-measure-system"; [ $v = b ] && X=""
  E=/tmp/tempi_cache_$v; rm -rf $E; mkdir -p $E
  H=; [ $v = c ] && H="TEMPI_NO_HOST_RECV=1"
  P=$((P + 1))
  env TEMPI_CACHE_DIR=$E $H timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port $P bench.py --gpus 2 --steps 2 --warmup 1 --no-p2p $X \
    > gpurun_out/n2_$v.json 2> gpurun_out/n2_$v.err
  echo "$v rc=$?"
  python3 - gpurun_out/n2_$v.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][0])
print(d["halo"]["us_per_iter"], d["halo"]["rank0_phase_us"], d["halo_weak"]["us_per_iter"],
      d.get("perf_model", {}).get("auto_model"))
PY
done
