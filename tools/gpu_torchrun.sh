#!/bin/bash
# The driver's multi-GPU bench command at N=2 and N=4 (ranks sharing this
# box's GPU): torchrun, every section of the line. JSON in gpurun_out/tr_N.json.
cd "$(dirname "$0")/.."
P=29611
for n in ${NS:-2 4}; do
  P=$((P + 1))
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $P bench.py --gpus $n --steps 5 --warmup 2 > gpurun_out/tr_$n.json 2> gpurun_out/tr_$n.err
  rc=$?
  echo "N=$n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python3 - gpurun_out/tr_$n.json <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
h = d["halo"]
pts = lambda k, c: [p[d[k]["cols"].index(c)] for p in d[k]["points"]]
print(d["value"], d["n_gpus"], h["us_per_iter"], h["rank0_phase_us"], d["halo_weak"]["us_per_iter"],
      pts("pingpong", "oneway_us"), pts("pingpong_1d", "oneway_us"), pts("alltoallv", "min_us"),
      pts("nbr_alltoallv", "min_us"), d.get("incomplete"), d["perf_model"].get("auto_model"))
PY
done
