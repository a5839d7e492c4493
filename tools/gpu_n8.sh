#!/bin/bash
# The driver's 8-GPU bench command shape, rehearsed with 8 ranks sharing this
# box's one GPU: torchrun --nproc-per-node 8 bench.py
# --gpus 8 with the default steps / warmup. Prints the wall time, the line's
# size and whether it parses; line in gpurun_out/tr_8.json, full record in
# gpurun_out/bench_detail_n8.json, stderr in gpurun_out/tr_8.err.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O
N=${N:-8}
t0=$(date +%s.%N)
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
  --master-port 29733 bench.py --gpus $N > $O/tr_$N.json 2> $O/tr_$N.err
rc=$?
t1=$(date +%s.%N)
echo "N=$N rc=$rc wall_s=$(python3 -c "print(round($t1-$t0,1))")"
[ $rc -eq 0 ] || exit $rc
python3 - $O/tr_$N.json <<'PY'
import json, sys
lines = [l for l in open(sys.argv[1]) if l.strip()]
assert len(lines) == 1 and lines[0].startswith("{"), f"stdout holds {len(lines)} lines besides the bench line"
l = lines[-1].strip()
d = json.loads(l)
print("line bytes", len(l), "value", d["value"], "ms_per_step", d["ms_per_step"], "incomplete", d.get("incomplete"),
      "dropped", d.get("dropped"))
print("halo", d.get("halo"))
print("alltoallv", d.get("alltoallv"))
print("transport", d.get("transport"))
PY
