#!/bin/bash
# The driver's N=1 bench command, timed; line in gpurun_out/bench_n1.json,
# full record in gpurun_out/bench_detail_n1.json.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
t0=$(date +%s.%N)
timeout -k 10 600 python bench.py > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err || exit 5
t1=$(date +%s.%N)
# stdout must be exactly one line, the JSON line (the driver's contract)
python3 -c "import json,sys; ls=open('gpurun_out/bench_n1.json').read().strip().splitlines(); assert len(ls) == 1, f'{len(ls)} stdout lines'; l=ls[0]; d=json.loads(l); print('line bytes', len(l), 'wall_s', round($t1-$t0,1), 'value', d['value'], 'frac', d['roofline']['frac'], 'cpu', d.get('cpu_baseline'))"
