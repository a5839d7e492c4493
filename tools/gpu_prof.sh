#!/bin/bash
# rocprofv3 kernel-trace stats of bench.py's headline, then FETCH_SIZE and
# WRITE_SIZE in passes of their own
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/prof_trace $O/prof_FETCH_SIZE $O/prof_WRITE_SIZE
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_trace -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-traffic --no-halo --no-sweep-geomean --detail-name bench_detail_prof.json > $O/prof_trace.log 2>&1 || exit 7
tail -c 400 $O/prof_trace.log
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/prof_$c -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-traffic --no-halo --no-sweep-geomean --detail-name bench_detail_prof.json > $O/prof_$c.log 2>&1 || exit 8
done
