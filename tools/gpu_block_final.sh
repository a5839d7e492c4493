#!/bin/bash
# The 128-lane packer build: GPU suite, A/B against the 256 build (bs256) on one
# box, bench.py, 1-rank halo.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=3 --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f $O/block_final_ab.jsonl
SHAPES="512:2097152:1024 4096:262144:4160 64:16777216:128 8:67108864:16 24:512:2386944:512:4608 1:268435456:2 1:134217728:8"
for rep in 1 2; do
  for v in cur bs256; do
    timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/block_final_ab.jsonl || exit 5
    timeout -k 10 120 tools/_variants/hbench tools/_variants/libtempi_hip_$v.so 20 >> $O/block_final_ab.jsonl || exit 6
  done
done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 7
tail -c 300 $O/bench.json
rm -f $O/halo1.jsonl
timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 10 512 >> $O/halo1.jsonl 2>> $O/halo1.err || exit 8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 9
tail -1 $O/smoke.log
