#!/bin/bash
# HBM bytes touched per pack / unpack launch for the kbench shapes: one
# rocprofv3 --pmc pass per counter and shape (FETCH_SIZE, WRITE_SIZE apart)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/kpmc
rm -rf $O
mkdir -p $O
export TMPDIR=/tmp
L=tools/_variants/libtempi_hip_cur.so
SHAPES="512:2097152:1024 4096:262144:4160 64:16777216:128 8:67108864:16 24:512:2386944:512:4608 1:268435456:2 3:89478485:7 2:134217728:4 1:134217728:8 4:67108864:16"
i=0
for sh in $SHAPES; do
  i=$((i+1))
  timeout -k 10 60 tools/_variants/kbench $L 3 $sh > $O/k$i.json 2>&1 || exit 2
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/p${i}_$c -o run -- tools/_variants/kbench $L 3 $sh > $O/p${i}_$c.log 2>&1 || exit 3
  done
done
python3 tools/kbench_pmc_summary.py $O > $O/summary.txt && cat $O/summary.txt
