#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -x -q --timeout 100 --timeout-method thread > $O/dense_tests.log 2>&1
rc=$?; tail -3 $O/dense_tests.log; [ $rc -eq 0 ] || exit $rc
SHAPES="1:268435456:2 2:134217728:4 3:89478485:7 4:67108864:8 1:134217728:8 3:44739242:24 5:53687091:13 7:38347922:50 12:22369621:40 24:512:2386944:512:4608 8:67108864:16"
rm -f $O/kbench_dense.jsonl
for v in cur nodense; do
  timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/kbench_dense.jsonl || exit 5
done
python3 -c "
import json
for l in open('$O/kbench_dense.jsonl'):
    r=json.loads(l); print(r['lib'].split('/')[-1], r['shape'], 'pack', round(r['pack_gbs']), 'unpack', round(r['unpack_gbs']))
"
