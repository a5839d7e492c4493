#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
SHAPES="1:268435456:2 1:134217728:8 3:44739242:24 7:38347922:50 2:67108864:16 4:67108864:16 12:22369621:40 8:67108864:16 8:33554432:64 24:512:2386944:512:4608 40:26843545:48"
rm -f $O/kbench_il.jsonl
for v in cur uil4 uil8 pil2 pil8; do
  timeout -k 10 120 tools/_variants/kbench tools/_variants/libtempi_hip_$v.so 10 $SHAPES >> $O/kbench_il.jsonl || exit 5
done
python3 -c "
import json
for l in open('$O/kbench_il.jsonl'):
    r=json.loads(l); print(r['lib'].split('/')[-1], r['shape'], 'pack', round(r['pack_gbs']), 'unpack', round(r['unpack_gbs']))
"
