#!/bin/bash
# Synchronous small-call latency by chunks per lane for 16-byte words
# (tools/build_ab.sh "u2:-DTEMPI_UNROLL_16=2" "u4:-DTEMPI_UNROLL_16=4"):
# tools/syncbench at the C ABI, three alternations -> gpurun_out/sync_u.jsonl
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O; : > $O/sync_u.jsonl
for r in 1 2 3; do
  for v in cur u2 u4; do
    timeout -k 10 60 tools/_variants/syncbench tools/_variants/libtempi_hip_$v.so 1000 \
      | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/sync_u.jsonl || exit 3
  done
done
grep -o '"variant": "[a-z0-9]*", "round": [0-9], "shape": "[^"]*".*"ticket_fold_us": [0-9.]*' $O/sync_u.jsonl \
  | sed 's/"packed.*"ticket_fold_us"/ fold_us/' | grep "1024, 512\|256, 512\|(2, 512"
