#!/bin/bash
# the folded ticket against the queued ticket kernel by
# grid size (1-256 workgroups), and HIP_FORCE_DEV_KERNARG=1 (kernel arguments
# in device memory), two alternations. gpurun_out/sync3.jsonl.
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O; OUT=$O/sync3.jsonl; : > $OUT
for r in 1 2; do
  for v in default nofold kernarg; do
    E="TEMPI_X=1"
    [ $v = nofold ] && E="TEMPI_FOLD_MAX_BLOCKS=0"
    [ $v = kernarg ] && E="HIP_FORCE_DEV_KERNARG=1"
    env $E timeout -k 10 60 tools/_variants/syncbench tempi_amd/lib/libtempi_hip.so 1000 \
      | sed "s/^{/{\"round\": $r, \"variant\": \"$v\", /" >> $OUT || exit 3
  done
done
echo "sync3 lines: $(wc -l < $OUT)"
