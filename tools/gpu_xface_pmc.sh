#!/bin/bash
# HBM traffic of the halo x-face kernels (pack / unpack / copy): kernel trace,
# then FETCH_SIZE and WRITE_SIZE in their own passes
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
export HBENCH_ONLY=${1:-x_faces}
L=tools/_variants/libtempi_hip_cur.so
rm -rf $O/xf_trace $O/xf_FETCH_SIZE $O/xf_WRITE_SIZE
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/xf_trace -o run -- tools/_variants/hbench $L 5 > $O/xf_trace.log 2>&1 || exit 2
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d $O/xf_$c -o run -- tools/_variants/hbench $L 5 > $O/xf_$c.log 2>&1 || exit 3
done
cat $O/xf_trace.log | grep '^{'
