#!/bin/bash
# Copy-kernel A/B on one box: mixed-width launches (TEMPI_COPY_MIXED) against
# per-width launches over the halo regions (hbench), interleaved 3x; then the
# direct-copy GPU tests and the 1-rank halo with the shipped library.
# Variants (built on the CPU first): cur = tools/build_variants.sh; nomix = the same
# hipcc line with -DTEMPI_COPY_MIXED=0 on the mixed-launch build this A/B measured
# (reverted).
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/copy_ab.jsonl $O/halo_ab.jsonl
for rep in 1 2 3; do
  for v in cur nomix; do
    timeout -k 10 120 tools/_variants/hbench tools/_variants/libtempi_hip_$v.so 20 >> $O/copy_ab.jsonl || exit 5
  done
done
timeout -k 10 400 python -u -m pytest tests/test_direct_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/direct_tests.log 2>&1 || exit 6
tail -2 $O/direct_tests.log
for rep in 1 2; do
  timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 10 512 >> $O/halo_ab.jsonl 2>> $O/halo_ab.err || exit 7
done
