#!/bin/bash
# coherent (new) vs coarse-grained (old) pinned slabs: ONESHOT / STAGED
# ping-pong one-way times, alternating builds on one box, then the p2p tests
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/pinned_ab.jsonl
for rep in 1 2; do
  for v in old new; do
    if [ $v = old ]; then LP=$PWD/tools/_variants/old; else LP=; fi
    for m in TEMPI_DATATYPE_ONESHOT TEMPI_DATATYPE_STAGED; do
      for tb in "1024 8" "1048576 8" "1048576 512" "4194304 512" "4194304 64"; do
        set -- $tb
        echo "{\"build\": \"$v\", \"m\": \"$m\"}" >> $O/pinned_ab.jsonl
        env $m=1 LD_LIBRARY_PATH=$LP timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 100 $1 $2 >> $O/pinned_ab.jsonl 2>> $O/pinned_ab.err || exit 4
      done
    done
  done
done
timeout -k 10 900 python -u -m pytest tests/test_p2p_gpu.py tests/test_pack_gpu.py -q --timeout 200 --timeout-method thread > $O/pinned_tests.log 2>&1
rc=$?; tail -2 $O/pinned_tests.log; exit $rc
