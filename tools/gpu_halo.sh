#!/bin/bash
# p2p tests + halo / pingpong measurements (method variants)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/halo2.jsonl
timeout -k 10 600 python -u -m pytest tests/test_p2p_gpu.py -q --maxfail=3 --timeout 300 --timeout-method thread > $O/p2p_tests.log 2>&1
rc=$?; tail -3 $O/p2p_tests.log; [ $rc -eq 0 ] || exit $rc
for m in AUTO TEMPI_DATATYPE_IPC TEMPI_DATATYPE_ONESHOT; do
  for n in 1 2 4; do
    echo "method=$m n=$n" >> $O/halo2.jsonl
    env $m=1 timeout -k 10 300 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 5 512 >> $O/halo2.jsonl 2>> $O/halo2.err || exit 9
  done
done
cat $O/halo2.jsonl | cut -c1-200
