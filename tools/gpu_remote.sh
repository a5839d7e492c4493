#!/bin/bash
# system-scope loads for IPC-mapped packed bytes: C-ABI batch tests (flag on
# and off), the p2p GPU tests, then the halo at 2 / 4 ranks with and without
# (TEMPI_IPC_PLAIN_LOADS) on one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_pack_gpu.py::test_batched_kernel_c_abi tests/test_p2p_gpu.py -x -q --timeout 120 --timeout-method thread > $O/remote_tests.log 2>&1
rc=$?; tail -3 $O/remote_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f $O/remote.txt
for rep in 1 2; do
  for v in sys plain; do
    for n in 2 4; do
      E=; [ $v = plain ] && E=TEMPI_IPC_PLAIN_LOADS=1
      r=$(env $E timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>&1 | grep '^{' | python3 -c "import sys,json; r=json.loads(sys.stdin.read()); print(r['us_per_iter'], r['us_min'])") || exit 3
      echo "$v n=$n $r" | tee -a $O/remote.txt
    done
  done
done
