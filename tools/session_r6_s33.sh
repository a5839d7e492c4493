set -o pipefail
# after reverting the transport hook: the N = 8 rehearsal, the resident tests (4 processes included), halo at 2 / 8 ranks
: # (n8 passed in s33)
timeout -k 10 600 python -u -m pytest tests/test_resident_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/s33_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s33_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
for n in 2 8; do
  timeout -k 10 120 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>/dev/null | grep '^{' | cut -c1-150 || exit 3
done
