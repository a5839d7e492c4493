set -o pipefail
FOCUS="peeled" bash tools/gpu_session.sh focus || exit 1
TEMPI_FUZZ_CHUNKS=1000 timeout -k 10 600 python -u -m pytest tests/test_fuzz_parity.py -m gpu -x -q --timeout 500 --timeout-method thread > gpurun_out/fuzz50k_r6.log 2>&1
rc=$?; tail -3 gpurun_out/fuzz50k_r6.log; exit $rc
