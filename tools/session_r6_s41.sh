set -o pipefail
# final tree: full -m gpu suite in the driver's form, the GPU parity fuzz at
# 50 000 random types (resident packer serving the small objects), the
# driver's bench, smoke(), then rocprofv3 stats + FETCH / WRITE passes of the headline
cd "$(dirname "$0")/.."
bash tools/gpu_session.sh tests || exit $?
TEMPI_FUZZ_CHUNKS=1000 timeout -k 10 900 python -u -m pytest tests/test_fuzz_parity.py -m gpu -x -q --timeout 500 \
  --timeout-method thread -k "tempi_gpu" > gpurun_out/fuzz50k.log 2>&1 || { tail -20 gpurun_out/fuzz50k.log; exit 4; }
tail -1 gpurun_out/fuzz50k.log
bash tools/gpu_session.sh bench || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log | cut -c1-200
bash tools/gpu_session.sh prof || exit $?
