set -o pipefail
# the GPU parity fuzz at 50 000 random types with the resident packer serving the small ones
TEMPI_FUZZ_CHUNKS=1000 timeout -k 10 900 python -u -m pytest tests/test_fuzz_parity.py -m gpu -x -q --timeout 500 --timeout-method thread -k "tempi_gpu" > gpurun_out/fuzz50k_resident.log 2>&1
rc=$?; tail -3 gpurun_out/fuzz50k_resident.log; exit $rc
