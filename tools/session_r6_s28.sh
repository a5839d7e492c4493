set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_resident_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/s28_tests.log 2>&1
rc=$?; tail -4 gpurun_out/s28_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_session.sh n8 || exit 2
grep -i "fatal\|error" gpurun_out/tr_8.err | grep -v "socket.cpp" | head -5
