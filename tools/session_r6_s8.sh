set -o pipefail
bash tools/gpu_session.sh n8 || exit 1
cp gpurun_out/tr_8.json gpurun_out/tr_8_s8.json
bash tools/gpu_session.sh tests || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -3 gpurun_out/smoke.log
