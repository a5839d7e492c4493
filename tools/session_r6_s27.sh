set -o pipefail
bash tools/gpu_session.sh tests bench n8 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -c 400 gpurun_out/smoke.log
