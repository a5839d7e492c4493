set -o pipefail
# final-tree check after the resident packer's bound/cleanup fix: full -m gpu
# suite in the driver's form, the driver's bench, smoke()
cd "$(dirname "$0")/.."
bash tools/gpu_session.sh tests bench || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -5 gpurun_out/smoke.log
