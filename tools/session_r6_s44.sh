set -o pipefail
# insurance on the built tree the driver will run (libraries rebuilt after
# s43's reverted experiment): full -m gpu suite in the driver's form, smoke()
cd "$(dirname "$0")/.."
bash tools/gpu_session.sh tests || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 3; }
tail -1 gpurun_out/smoke.log | cut -c1-120
