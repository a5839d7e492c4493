set -o pipefail
# the driver's torchrun command on the final tree: N = 2 (resident packer on:
# two ranks per GPU) and N = 8 (packer off), ranks sharing this box's GPU
cd "$(dirname "$0")/.."
NS="2" bash tools/gpu_session.sh torchrun || exit $?
bash tools/gpu_session.sh n8 || exit $?
