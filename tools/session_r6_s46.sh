set -o pipefail
# the resident tests with the exit race's relaxed served count
cd "$(dirname "$0")/.."
FOCUS="resident" bash tools/gpu_session.sh focus || exit $?
