set -o pipefail
FOCUS="xcd_mapped or full_size or phase8 or copy" bash tools/gpu_session.sh focus || exit 1
bash tools/gpu_session.sh bench prof n8 || exit 1
