set -o pipefail
# a fresh resident server waits >= 100 us for its first record: the resident
# tests, then config 1's call split on the in-tree library
cd "$(dirname "$0")/.."
FOCUS="resident" bash tools/gpu_session.sh focus || exit $?
timeout -k 10 60 tools/bin/resident_split tempi_amd/lib/libtempi_hip.so 2000 > gpurun_out/resident_split_s40.jsonl || exit 2
cat gpurun_out/resident_split_s40.jsonl
