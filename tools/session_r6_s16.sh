set -o pipefail
# resident packer: its tests, the ticket / golden tests beside it, then config 1 on / off
FOCUS="resident or synchronous_ticket or golden" bash tools/gpu_session.sh focus || exit 1
timeout -k 10 300 python -u tools/config1_ab.py 3 > gpurun_out/config1_ab.jsonl 2>&1 || exit 2
cat gpurun_out/config1_ab.jsonl
