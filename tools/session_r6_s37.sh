set -o pipefail
# the resident packer's hand-off slot is overwritten only once every worker
# has read it: its GPU tests (four processes time-slicing one GPU included),
# then config 1's call time against the tree before (HEAD), 4 rotations
cd "$(dirname "$0")/.."
FOCUS="resident" bash tools/gpu_session.sh focus || exit $?
O=gpurun_out/resident_seen_ab.jsonl
rm -f $O
for r in 1 2 3 4; do
  for lib in tools/bin/v/libtempi_hip_HEAD.so tools/bin/v/libtempi_hip_cur.so; do
    v=$(basename $lib .so); v=${v#libtempi_hip_}
    timeout -k 10 60 tools/bin/resident_split $lib 2000 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O || exit 2
  done
done
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); print(d['variant'], d['round'], d['call_us'], d['back_to_back_call_us'], d['launched_call_us'])"
