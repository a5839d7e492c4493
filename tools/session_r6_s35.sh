set -o pipefail
# resident packer: 2 vs 4 host-link polls in flight, config 1 object, alternated
O=gpurun_out/resident_polls_ab.jsonl
rm -f $O
for r in 1 2 3 4; do
  for lib in tools/bin/v/libtempi_hip_cur.so tools/bin/v/libtempi_hip_polls4.so; do
    v=$(basename $lib .so); v=${v#libtempi_hip_}
    timeout -k 10 60 tools/bin/resident_split $lib 2000 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O || exit 2
  done
done
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); print(d['variant'], d['round'], d['call_us'], d['back_to_back_call_us'], d['launched_call_us'])"
