set -o pipefail
# (1) the resident packer's hand-off slot waits for every worker, and the
# leader polls once more before an idle exit: its GPU tests; (2) config 1's
# call time against the tree before (HEAD), 4 rotations; (3) kernel A/B: packs
# of 2-, 4-, 8-byte words through the interleaved gather (today 1-byte only)
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
KAB_DIR=tools/bin/pil bash tools/kab.sh pack_il_widths_ab.jsonl 3 20 \
  2:134217728:18 2:11585:208584:11585:18 2:134217728:512 4:67108864:20 4:67108864:8 4:67108864:512 \
  8:33554432:24 8:33554432:512 || exit $?
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/pack_il_widths_ab.jsonl'):
    r = json.loads(l); d[(r['shape'], r['variant'])].append(r['pack_gbs'])
for k in sorted(d): print(k, ' '.join('%.0f' % x for x in d[k]))
PY
