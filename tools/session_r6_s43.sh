set -o pipefail
# window-compaction gather (TEMPI_PACK_WIN=1) for narrow rows beyond the dense
# window: byte-exact check of both builds, then kernel A/B, 3 rotations
cd "$(dirname "$0")/.."
for lib in tools/bin/v/libtempi_hip_cur.so tools/bin/v/libtempi_hip_win.so; do
  timeout -k 10 120 tools/bin/wincheck $lib || exit 2
done
KAB_DIR=tools/bin/v bash tools/kab.sh pack_win_ab.jsonl 3 20 \
  2:134217728:18 2:11585:208584:11585:18 3:89478485:19 3:9459:179778:9459:19 4:67108864:20 \
  1:268435456:17 5:53687091:33 || exit $?
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open('gpurun_out/pack_win_ab.jsonl'):
    r = json.loads(l); d[(r['shape'], r['variant'])].append(r['pack_gbs'])
for k in sorted(d): print(k, ' '.join('%.0f' % x for x in d[k]))
PY
