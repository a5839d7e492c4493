set -o pipefail
# resident vs launched for 1- and 2-byte words (3 : 7 and 2 : 18 rows) by size, narrow limit lifted
O=gpurun_out/resident_narrow.jsonl
rm -f $O
for r in 1 2; do
  for shape in "3 7" "2 18"; do
    set -- $shape
    for bytes in 1024 16384 131072 262144 1048576; do
      rows=$((bytes / $1))
      TEMPI_RESIDENT_NARROW_MAX_BYTES=1073741824 timeout -k 10 60 tools/bin/resident_split tempi_amd/lib/libtempi_hip.so 300 $rows $1 $2 \
        | sed "s/^{/{\"round\": $r, /" >> $O || exit 2
    done
  done
done
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); print(d['round'], d['block'], d['stride'], d['rows']*d['block'], d['call_us'], d['back_to_back_call_us'], d['launched_call_us'], d['worker0_share_us'])"
