set -o pipefail
# resident packer against the launched path by object size (512-byte rows, stride 1 KiB), packer limit lifted
O=gpurun_out/resident_size.jsonl
rm -f $O
for r in 1 2; do
  for rows in 2 16 128 1024 2048 4096 8192 16384; do
    TEMPI_RESIDENT_MAX_BYTES=1073741824 timeout -k 10 60 tools/bin/resident_split tempi_amd/lib/libtempi_hip.so 500 $rows 512 1024 \
      | sed "s/^{/{\"round\": $r, /" >> $O || exit 2
  done
done
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); print(d['round'], d['rows']*512, d['call_us'], d['back_to_back_call_us'], d['launched_call_us'], d['acquire_us'], d['worker0_share_us'])"
