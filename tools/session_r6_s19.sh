set -o pipefail
# resident packer: lanes' chunks in flight (TEMPI_RESIDENT_U 1 / 2 / 4) x workers 64 / 128, alternated on one box
O=gpurun_out/resident_u_ab.jsonl
rm -f $O
for r in 1 2 3; do
  for lib in tools/bin/v/libtempi_hip_u2.so tools/bin/v/libtempi_hip_u2flat.so tools/bin/v/libtempi_hip_u1flat.so; do
    for p in 96 128; do
      v=$(basename $lib .so); v=${v#libtempi_hip_}
      TEMPI_RESIDENT_WORKERS=$p timeout -k 10 60 tools/bin/resident_split $lib 1000 \
        | sed "s/^{/{\"variant\": \"${v}_P$p\", \"round\": $r, /" >> $O || exit 2
    done
  done
done
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); print(d['variant'], d['round'], d['call_us'], d['back_to_back_call_us'], d['acquire_us'], d['worker0_share_us'])"
timeout -k 10 60 tools/bin/vram_probe 2000 > gpurun_out/vram_probe.jsonl 2>&1; cat gpurun_out/vram_probe.jsonl
