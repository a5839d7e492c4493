set -o pipefail
# resident packer variants on config 1: workers 64 / 128 / 256, acquire at agent / system scope
O=gpurun_out/config1_variants.jsonl
rm -f $O
for r in 1 2; do
  for v in "P128_sys" "P128_agent:TEMPI_RESIDENT_ACQUIRE=agent" "P64_sys:TEMPI_RESIDENT_WORKERS=64" "P96_sys:TEMPI_RESIDENT_WORKERS=96" \
           "P64_agent:TEMPI_RESIDENT_WORKERS=64 TEMPI_RESIDENT_ACQUIRE=agent"; do
    name=${v%%:*}; envs=""; [ "$v" != "$name" ] && envs=${v#*:}
    env VARIANT=$name $envs timeout -k 10 120 python -u tools/config1_ab.py 1 on >> $O 2>&1 || exit 2
  done
done
grep '^{' $O | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); p=d['c_phases']
    print(d['variant'], d['gpu_us'], p['mpi_pack_device_us'], p['phases_us']['resident_call'], p['phases_us']['resident_served'], p['mpich_host_us'])"
