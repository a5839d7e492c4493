set -o pipefail
# where the resident call's time goes, by variant
O=gpurun_out/resident_split.jsonl
rm -f $O
for r in 1 2; do
  for v in "P128" "P64:TEMPI_RESIDENT_WORKERS=64" "P32:TEMPI_RESIDENT_WORKERS=32" "P64_agent:TEMPI_RESIDENT_WORKERS=64 TEMPI_RESIDENT_ACQUIRE=agent"; do
    name=${v%%:*}; envs=""; [ "$v" != "$name" ] && envs=${v#*:}
    env $envs timeout -k 10 60 tools/bin/resident_split 1000 | sed "s/^{/{\"variant\": \"$name\", /" >> $O || exit 2
  done
done
cat $O
