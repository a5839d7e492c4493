set -o pipefail
# the resident packer with a high-priority stream, 200 us idle, off beyond 2 ranks per GPU
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
for v in "8:default:" "8:forced:TEMPI_RESIDENT=1" "2:default:" "2:off:TEMPI_RESIDENT=0" "4:default:" "4:forced:TEMPI_RESIDENT=1"; do
  n=${v%%:*}; rest=${v#*:}; name=${rest%%:*}; envs=${rest#*:}
  env $envs timeout -k 10 120 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 > gpurun_out/hq.out 2> gpurun_out/hq.err
  rc=$?
  echo "{\"ranks\": $n, \"resident\": \"$name\", \"rc\": $rc, \"us_per_iter\": $(grep -h '^{' gpurun_out/hq.out | python3 -c 'import json,sys; print(json.loads(sys.stdin.readline())["us_per_iter"])' 2>/dev/null || echo null)}" | tee -a gpurun_out/halo_resident_ranks.jsonl
  grep -h "FATAL" gpurun_out/hq.err | head -2
done
for on in 1 0; do
  TEMPI_RESIDENT=$on timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 300 1024 8 512 --check 2>/dev/null | grep '^{' | cut -c1-200
done
bash tools/gpu_session.sh n8 || exit 2
