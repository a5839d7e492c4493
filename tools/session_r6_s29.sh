set -o pipefail
# the 8-rank halo on one GPU with the resident packer off / on / 32 workers: which one fails
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
for v in "off:TEMPI_RESIDENT=0" "on:TEMPI_RESIDENT=1" "w32:TEMPI_RESIDENT_WORKERS=32"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 120 /opt/conda/bin/mpiexec -n 8 tempi_amd/lib/halo_exchange 5 512 > gpurun_out/h8_$name.out 2> gpurun_out/h8_$name.err
  echo "$name rc=$?"; grep -h "^{" gpurun_out/h8_$name.out | cut -c1-200; grep -h "FATAL\|error" gpurun_out/h8_$name.err | head -3
done
