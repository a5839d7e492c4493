#!/bin/bash
# Variance of the 1-rank 512^3 halo on one box: standalone runs and the
# bench's in-process halo with and without the sweep before it.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out/halo_var.txt
: > $O
for i in 1 2 3; do
  r=$(timeout -k 10 120 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 10 512 | grep '^{') || exit 3
  echo "standalone $(echo "$r" | grep -o '"us_per_iter": [0-9.]*') $(echo "$r" | grep -o '"rank0_us_per_iter": {[^}]*}')" | tee -a $O
done
for flags in "--no-sweep-geomean" "" "--no-sweep-geomean"; do
  timeout -k 10 300 python bench.py --no-traffic --no-cpu-baseline $flags > gpurun_out/hv.json 2>/dev/null || exit 4
  python -c "import json; r=json.loads(open('gpurun_out/hv.json').read().splitlines()[-1]); h=r['halo']; print('bench [$flags]', h['us_per_iter'], h['rank0_phase_us'])" | tee -a $O
done
