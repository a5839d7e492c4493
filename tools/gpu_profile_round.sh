#!/bin/bash
# The round's profile set on the final tree (no tests): rocprofv3 kernel-trace
# stats of bench.py's headline + FETCH_SIZE / WRITE_SIZE passes
# (tools/gpu_prof.sh), the halo at 1 / 2 / 4 ranks in both forms (Isend/Irecv
# and MPI_Neighbor_alltoallw), and the 1-rank halo's kernel trace.
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
echo "== rocprof"
bash tools/gpu_prof.sh || exit 7
echo "== halo"
rm -f $O/halo.jsonl
for n in 1 2 4; do
  for mode in "" "--neighbor"; do
    timeout -k 10 300 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 $mode >> $O/halo.jsonl 2>> $O/halo.err || exit 9
  done
done
python3 -c "
import json
for l in open('$O/halo.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); print(d['ranks'], d['api'], d['us_per_iter'])
"
echo "== halo-prof"
rm -rf $O/halo_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/halo_prof -o run -- tempi_amd/lib/halo_exchange 10 512 > $O/halo_prof.log 2>&1 || exit 12
echo done
