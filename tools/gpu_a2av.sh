#!/bin/bash
# config 5 at 2 and 4 ranks sharing this box's one GPU: the bench.py points
# (scale 1e5 density 1 / 0.5, scale 1e3 density 1), content-checked once;
# A/B: IPC COPY at every size inside the collective (default) vs
# TEMPI_NO_COLL_COPY=1 (the point-to-point 128 KiB threshold)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
rm -f $O/a2av.jsonl
for n in 2 4; do
  timeout -k 10 120 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/alltoallv_sparse 5 --scale 1000 --check >> $O/a2av.jsonl 2>> $O/a2av.err || exit 3
  timeout -k 10 120 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/alltoallv_sparse 5 --scale 100000 --check >> $O/a2av.jsonl 2>> $O/a2av.err || exit 3
  for rep in 1 2; do
    for ab in "" TEMPI_NO_COLL_COPY=1; do
      for p in "100000 1.0" "100000 0.5" "1000 1.0" "10000 1.0"; do
        set -- $p
        echo "{\"ab\": \"$ab\"}" >> $O/a2av.jsonl
        env $ab TEMPI_X=1 timeout -k 10 120 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/alltoallv_sparse 20 --scale $1 --density $2 >> $O/a2av.jsonl 2>> $O/a2av.err || exit 4
      done
    done
  done
done
