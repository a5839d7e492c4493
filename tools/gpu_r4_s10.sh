#!/bin/bash
# (The switch was removed after this A/B; rebuild from commit 376322d to repeat.)
# Halo A/B of the narrow strided-side load policy (tools/build_ab.sh
# "nt:-DTEMPI_NARROW_LD=1" "sc1:-DTEMPI_NARROW_LD=2", copied to
# tools/_variants/ld_<v>/libtempi_hip.so): 512^3, 10 iterations, content
# checked, at 2 and 4 ranks on the one GPU, three rounds with the order
# rotated, then 1 rank once each.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; : > $O/halo_ld2.jsonl
run() { # variant ranks round
  h=$(LD_LIBRARY_PATH=$PWD/tools/_variants/ld_$1 timeout -k 10 200 /opt/conda/bin/mpiexec -n $2 tempi_amd/lib/halo_exchange 10 512 --check 2>/dev/null | grep '^{') || exit 6
  echo "{\"variant\": \"$1\", \"round\": $3, \"ranks\": $2, \"r\": $h}" >> $O/halo_ld2.jsonl
  echo "$1 n=$2 r=$3 $(echo "$h" | grep -o '"us_per_iter": [0-9.]*')"
}
for n in 2 4; do
  r=0
  for order in "cur nt sc1" "nt sc1 cur" "sc1 cur nt"; do
    r=$((r + 1))
    for v in $order; do run $v $n $r; done
  done
done
for v in sc1 nt cur; do run $v 1 1; done
