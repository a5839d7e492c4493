#!/bin/bash
# stream lanes with a high-priority gather lane: halo at 1/2/4 ranks for
# TEMPI_STREAMS=1, 3, 3 without priority, 4; alternating, one box
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
rm -f $O/lanes3.txt
j() { python3 -c "import sys,json; r=json.loads([l for l in sys.stdin.read().splitlines() if l.startswith('{')][0]); print(r['us_per_iter'], r['us_min'], r.get('rank0_us_per_iter'))"; }
for rep in 1 2; do
  for v in s1 s3 s3np s4; do
    for n in 1 2 4; do
      E="TEMPI_STREAMS=${v:1:1}"; [ $v = s3np ] && E="$E TEMPI_NO_STREAM_PRIORITY=1"
      r=$(env $E timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 2>&1 | j) || exit 3
      echo "$v n=$n $r" | tee -a $O/lanes3.txt
    done
  done
done
