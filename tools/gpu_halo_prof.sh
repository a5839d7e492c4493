#!/bin/bash
# 1-rank halo exchange under rocprofv3 kernel trace (singleton MPI, no mpiexec
# between the profiler and the program)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
rm -rf $O/halo_prof
timeout -k 10 120 tempi_amd/lib/halo_exchange 5 512 --check > $O/halo_check.json 2>&1 || exit 3
cat $O/halo_check.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/halo_prof -o run -- tempi_amd/lib/halo_exchange 10 512 > $O/halo_prof.log 2>&1 || exit 4
tail -2 $O/halo_prof.log
