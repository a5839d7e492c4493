#!/bin/bash
# Where ten overlapping small device messages spend their time (the
# reference's bench_mpi_isend pattern, apps/mpi_isend): 2 ranks on the one
# GPU, 1 tag vs 10 tags, 1 B and 64 KiB, with TEMPI's host-phase counters,
# then one kernel trace of the 10-tag 1 B case.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; : > $O/isend_phases.txt
for tags in 1 10; do
  for b in 1 65536; do
    echo "== tags=$tags bytes=$b" >> $O/isend_phases.txt
    TEMPI_PRINT_COUNTERS=1 timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/mpi_isend 200 $b --tags $tags >> $O/isend_phases.txt 2>&1 || exit 3
  done
done
cat $O/isend_phases.txt
rm -rf $O/isend_trace
# (each rank under its own rocprofv3, as tools/gpu_halo_trace.sh: never a launcher after --)
timeout -k 10 180 /opt/conda/bin/mpiexec -n 2 rocprofv3 --kernel-trace --stats --output-format csv -d $O/isend_trace \
  -- tempi_amd/lib/mpi_isend 50 1 > $O/isend_trace.log 2>&1 || exit 4
find $O/isend_trace -name "*kernel_stats.csv" | head -3 | xargs -r cat | cut -c1-160
