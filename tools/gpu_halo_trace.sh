#!/bin/bash
# Kernel trace of the 512^3 halo (10 iterations) for busy/idle analysis
# (tools/halo_trace_summary.py): gpurun_out/halo_trace/. RANKS (default 1)
# processes, each under its own rocprofv3 (one trace file per process; the
# summary merges them: ranks sharing the box's GPU).
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
rm -rf gpurun_out/halo_trace
timeout -k 10 200 /opt/conda/bin/mpiexec -n ${RANKS:-1} rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/halo_trace -- tempi_amd/lib/halo_exchange 10 512 ${HALO_ARGS} > gpurun_out/halo_trace.log 2>&1 || exit 3
grep '^{' gpurun_out/halo_trace.log
