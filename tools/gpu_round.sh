#!/bin/bash
# One GPU session: GPU tests, the bench line, rocprof (kernel trace + the
# FETCH_SIZE / WRITE_SIZE passes, tools/gpu_prof.sh), the halo at 1/2/4 ranks
# (Isend/Irecv and neighbourhood collective) and its rocprof kernel trace.
# Every GPU step has its own time limit; the script stops at the first failure.
# (Round 1's one-off A/B scripts are retired: their results stay under
# profiles/r01/; tools/build_ab.sh + tools/kab.sh and tools/gpu_halo_ab.sh
# reproduce kernel and halo A/Bs.)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
step() { echo "== $*"; }
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 250 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -n 3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
step bench
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || exit 6
tail -c 400 $O/bench.json
step rocprof
bash tools/gpu_prof.sh || exit 7
step halo
rm -f $O/halo.jsonl
for n in 1 2 4; do
  for mode in "" "--neighbor"; do
    timeout -k 10 300 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 $mode >> $O/halo.jsonl 2>> $O/halo.err || exit 9
  done
done
step halo-prof
rm -rf $O/halo_prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/halo_prof -o run -- tempi_amd/lib/halo_exchange 10 512 > $O/halo_prof.log 2>&1 || exit 12
step done
