set -o pipefail
KBENCH_NO_COPY=1 KOFF_OFFSETS="0 16 32" KOFF_ROUNDS=2 KOFF_SHAPES="4096:233016:4608 4096:262144:4112" bash tools/gpu_session.sh koff || exit 1
cp gpurun_out/koff.jsonl gpurun_out/koff_rowphase.jsonl
for v in 1 0 1 0; do
  TEMPI_COPY_PEEL=$v KBENCH_POFF=24 KOFF_OFFSETS=24 KOFF_ROUNDS=1 KOFF_SHAPES="4096:1536:4608 4096:6144:4608 4096:24576:4608 4096:98304:4608" bash tools/gpu_session.sh koff || exit 1
  sed "s/^{/{\"peel\": $v, /" gpurun_out/koff.jsonl >> gpurun_out/koff_peelsize.jsonl
done
HALO_AB="- TEMPI_COPY_PEEL=0" HALO_ROUNDS=6 bash tools/gpu_session.sh halo-ab || exit 1
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n1.jsonl
HALO_RANKS=2 HALO_AB="- TEMPI_COPY_PEEL=0 TEMPI_PEEL_REMOTE=0" HALO_ROUNDS=4 HALO_ITERS=20 bash tools/gpu_session.sh halo-ab || exit 1
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n2.jsonl
