set -o pipefail
FOCUS="copy or phase8" bash tools/gpu_session.sh focus || exit 1
HALO_AB="- TEMPI_COPY_PEEL=0 TEMPI_COPY_PEEL=2" HALO_ROUNDS=5 bash tools/gpu_session.sh halo-ab || exit 1
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n1.jsonl
HALO_RANKS=2 HALO_AB="- TEMPI_COPY_PEEL=0" HALO_ROUNDS=3 HALO_ITERS=20 bash tools/gpu_session.sh halo-ab || exit 1
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n2.jsonl
KBENCH_NO_COPY=1 KAB_DIR=tools/bin/v KAB_OUT=xcd_ab.jsonl KAB_ROUNDS=3 KAB_ITERS=20 KAB_SHAPES="4096:262144:4112" bash tools/gpu_session.sh kab
