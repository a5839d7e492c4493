set -o pipefail
FOCUS="peel or probe_holds" HALO_AB="- TEMPI_COPY_PEEL=2 TEMPI_COPY_PEEL=0" HALO_ROUNDS=4 KOFF_OFFSETS=24 KOFF_ROUNDS=1 KOFF_SHAPES="4096:512:2386944:3:4608 4096:3:2386944:512:4608 4096:512:2386944:512:4608" LS_AB="- TEMPI_SYNC_UNROLL=2 TEMPI_SYNC_UNROLL=4" LS_ROUNDS=3 bash tools/gpu_session.sh focus ls-ab halo-ab koff || exit 1
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n1.jsonl && cp gpurun_out/koff.jsonl gpurun_out/koff_a.jsonl || exit 1
HALO_RANKS=2 HALO_AB="- TEMPI_COPY_PEEL=0" HALO_ROUNDS=3 HALO_ITERS=20 bash tools/gpu_session.sh halo-ab || exit 1
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n2.jsonl || exit 1
TEMPI_COPY_PEEL=2 KOFF_OFFSETS=24 KOFF_ROUNDS=1 KOFF_SHAPES="4096:512:2386944:3:4608 4096:3:2386944:512:4608 4096:512:2386944:512:4608" bash tools/gpu_session.sh koff || exit 1
bash tools/gpu_session.sh tests || exit 1
KPMC_SHAPES="4096:262144:4112 4096:233016:4608 512:2097152:1024" KPMC_PASSES="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum;TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum;TCC_HIT_sum TCC_MISS_sum" bash tools/gpu_session.sh kpmc
