set -o pipefail
export KAB_DIR=tools/bin/v KBENCH_NO_COPY=1
KAB_OUT=phase_regs_ab.jsonl KAB_ROUNDS=3 KAB_ITERS=10 KAB_SHAPES="8:134217728:16 8:134217728:24 8:134217728:512 24:44739242:40 24:44739242:48 24:44739242:512 16:67108864:32" bash tools/gpu_session.sh kab || exit 1
KBENCH_OFFSET=24 KBENCH_POFF=8 KAB_OUT=phase_halo_ab.jsonl KAB_ROUNDS=3 KAB_ITERS=20 KAB_SHAPES="4096:512:2386944:3:4608 4096:3:2386944:512:4608 4096:512:2386944:512:4608" bash tools/gpu_session.sh kab || exit 1
unset KAB_DIR KBENCH_NO_COPY
HALO_RANKS=2 HALO_AB="- TEMPI_IPC_PHASE=0" HALO_ROUNDS=4 HALO_ITERS=20 bash tools/gpu_session.sh halo-ab || exit 1
FOCUS="phase8 or golden or misaligned or batched_kernel" bash tools/gpu_session.sh focus
