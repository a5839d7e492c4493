set -o pipefail
# the final tree's 1- and 2-rank 512^3 halo, 4 rotations each, with the
# resident packer on (default) and off: run-to-run spread on one box, and no
# effect of the packer on the transport
cd "$(dirname "$0")/.."
HALO_AB="- TEMPI_RESIDENT=0" HALO_ROUNDS=4 HALO_RANKS=1 bash tools/gpu_session.sh halo-ab || exit $?
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n1.jsonl
HALO_AB="- TEMPI_RESIDENT=0" HALO_ROUNDS=4 HALO_RANKS=2 bash tools/gpu_session.sh halo-ab || exit $?
cp gpurun_out/halo_ab.jsonl gpurun_out/halo_ab_n2.jsonl
