#!/bin/bash
# Round 4, fourth session: the halo's x faces against
# their bare access pattern.
#  1. tools/xface.hip timed: paired / single / full-sector / reads-only
#     (build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o
#     tools/_variants/xface tools/xface.hip);
#  2. memory counters of those kernels, one rocprofv3 --pmc pass each;
#  3. the packer's own x-face copy (tools/_variants/hbench, HBENCH_ONLY=x_faces)
#     timed and under the same counter passes;
#  4. the 1-rank 512^3 halo, three runs (box spread).
# Stops at the first failing step.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out
mkdir -p $O
echo "== xface timed"
timeout -k 10 120 tools/_variants/xface 20 | tee $O/xface.jsonl || exit 3
echo "== hbench x faces timed"
HBENCH_ONLY=x_faces timeout -k 10 120 tools/_variants/hbench tempi_amd/lib/libtempi_hip.so 20 | tee $O/hbench_x.jsonl || exit 4
echo "== counters"
for c in FETCH_SIZE WRITE_SIZE "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  n=$(echo $c | cut -d' ' -f1)
  rm -rf $O/xf_$n $O/hb_$n
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/xf_$n -o run -- tools/_variants/xface 2 \
    > $O/xf_$n.log 2>&1 || exit 5
  HBENCH_ONLY=x_faces timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/hb_$n -o run -- \
    tools/_variants/hbench tempi_amd/lib/libtempi_hip.so 2 > $O/hb_$n.log 2>&1 || exit 6
done
python3 tools/pmc_kernels.py $O/xf_* $O/hb_* | tee $O/xface_pmc.txt
echo "== halo 1 rank x3"
: > $O/halo1_spread.jsonl
for rep in 1 2 3; do
  timeout -k 10 200 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/halo_exchange 10 512 > $O/halo1.out 2>&1 || exit 7
  grep '^{' $O/halo1.out | tee -a $O/halo1_spread.jsonl | cut -c1-160
done
