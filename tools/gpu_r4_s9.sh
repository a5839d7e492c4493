#!/bin/bash
# (The build switch was removed after this A/B; rebuild from commit 376322d to repeat.)
# Round 4: can a load's cache policy cut the isolated 24-byte rows' fetch?
# (1) tools/xface.hip bare pattern by load policy, two rounds, then FETCH_SIZE /
#     WRITE_SIZE passes; (2) hbench (the halo's regions as the transport
#     batches them) and (3) the 1- and 2-rank 512^3 halo, each for the builds
#     tools/build_ab.sh "nt:-DTEMPI_NARROW_LD=1" "sc1:-DTEMPI_NARROW_LD=2"
#     (copied to tools/_variants/ld_<v>/libtempi_hip.so), alternating.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; : > $O/xface_pol.jsonl
echo "== smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 2; }
tail -2 $O/smoke.log
for r in 1 2; do
  timeout -k 10 120 tools/_variants/xface 20 | sed "s/^{/{\"round\": $r, /" >> $O/xface_pol.jsonl || exit 3
done
grep -o '"round": [0-9], .*"variant": "[a-z0-9_]*".*"us": [0-9.]*' $O/xface_pol.jsonl | sed 's/"rows.*"us"/us/'
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf $O/xpol_$c
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O/xpol_$c -o run -- tools/_variants/xface 5 > $O/xpol_$c.log 2>&1 || exit 4
done
python3 tools/pmc_kernels.py $O/xpol_FETCH_SIZE $O/xpol_WRITE_SIZE > $O/xface_pol_pmc.txt 2>&1; cat $O/xface_pol_pmc.txt
: > $O/hbench_ld.jsonl
for r in 1 2; do
  for v in cur nt sc1; do
    timeout -k 10 120 tools/_variants/hbench tools/_variants/libtempi_hip_$v.so 10 | sed "s/^{/{\"variant\": \"$v\", \"round\": $r, /" >> $O/hbench_ld.jsonl || exit 5
  done
done
grep -o '"variant": "[a-z0-9]*", "round": [0-9].*' $O/hbench_ld.jsonl | cut -c1-220
: > $O/halo_ld.jsonl
for r in 1 2; do
  for n in 1 2; do
    for v in cur nt sc1; do
      h=$(LD_LIBRARY_PATH=$PWD/tools/_variants/ld_$v timeout -k 10 200 /opt/conda/bin/mpiexec -n $n tempi_amd/lib/halo_exchange 10 512 --check 2>/dev/null | grep '^{') || exit 6
      echo "{\"variant\": \"$v\", \"round\": $r, \"ranks\": $n, \"r\": $h}" >> $O/halo_ld.jsonl
      echo "$v n=$n $(echo "$h" | grep -o '"us_per_iter": [0-9.]*') $(echo "$h" | grep -o '"errors": [0-9]*')"
    done
  done
done
