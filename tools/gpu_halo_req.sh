#!/bin/bash
# Memory-side request counts of the 1-rank 512^3 halo's copy kernels (the
# calibration's counters, tools/calib.sh): TCC_EA0_RDREQ / _RDREQ_32B and
# TCC_EA0_WRREQ / _WRREQ_64B, one rocprofv3 --pmc pass per pair, over
# halo_exchange 3 512 (1 warm-up + 3 iterations). gpurun_out/halo_req/.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out/halo_req
rm -rf $O; mkdir -p $O
for pair in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  n=$(echo $pair | cut -d' ' -f1)
  timeout -s KILL 180 rocprofv3 --pmc $pair --output-format csv -d $O/$n -o run -- \
    tempi_amd/lib/halo_exchange 3 512 > $O/$n.log 2>&1 || exit 5
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
n = collections.defaultdict(int)
for f in glob.glob("gpurun_out/halo_req/**/*counter_collection*.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "copy" in row.get("Kernel_Name", ""):
            tot[row["Counter_Name"]] += float(row["Counter_Value"])
            n[row["Counter_Name"]] += 1
iters = 4  # warm-up + 3
for k in sorted(tot):
    print(f"{k:24s} {tot[k] / iters:14.0f} per iteration ({n[k]} dispatch records)")
PY
