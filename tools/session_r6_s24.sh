set -o pipefail
# kernel trace of config 1 with the resident packer on: one server launch serves the calls
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
rm -rf gpurun_out/prof_c1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c1 -o c1 -- python3 tools/config1_ab.py 1 on > gpurun_out/prof_c1.log 2>&1 || exit 2
tail -2 gpurun_out/prof_c1.log
find gpurun_out/prof_c1 -name "*kernel_stats.csv" | head -3
for f in $(find gpurun_out/prof_c1 -name "*kernel_stats.csv"); do cut -d, -f1-8 $f | head -12; done
