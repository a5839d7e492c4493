set -o pipefail
export TMPDIR=/tmp
O=gpurun_out; mkdir -p $O; rm -f $O/tl10*
TEMPI_TIMELINE=$O/tl10 timeout -k 10 200 tempi_amd/lib/halo_exchange 10 512 > $O/tl10.out 2>&1 || exit 1
grep '^{' $O/tl10.out | cut -c1-400
python3 tools/halo_timeline.py $O/tl10.r0.csv - > $O/tl10_timeline.txt 2>&1 || exit 2
tail -30 $O/tl10_timeline.txt
