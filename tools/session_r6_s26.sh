set -o pipefail
# resident packer in blocking transport waits: transport tests, then the 2-rank ping-pong on / off
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
timeout -k 10 900 python -u -m pytest tests/test_resident_gpu.py tests/test_p2p_gpu.py tests/test_round3_gpu.py -m gpu -x -q \
  --timeout 250 --timeout-method thread > gpurun_out/s26_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s26_tests.log; [ $rc -eq 0 ] || exit $rc
O=gpurun_out/pingpong_resident_ab.jsonl
rm -f $O
for r in 1 2 3; do
  for on in 1 0; do
    for tb in "1024 8" "1024 256" "65536 64" "1048576 8" "1048576 512"; do
      set -- $tb
      TEMPI_RESIDENT=$on timeout -k 10 120 /opt/conda/bin/mpiexec -n 2 tempi_amd/lib/pingpong_nd 300 $1 $2 512 --check 2>/dev/null \
        | grep '^{' | sed "s/^{/{\"resident\": $on, \"round\": $r, /" >> $O || exit 3
    done
  done
done
python3 -c "
import json
for l in open('$O'):
    d=json.loads(l); print(d['round'], d['resident'], d.get('total'), d.get('block'), d.get('oneway_us'), d.get('errors'), d.get('method'))"
