#!/bin/bash
# Memory-counter calibration: tools/calib timed, then one
# rocprofv3 --pmc pass per counter group over the same binary. Results under
# gpurun_out/calib/; summarise with tools/calib_summary.py.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/calib
rm -rf $O; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/avail.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 300 tools/calib 10 > $O/time.jsonl || exit 4
echo "timed $(wc -l < $O/time.jsonl) cases"
pass() { # name counters...
  local n=$1; shift
  for c in "$@"; do
    grep -q "${c%_sum}" $O/avail.txt || { echo "skip $n: $c not listed"; return 0; }
  done
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $O/$n -o run -- tools/calib 1 > $O/$n.log 2>&1
  local rc=$?
  echo "pass $n rc=$rc"
  [ $rc -eq 0 ] || exit 5
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass rdreq TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
pass wrreq TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
echo done
