#!/bin/bash
# Retry a gpurun call ONLY when the infrastructure did not run it (transient
# box failure / back-off / no box free); a command that ran is never retried.
# usage: tools/gpurun_retry.sh TIMEOUT 'command'
T=$1; shift
for i in 1 2 3 4 5 6; do
  out=$(/usr/local/graft/bin/gpurun --timeout "$T" -- "$@" 2>&1)
  rc=$?
  if echo "$out" | grep -qE "status=transient|backing off|no box|slot free"; then
    echo "[retry $i] $(echo "$out" | grep -E 'status=|backing' | head -2)" >&2
    sleep 45
    continue
  fi
  echo "$out"
  exit $rc
done
echo "gave up after transient failures" >&2
exit 3
