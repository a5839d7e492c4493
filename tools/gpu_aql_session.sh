#!/bin/bash
# The AQL dispatch path (hip/aql.hpp, TEMPI_AQL=1): first the bare probe
# (tools/aqlbench.hip: HIP launch vs a hand-written packet, one workgroup),
# then its GPU test (every result checked against torch's view), then BASELINE
# config 1 and the 1 KiB object through MPI_Pack in C (apps/mpi_pack --shape,
# pinned core) with TEMPI_AQL off / on, three alternations, then the
# persistent-request GPU tests. gpurun_out/aql.jsonl, aql_ab.jsonl.
cd "$(dirname "$0")/.."
export TMPDIR=/tmp HYDRA_LAUNCHER=fork
O=gpurun_out; mkdir -p $O; : > $O/aql_sync.jsonl
echo "== probe"
timeout -k 10 90 tools/_variants/aqlbench tools/_variants/aqlbench.hsaco 2000 > $O/aql.jsonl 2> $O/aql.err
rc=$?; cat $O/aql.err $O/aql.jsonl; [ $rc -eq 0 ] || exit $rc
echo "== syncbench (C ABI): HIP launches vs TEMPI_AQL=1"
for v in hip aql aqldev; do
  E="TEMPI_X=1"; [ $v = aql ] && E="TEMPI_AQL=1"; [ $v = aqldev ] && E="TEMPI_AQL=1 TEMPI_AQL_DEVICE_KERNARG=1"
  env $E timeout -k 10 60 tools/_variants/syncbench tempi_amd/lib/libtempi_hip.so 2000 \
    | sed "s/^{/{\"variant\": \"$v\", /" >> $O/aql_sync.jsonl || exit 5
done
grep -o '"variant": "[a-z]*", "shape": "[^"]*".*"ticket_fold_us": [0-9.]*' $O/aql_sync.jsonl | sed 's/"packed.*"ticket_fold_us"/ fold_us/'
echo "== aql test"
TEMPI_TEST_AQL=1 timeout -k 10 300 python -u -m pytest tests/test_round3_gpu.py -q -x --timeout 200 --timeout-method thread -k aql \
  > $O/aql_test.log 2>&1
rc=$?; tail -n 5 $O/aql_test.log; [ $rc -eq 0 ] || exit $rc
echo "== config 1 A/B"
OUT=$O/aql_ab.jsonl; : > $OUT
for r in 1 2 3; do
  for v in hip aql aqldev; do
    E="TEMPI_X=1"; [ $v = aql ] && E="TEMPI_AQL=1"; [ $v = aqldev ] && E="TEMPI_AQL=1 TEMPI_AQL_DEVICE_KERNARG=1"
    env $E TEMPI_PRINT_COUNTERS=1 timeout -k 10 60 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/mpi_pack 1000 --shape 1024:512:1024 --pin \
      2>> $O/aql_ab.err | sed "s/^{/{\"round\": $r, \"bench\": \"config1\", \"variant\": \"$v\", /" >> $OUT || exit 4
    env $E timeout -k 10 60 /opt/conda/bin/mpiexec -n 1 tempi_amd/lib/mpi_pack 1000 --shape 2:512:1024 --pin \
      2>> $O/aql_ab.err | sed "s/^{/{\"round\": $r, \"bench\": \"1KiB\", \"variant\": \"$v\", /" >> $OUT || exit 4
  done
done
grep -o '"bench": "[^"]*", "variant": "[^"]*".*"pack_us": [0-9.]*, "unpack_us": [0-9.]*' $OUT | sed 's/"target.*"pack_us"/ pack_us/'
echo "== persistent tests"
timeout -k 10 400 python -u -m pytest tests -m gpu -q -x --timeout 200 --timeout-method thread -k persistent \
  > $O/persistent_test.log 2>&1
rc=$?; tail -n 5 $O/persistent_test.log; exit $rc
