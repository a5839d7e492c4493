#!/bin/bash
# Host-side ThreadSanitizer pass (CPU only, no GPU) over MPI_THREAD_MULTIPLE:
# libtempi.so's C++ rebuilt with gcc -fsanitize=thread into build/tsan/, and
# tools/tsan_threads.cpp (threads waiting on each other's messages through
# TEMPI, no application lock) linked against it, run at 1 and 2 ranks with
# TEMPI's host-side paths forced on. Prints each run's result line and the
# number of TSan reports whose stack names a TEMPI frame (tempi::);
# reports entirely inside MPICH (not instrumented) are counted apart. A
# negative control runs the same program with TEMPI_FAULT_NO_MT_LOCK=1 (MULTIPLE
# reported, TEMPI's lock left off): TSan must report races in TEMPI there.
set -e
cd "$(dirname "$0")/.."
ROOT=$PWD
T=build/tsan
mkdir -p $T
for f in tempi_amd/csrc/core/*.cpp; do
  g++ -std=c++17 -O1 -g -fPIC -fvisibility=hidden -fsanitize=thread -Iinclude -I/opt/conda/include \
    -c $f -o $T/$(basename $f .cpp).o &
done
wait
g++ -shared -fsanitize=thread -o $T/libtempi.so $T/*.o -Ltempi_amd/lib -ltempi_hip /opt/conda/lib/libmpi.so \
  -ldl -lpthread -Wl,-rpath,$ROOT/tempi_amd/lib -Wl,-rpath,/opt/conda/lib -Wl,--enable-new-dtags
g++ -std=c++17 -O1 -g -fsanitize=thread -Iinclude -I/opt/conda/include -o $T/tsan_threads tools/tsan_threads.cpp \
  -L$T -ltempi /opt/conda/lib/libmpi.so -lpthread -Wl,-rpath,/usr/lib/x86_64-linux-gnu -Wl,-rpath,$ROOT/$T -Wl,-rpath,$ROOT/tempi_amd/lib \
  -Wl,-rpath,/opt/conda/lib -Wl,--enable-new-dtags
set +e
rc=0
run() { # name ranks [env]; sets R (rc) and N (TSan reports)
  TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 log_path=$ROOT/$T/report_$1" TEMPI_TEST_HOST_ONLY=1 \
    HYDRA_LAUNCHER=fork env $3 timeout -k 10 300 /opt/conda/bin/mpiexec -n $2 $T/tsan_threads 3 100 > $T/run_$1.log 2>&1
  R=$?
  N=$(cat $T/report_$1.* 2>/dev/null | grep -c "WARNING: ThreadSanitizer" || true)
  local tempi
  tempi=$(for f in $T/report_$1.*; do [ -f $f ] && awk '/WARNING: ThreadSanitizer/{n++} /tempi::/{t[n]=1} END{c=0; for (k in t) c++; print c}' $f; done | awk '{s+=$1} END{print s+0}')
  echo "$1: ranks=$2 rc=$R $(grep RESULT $T/run_$1.log | tr '\n' ' ') tsan_reports=$N reports_with_tempi_frames=$tempi"
}
rc=0
for n in 1 2; do
  run n$n $n
  [ $R -eq 0 ] && [ $N -eq 0 ] || rc=1
done
run control_no_lock_n1 1 TEMPI_FAULT_NO_MT_LOCK=1
[ $N -gt 0 ] || { echo "negative control: TSan saw no race without the lock"; rc=1; }
exit $rc
