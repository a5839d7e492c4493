#!/bin/bash
# Host-side AddressSanitizer pass (CPU only, no GPU): libtempi.so's C++ and
# the reference's benchmarks restated in apps/ rebuilt with clang's ASan
# (-Xarch_host on the hipcc lines, so no device code is instrumented; the
# runtime is the executables' own dependency, nothing is preloaded), into
# build/asan/. Each app then runs on host buffers (TEMPI_BENCH_HOST=1)
# through the interposer, with TEMPI's own host-side paths forced on
# (TEMPI_TEST_HOST_ONLY=1) and every received byte checked. Any memory error
# aborts the rank that hit it.
set -e
cd "$(dirname "$0")/.."
ROOT=$PWD
A=build/asan
mkdir -p $A
CXX=/opt/rocm/llvm/bin/clang++
H=/opt/rocm/bin/hipcc
RT=$(dirname $($CXX -print-file-name=libclang_rt.asan-x86_64.so))
for f in tempi_amd/csrc/core/*.cpp; do
  $CXX -std=c++17 -O1 -g -fPIC -fvisibility=hidden -fsanitize=address -fno-omit-frame-pointer \
    -Iinclude -I/opt/conda/include -c $f -o $A/$(basename $f .cpp).o &
done
wait
$CXX -shared -fsanitize=address -shared-libsan -o $A/libtempi.so $A/*.o -Ltempi_amd/lib -ltempi_hip \
  /opt/conda/lib/libmpi.so -ldl -lpthread -static-libstdc++ -Wl,--exclude-libs,ALL -Wl,-rpath,'$ORIGIN' \
  -Wl,-rpath,$ROOT/tempi_amd/lib -Wl,-rpath,/opt/conda/lib -Wl,-rpath,$RT -Wl,--enable-new-dtags
SAN="-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer -shared-libsan"
R="-static-libstdc++ -Wl,-rpath,$ROOT/$A -Wl,-rpath,$ROOT/tempi_amd/lib -Wl,-rpath,/opt/conda/lib -Wl,-rpath,$RT"
INC="-Iinclude -I/opt/conda/include"
LIBS="-L$A -ltempi -Ltempi_amd/lib -ltempi_hip -L/opt/conda/lib -lmpi"
$H --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC -shared $SAN $INC -o $A/libtempi_apps.so apps/halo_lib.cpp apps/bench_lib.cpp $LIBS $R
for a in halo_exchange_main:halo_exchange pingpong_nd:pingpong_nd pingpong_1d:pingpong_1d \
         alltoallv_sparse:alltoallv_sparse mpi_isend:mpi_isend; do
  $H --offload-arch=gfx950 -O1 -g -std=c++17 $SAN $INC -o $A/${a##*:} apps/${a%%:*}.cpp -L$A -ltempi_apps $LIBS $R
done
for a in type_commit mpi_pack; do
  $H --offload-arch=gfx950 -O1 -g -std=c++17 $SAN $INC -o $A/$a apps/$a.cpp $LIBS $R
done
set +e
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 HYDRA_LAUNCHER=fork TEMPI_BENCH_HOST=1
MPI=/opt/conda/bin/mpiexec
fails=0
run() { # ranks cmd...
  local n=$1; shift
  if out=$(timeout -k 10 300 $MPI -n $n "$@" 2>&1) && ! grep -q "ERROR: AddressSanitizer" <<< "$out" \
     && ! grep -q '"errors": [1-9]' <<< "$out"; then
    echo "ok   n=$n $*"
  else
    echo "FAIL n=$n $*"; echo "$out" | tail -30; fails=$((fails + 1))
  fi
}
for host_only in 1 0; do
  export TEMPI_TEST_HOST_ONLY=$host_only
  echo "== TEMPI_TEST_HOST_ONLY=$host_only"
  for n in 1 2 4; do run $n $A/halo_exchange 2 24 --quants 2 --check; done
  run 8 $A/halo_exchange 2 24 --quants 2 --check
  run 2 $A/halo_exchange 2 24 --quants 2 --check --neighbor
  run 2 $A/pingpong_nd 3 1024 8 --check
  run 2 $A/pingpong_nd 3 65536 64 --check
  run 4 $A/pingpong_1d 2 65536 --check
  run 2 $A/mpi_isend 2 1 4096 65536 --check
  run 4 $A/alltoallv_sparse 2 --scale 1000 --density 0.5 --check
  run 4 $A/alltoallv_sparse 2 --scale 1000 --density 0.5 --check --neighbor
  run 1 $A/type_commit
  run 1 $A/mpi_pack 2 --host --max-target 1024
done
echo "failures: $fails"
exit $fails
