#!/bin/bash
# Host-side UndefinedBehaviorSanitizer pass (CPU only, no GPU): libtempi.so's
# C++ rebuilt with -fsanitize=undefined -fno-sanitize-recover=all (the
# runtime linked in statically, nothing preloaded), swapped into
# tempi_amd/lib for one run of the CPU suite, then the normal build put back.
# Any undefined behaviour aborts the process that hit it, so its test fails.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ubsan
for f in tempi_amd/csrc/core/*.cpp; do
  g++ -std=c++17 -O1 -g -fPIC -fvisibility=hidden -fsanitize=undefined -fno-sanitize-recover=all -fno-sanitize=vptr \
    -Iinclude -I/opt/conda/include -c $f -o build/ubsan/$(basename $f .cpp).o &
done
wait
g++ -shared -fsanitize=undefined -static-libubsan -o build/ubsan/libtempi.so build/ubsan/*.o -Ltempi_amd/lib -ltempi_hip \
  /opt/conda/lib/libmpi.so -ldl -lpthread -static-libstdc++ -static-libgcc -Wl,--exclude-libs,ALL \
  -Wl,-rpath,'$ORIGIN' -Wl,-rpath,/opt/conda/lib -Wl,--enable-new-dtags
cp tempi_amd/lib/libtempi.so build/ubsan/libtempi.so.normal
cp build/ubsan/libtempi.so tempi_amd/lib/libtempi.so
set +e
python -m pytest tests -q -m "not gpu" -n 4 -p no:cacheprovider
rc=$?
cp build/ubsan/libtempi.so.normal tempi_amd/lib/libtempi.so
exit $rc
