#!/bin/bash
# Build libtempi_hip.so tuning variants into tools/_variants/ plus the kernel
# benches (kbench: pack/unpack shapes, hbench: halo regions incl. the copy).
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
rm -f tools/_variants/*.so
build() { # name flags...
  local name=$1; shift
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude "$@" \
    -o tools/_variants/libtempi_hip_$name.so tempi_amd/csrc/hip/pack_kernels.hip tempi_amd/csrc/hip/runtime.hip \
    -Wl,-rpath,/opt/rocm/lib &
}
build cur
build base -DTEMPI_DENSE=0 -DTEMPI_PACK_IL_WIDTHS=0 -DTEMPI_UNPACK_IL_WIDTHS=0
wait
g++ -O2 -std=c++17 -Iinclude -o tools/_variants/kbench tools/kbench.cpp -ldl
g++ -O2 -std=c++17 -Iinclude -o tools/_variants/hbench tools/hbench.cpp -ldl
ls tools/_variants
# hostbench: built like the apps (hipcc, static libstdc++: conda's older
# libstdc++ sits on the MPI rpath)
hipcc -O2 -std=c++17 -Iinclude -I/opt/conda/include -o tools/_variants/hostbench tools/hostbench.cpp \
  -Ltempi_amd/lib -ltempi_hip -L/opt/conda/lib -lmpi -static-libstdc++ \
  -Wl,-rpath,'$ORIGIN/../../tempi_amd/lib' -Wl,-rpath,/opt/conda/lib
