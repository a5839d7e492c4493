#!/bin/bash
# Build libtempi_hip.so tuning variants into tools/_variants/ and kbench.
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_variants
build() { # name flags...
  local name=$1; shift
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude "$@" \
    -o tools/_variants/libtempi_hip_$name.so tempi_amd/csrc/hip/pack_kernels.hip tempi_amd/csrc/hip/runtime.hip \
    -Wl,-rpath,/opt/rocm/lib &
}
build cur
build u8_1 -DTEMPI_UNROLL_WIDE=1
build u16_2 -DTEMPI_UNROLL_16=2
wait
g++ -O2 -std=c++17 -Iinclude -o tools/_variants/kbench tools/kbench.cpp -ldl
ls tools/_variants
