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
build u1b128k -DTEMPI_UNROLL_WIDE=1 -DTEMPI_MAX_BLOCKS=131072
build u1b256k -DTEMPI_UNROLL_WIDE=1 -DTEMPI_MAX_BLOCKS=262144
build u2b128k -DTEMPI_MAX_BLOCKS=131072
build u2b32k -DTEMPI_MAX_BLOCKS=32768
build u4b64k -DTEMPI_UNROLL_WIDE=4 -DTEMPI_MAX_BLOCKS=65536
build n2 -DTEMPI_UNROLL_NARROW=2
wait
g++ -O2 -std=c++17 -Iinclude -o tools/_variants/kbench tools/kbench.cpp -ldl
ls tools/_variants
