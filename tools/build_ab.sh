#!/bin/bash
# A/B builds of the gfx950 kernels: tools/_variants/libtempi_hip_<name>.so for
# the working tree ("cur") and for each git REF given (every file of its
# tempi_amd/csrc/hip/), plus the kernel benches kbench / hbench.
# An argument NAME:FLAGS instead builds the working tree with those compiler
# flags (e.g. "nowave:-DTEMPI_WAVE_DECODE=0").
# usage: tools/build_ab.sh [REF | NAME:FLAGS ...]   (then tools/kab.sh on the GPU box;
# tools/_variants is listed in .gpurunignore: drop that line for the A/B session)
set -e
cd "$(dirname "$0")/.."
V=${KAB_DIR:-tools/_variants} # KAB_DIR=tools/bin/v: a directory that travels to the GPU box
mkdir -p $V
rm -f $V/*.so
build() { # name dir [flags]
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Iinclude $3 \
    -o $V/libtempi_hip_$1.so $2/*.hip -Wl,-rpath,/opt/rocm/lib
}
build cur tempi_amd/csrc/hip &
for ref in "$@"; do
  if [[ "$ref" == *:* ]]; then
    build "${ref%%:*}" tempi_amd/csrc/hip "${ref#*:}" &
    continue
  fi
  d=$(mktemp -d)
  git archive "$ref" tempi_amd/csrc/hip | tar -x -C $d --strip-components=3
  build "$(echo "$ref" | tr -c 'A-Za-z0-9_\n' '_')" $d &
done
wait
g++ -O2 -std=c++17 -Iinclude -o $V/kbench tools/kbench.cpp -ldl
g++ -O2 -std=c++17 -Iinclude -o $V/hbench tools/hbench.cpp -ldl
ls $V
