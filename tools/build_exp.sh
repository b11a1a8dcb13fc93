#!/bin/bash
# Experiment builds of the engine library into build/exp_<name>.so (loaded with ATRAY_LIB=...),
# one per "name:defines" argument, compiled in parallel. Never the product library.
cd "$(dirname "$0")/../atray_amd/csrc" || exit 1
mkdir -p ../../build
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function"
for v in "$@"; do
  n=${v%%:*}
  d=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F $d -shared -o ../../build/exp_$n.so \
    render.hip persist.hip wavefront.hip capi.cpp host_scene.cpp &
done
wait
ls -la ../../build/*.so
