#!/bin/bash
# Experiment builds of the engine library into atray_amd/_lib/exp/<name>.so (loaded with
# ATRAY_LIB=...; git-ignored, travels to the GPU box), one per "name:defines" argument, compiled
# in parallel. Never the product library.
cd "$(dirname "$0")/../atray_amd/csrc" || exit 1
mkdir -p ../_lib/exp
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function"
for v in "$@"; do
  n=${v%%:*}
  d=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $F $d -shared -o ../_lib/exp/$n.so \
    render.hip paths.hip build.hip exchange.hip plan.hip capi.cpp host_scene.cpp obj_parse.cpp -lpthread &
done
wait
ls -la ../_lib/exp/*.so
