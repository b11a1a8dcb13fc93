#!/bin/bash
# After the slot-map fix: packed per-tile counters under a cell plan, then the gloo N=2 / N=8 frame checks.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3mu
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "packed_tile_ray_casts or plan" > $O/plan_tests.log 2>&1 || { tail -30 $O/plan_tests.log; exit 1; }
tail -1 $O/plan_tests.log
bash tools/gpu_r3_multi.sh
