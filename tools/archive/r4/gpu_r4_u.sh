#!/bin/bash
# Occupancy recheck after the spill cuts: bounce 7 vs 6 waves/SIMD, camera 6 vs 5, c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2; do
run base_$rep --config c4 --steps 8 --warmup 2
run b6_$rep --config c4 --steps 8 --warmup 2 --tuning path_bounce_occ=6
run c5_$rep --config c4 --steps 8 --warmup 2 --tuning path_camera_occ=5
done
