#!/bin/bash
# Path engine: per-XCD-group claim segments (path_segments 1 / 4 / 8) and the camera kernel at 6
# waves/SIMD, c4 bench lines; the tuning parity test.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "tuning" -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 200 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2; do
run seg1_$rep
run seg8_$rep --tuning path_segments=8
run seg4_$rep --tuning path_segments=4
run cam6_$rep --tuning path_camera_occ=6
done
