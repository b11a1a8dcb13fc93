#!/bin/bash
# Lane-refilled bounce kernel (path_refill): multi-bounce parity, tuning test, c4 A/B against the
# claim-64 kernel, c3 (refactored scan helpers).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  -k "multibounce or ragged or spheres or variants_agree or tuning or paths or PATHS or schedules or band" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2; do
run refill_$rep --config c4 --steps 8 --warmup 2
run claim64_$rep --config c4 --steps 8 --warmup 2 --tuning path_refill=1
run c3_$rep --steps 20 --warmup 5
done
# W as the L1 distance (no square root per cluster): experiment build
for rep in 1 2; do
ATRAY_LIB=atray_amd/_lib/exp/wl1.so run wl1_c3_$rep --steps 20 --warmup 5
ATRAY_LIB=atray_amd/_lib/exp/wl1.so run wl1_c4_$rep --config c4 --steps 8 --warmup 2
done
