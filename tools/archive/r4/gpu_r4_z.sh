#!/bin/bash
# Bounce rays with a 6-entry leaf buffer (LDS 18 KB per workgroup): at 7 waves/SIMD (k6) and at 8
# (k6o8, 64 VGPRs); parity of the multi-bounce suite on k6o8; c4 against HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O
ATRAY_LIB=atray_amd/_lib/exp/k6o8.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "multibounce or PATHS or paths or tuning or spheres" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2; do
run head_$rep --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/k6.so run k6_$rep --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/k6o8.so run k6o8_$rep --config c4 --steps 8 --warmup 2
done
