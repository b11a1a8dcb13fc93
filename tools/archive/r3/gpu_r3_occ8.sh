#!/bin/bash
# HYBRID primary at 8 waves/SIMD (diagnostic 88; 64 VGPRs, 20.2 KB LDS) vs 7 (87) vs AUTO, c3 driver
# shape, three interleaved repeats; the plan/packed tests on the rebuilt library.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3o8
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() {
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for rep in 1 2 3; do b auto_$rep; b o8_$rep --variant-code 88; b o7_$rep --variant-code 87; done
