#!/bin/bash
# Which change breaks the gloo N=2 frame check: graded cell order, the frame plan on top of it, or neither.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3mu
mkdir -p $O
c() {
  ATR_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 11 --warmup 3 --check --no-cpu-baseline --no-pmc --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d.get('check_mismatched_pixels'))"
}
c list --cell-order list
c graded_noframeplan --tuning frame_plan=0
c list_noframeplan --cell-order list --tuning frame_plan=0
c graded
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "plan" > $O/plan_tests.log 2>&1; tail -3 $O/plan_tests.log
