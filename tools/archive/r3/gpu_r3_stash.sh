#!/bin/bash
# Camera rays stash no constants (ret, w, sample 0's hit record): GPU suite, then c4 / c5 A/B against
# the same build with the full stash (ATRAY_LIB=atray_amd/_lib/exp/stashall.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3st
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() {
  timeout -k 10 300 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for rep in 1 2; do
  ATRAY_LIB= b c4_new_$rep --config c4 --steps 8 --warmup 2
  ATRAY_LIB=atray_amd/_lib/exp/stashall.so b c4_old_$rep --config c4 --steps 8 --warmup 2
done
ATRAY_LIB= b c5_new --config c5 --steps 2 --warmup 1
ATRAY_LIB=atray_amd/_lib/exp/stashall.so b c5_old --config c5 --steps 2 --warmup 1
