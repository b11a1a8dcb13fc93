#!/bin/bash
# FLAT with path regeneration (diagnostic codes 101 = 4 waves/SIMD, 102 = 5): parity suites on the
# new schedule, then c4 bench lines against FLAT (variant 8) and the FLAT probe of both.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
ATR_TEST_VARIANTS=101,102 ATR_TEST_EXTRA_VARIANTS=101,102 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread -k "not c5" > $O/pytest_regen.log 2>&1 || { tail -30 $O/pytest_regen.log; exit 1; }
tail -1 $O/pytest_regen.log
b() {
  timeout -k 10 200 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame'])"
}
for rep in 1 2; do b flat_$rep; b regen4_$rep --variant-code 101; b regen5_$rep --variant-code 102; done
timeout -k 10 300 python3 -u tools/flat_probe.py 16 8 101 102 > $O/flat_probe.jsonl 2> $O/flat_probe.err || { tail $O/flat_probe.err; exit 1; }
cut -c1-600 $O/flat_probe.jsonl
