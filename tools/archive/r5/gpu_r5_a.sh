#!/bin/bash
# Round 5 set A: the new GPU tests (API validation, workspaces, the c3 timed-shape launch), then the
# bench lines (c3 driver shape, c4, c5; no PMC) and the 2- and 4-way shard sets of the same shapes
# for the 1/2/4/8 projection (bench.py --sim-world N --sim-rank r).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_engine_api.py "tests/test_gpu_configs.py::test_c3_timed_shape_launch" -x -v --timeout 300 --timeout-method thread > $O/pytest_new.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_new.log | head -20; tail -40 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
run() {  # name, timeout, args
  timeout -k 10 $2 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:3}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for cfg in ${1:-c3 c4 c5}; do
  case $cfg in
    c3) A="--steps 20 --warmup 5"; T=120;;
    c4) A="--config c4 --steps 8 --warmup 2"; T=300;;
    c5) A="--config c5 --steps 2 --warmup 1"; T=600;;
  esac
  run ${cfg}_full $T $A
  for w in 2 4; do
    for r in $(seq 0 $((w - 1))); do run ${cfg}_sim${w}_r$r $T $A --sim-world $w --sim-rank $r; done
  done
done
echo all done
