#!/bin/bash
# Round 5 A/B: the product library against experiment builds (atray_amd/_lib/exp/<name>.so),
# interleaved, at the driver's c3 shape and the c4 line; optionally the GPU suite first.
# usage: gpu_r5_ab.sh OUTDIR "exp1 exp2 ..." [tests] [configs]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
if [ "${3:-notests}" = "tests" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
run() {  # name, timeout, lib, args
  ATRAY_LIB=$3 timeout -k 10 $2 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:4}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for i in 1 2; do
  for v in prod $2; do
    if [ $v = prod ]; then L=atray_amd/_lib/libatray_hip.so; else L=atray_amd/_lib/exp/$v.so; fi
    for cfg in ${4:-c3 c4}; do
      case $cfg in
        c3) run c3_${v}_$i 120 $L --steps 20 --warmup 5;;
        c4) run c4_${v}_$i 300 $L --config c4 --steps 8 --warmup 2;;
      esac
    done
  done
done
echo all done
