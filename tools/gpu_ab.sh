#!/bin/bash
# A/B of the product library against experiments, general form: variants "prod", "exp=<name>" (atray_amd/_lib/exp/<name>.so) or
# "tune=<k=v,...>" (product library, bench.py --tuning), "exp=<name>@<k=v,...>" (both) or
# "args=<arg>+<arg>..." (product library, these bench.py arguments, e.g. args=--streams=1),
# "expargs=<name>:<arg>+<arg>..." (an experiment build with bench.py arguments),
# interleaved twice, on the configs given.
# usage: gpu_ab.sh OUTDIR "variant ..." "c3 c4" [tests]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
if [ "${4:-notests}" = "tests" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
run() {  # name, timeout, lib, args
  ATRAY_LIB=$3 timeout -k 10 $2 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:4}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], d['single_frame']['kernel_ms'], d['single_frame']['mrays_s'])"
}
for i in 1 2; do
  n=0
  for v in $2; do
    n=$((n + 1))
    L=atray_amd/_lib/libatray_hip.so; T=""
    case $v in
      exp=*@*) x=${v#exp=}; L=atray_amd/_lib/exp/${x%%@*}.so; T="--tuning ${x#*@}";;
      exp=*) L=atray_amd/_lib/exp/${v#exp=}.so;;
      tune=*) T="--tuning ${v#tune=}";;
      args=*) T=$(echo ${v#args=} | tr '+' ' ');;
      expargs=*) x=${v#expargs=}; L=atray_amd/_lib/exp/${x%%:*}.so; T=$(echo ${x#*:} | tr '+' ' ');;
    esac
    for cfg in $3; do
      case $cfg in
        c3) run c3_v${n}_$i 120 $L --steps 20 --warmup 5 $T;;
        c4) run c4_v${n}_$i 300 $L --config c4 --steps 8 --warmup 2 $T;;
        c5) run c5_v${n}_$i 600 $L --config c5 --steps 2 --warmup 1 $T;;
      esac
    done
  done
done
echo "variants: $2"
echo all done
