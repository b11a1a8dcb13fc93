#!/bin/bash
# Round-4 measurement set (copied into profiles/r04 by tools/collect_r04.py).
#   tests: the GPU suite + smoke
#   bench: the driver's c3 command with PMC passes and the CPU baseline, c4 and c5 lines,
#          rocprofv3 kernel traces of the c3 driver command and of the c4 line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4final
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
case ${1:-bench} in
tests)
  timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  ;;
bench)
  line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r.get('frac'), r.get('traffic_per_frame'), d['cpu_baseline'].get('value'))" $1; }
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
  line $O/bench_c3.json
  timeout -k 10 400 python3 bench.py --config c4 --steps 8 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
  line $O/bench_c4.json
  timeout -k 10 400 python3 bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
  line $O/bench_c5.json
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_c3_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/trace_c3_driver.log 2>&1 || { tail -20 $O/trace_c3_driver.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-steady > $O/trace_c4.log 2>&1 || { tail -20 $O/trace_c4.log; exit 1; }
  echo traces done
  ;;
esac
