#!/bin/bash
# Round-6 measurement set (copied into profiles/r06 by tools/collect_r06.py). Steps, in order:
#   tests     the GPU suite + smoke
#   c3 c4 c5  the bench lines: the driver's c3 command (PMC passes + CPU baseline), c4, c5
#   trace_c3  rocprofv3 kernel trace of the driver's c3 command
#   trace_c4  rocprofv3 kernel trace of the c4 line
# usage: bash tools/gpu_r6_final.sh "tests c3 trace_c3"   (OUTDIR=r6final by default; BENCH_ARGS:
# extra bench.py arguments of the c4, c5 and trace_c4 steps, e.g. "--tuning path_sort_bits=6")
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r6final}
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
line() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[1], d['value'], d['ms_per_step'], r.get('frac'), r.get('traffic_per_frame'), d['cpu_baseline'].get('value'))" $1; }
for step in ${1:-tests c3 c4 c5 trace_c3 trace_c4}; do
  case $step in
  tests)
    timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
    tail -1 $O/pytest_gpu.log
    timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log;;
  c3)
    timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -20 $O/bench_c3.err; exit 1; }
    line $O/bench_c3.json;;
  c4)
    timeout -k 10 500 python3 bench.py --config c4 --steps 8 --warmup 2 $BENCH_ARGS > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
    line $O/bench_c4.json;;
  c5)
    timeout -k 10 600 python3 bench.py --config c5 --steps 2 --warmup 1 $BENCH_ARGS > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
    line $O/bench_c5.json;;
  trace_c3)
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace_c3_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/trace_c3_driver.log 2>&1 || { tail -20 $O/trace_c3_driver.log; exit 1; }
    echo trace_c3 done;;
  trace_c4)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-steady $BENCH_ARGS > $O/trace_c4.log 2>&1 || { tail -20 $O/trace_c4.log; exit 1; }
    echo trace_c4 done;;
  esac
done
echo all done
