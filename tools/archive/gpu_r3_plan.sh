#!/bin/bash
# Round 3: the GPU-built single-frame plan -- GPU suite, one-frame latency (plan on vs off), c3
# driver shape, flat probe.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for t in frame_plan=1 frame_plan=0 frame_plan=1 frame_plan=0; do
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --tuning $t > $O/bench_$t.json 2> $O/bench_$t.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$t.json').read().strip().splitlines()[-1]); print('$t', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d.get('steady_state',{}).get('mrays_s'))"
done
echo all done
