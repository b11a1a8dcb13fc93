#!/bin/bash
# LDS-resident scan results: GPU suite, c3 driver-shape bench, c4 kernel times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/c3_$i.json 2> $O/c3_$i.err || { tail -20 $O/c3_$i.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], d.get('steady_state'))" $O/c3_$i.json
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o c4 -- python3 tools/path_probe.py c4 0 3 > $O/trace_c4.log 2>&1 || { tail -20 $O/trace_c4.log; exit 1; }
grep "^frame" $O/trace_c4.log | tail -2
find $O/trace_c4 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-130 | head -4 | tail -3
