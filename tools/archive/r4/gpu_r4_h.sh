#!/bin/bash
# AoS 48-B primitive records: parity subset, c3 bench, c4 kernel times.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cluster.py -x -q --timeout 200 --timeout-method thread \
  -k "multibounce or ragged or spheres or primary or hash or grazing or counters" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-steady > $O/c3_$i.json 2> $O/c3_$i.err || { tail -20 $O/c3_$i.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c3', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" $O/c3_$i.json
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o c4 -- python3 tools/path_probe.py c4 0 3 > $O/trace_c4.log 2>&1 || { tail -20 $O/trace_c4.log; exit 1; }
grep "^frame" $O/trace_c4.log | tail -2
find $O/trace_c4 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-130 | head -4 | tail -3
