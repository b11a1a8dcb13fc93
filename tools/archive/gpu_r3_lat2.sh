#!/bin/bash
# Round 3: one-frame latency probe with 128-B cluster blocks (product) and wave-priority builds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cluster.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u tools/latency_probe.py > $O/latency.jsonl 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cut -c1-600 $O/latency.jsonl
for lib in prio4 prio8 prio16; do
  ATRAY_LIB=atray_amd/_lib/exp/$lib.so timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep > $O/bench_$lib.json 2> $O/bench_$lib.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d.get('steady_state',{}).get('mrays_s'))"
done
timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep > $O/bench_prod.json 2> $O/bench_prod.err || exit $?
python3 -c "import json,sys; d=json.loads(open('$O/bench_prod.json').read().strip().splitlines()[-1]); print('prod', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d.get('steady_state',{}).get('mrays_s'))"
timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 > $O/flat_probe.jsonl 2> $O/flat_probe.err || exit $?
grep -h '"bounces": 5' $O/flat_probe.jsonl | cut -c1-100
echo all done
