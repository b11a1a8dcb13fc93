#!/bin/bash
# Round 3: descent cull (inner children behind the origin) -- GPU suite, A/B against the no-cull
# build on the c4 shape and c3, phase clocks of the CC kernels.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for lib in prod nocull prod nocull; do
  L=""; [ $lib = nocull ] && L=atray_amd/_lib/exp/nocull.so
  ATRAY_LIB=$L timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 > $O/flat_probe_$lib.jsonl 2> $O/flat_probe_$lib.err || exit $?
  grep -h '"bounces": 5' $O/flat_probe_$lib.jsonl | cut -c1-100
  ATRAY_LIB=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep > $O/bench_$lib.json 2> $O/bench_$lib.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$lib.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d.get('steady_state',{}).get('mrays_s'))"
done
PHASES=1 ATRAY_LIB=atray_amd/_lib/exp/phase.so timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 > $O/flat_probe_phase.jsonl 2> $O/flat_probe_phase.err || exit $?
echo all done
