#!/bin/bash
# Round 3: the product kernels with candidate compaction -- full GPU suite, then A/B of the FLAT
# variants on the c4 shape and of HYBRID occupancy / deal thresholds on c3 (driver shape).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 96 100 > $O/flat_probe.jsonl 2> $O/flat_probe.err || exit $?
grep -h '"bounces": 5' $O/flat_probe.jsonl | cut -c1-100
b() {  # name, extra bench args
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep "${@:2}" > $O/bench_$1.json 2> $O/bench_$1.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d.get('steady_state',{}).get('mrays_s'))"
}
for rep in 1 2; do
  b auto_$rep
  b occ5_$rep --variant-code 85
  b occ7_$rep --variant-code 87
  b nocc_$rep --variant-code 97
  b a1b0_$rep --tuning hybrid_a=1,hybrid_b=0
  b a3b2_$rep --tuning hybrid_a=3,hybrid_b=2
  b a4b4_$rep --tuning hybrid_a=4,hybrid_b=4
  b never_$rep --tuning hybrid_a=4096,hybrid_b=4096
  b always_$rep --tuning hybrid_a=-4096,hybrid_b=-4096
done
echo all done
