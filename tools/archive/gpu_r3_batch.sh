#!/bin/bash
# Round 3 batch: GPU suite; single-frame plan A/B (split fractions); HYBRID frames-in-flight at 7 vs
# 6 waves/SIMD on the driver's shape; then the 8-way shard simulation (tools/gpu_r3_sim8.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for lib in prod s2 s4a; do
  L=""; [ $lib != prod ] && L=atray_amd/_lib/exp/$lib.so
  ATRAY_LIB=$L timeout -k 10 300 python3 -u tools/plan_probe.py > $O/plan_$lib.jsonl 2> $O/plan_$lib.err || { tail $O/plan_$lib.err; exit 1; }
  echo $lib; cut -c1-120 $O/plan_$lib.jsonl
done
b() {
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep "${@:2}" > $O/bench_$1.json 2> $O/bench_$1.err || exit $?
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d.get('steady_state',{}).get('mrays_s'))"
}
for rep in 1 2; do b auto7_$rep; b occ6_$rep --variant-code 86; done
bash tools/gpu_r3_sim8.sh
