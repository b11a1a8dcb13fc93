#!/bin/bash
# HYBRID deal threshold re-sweep after the in-place candidate tests (c3 driver shape; c4 camera rays).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4y
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
for t in 2,0 3,0 4,0 2,2 1,0; do
  a=${t%,*}; b=${t#*,}
  run c3_${a}_${b}_$rep --steps 20 --warmup 5 --tuning hybrid_a=$a,hybrid_b=$b
done
done
for t in 2,0 3,0 4,0 1,0; do
  a=${t%,*}; b=${t#*,}
  run c4_${a}_${b} --config c4 --steps 8 --warmup 2 --tuning hybrid_a=$a,hybrid_b=$b
done
