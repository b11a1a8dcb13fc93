#!/bin/bash
# c3 at HEAD: HYBRID primary at 6 waves/SIMD for frames in flight, and XCD chunks of 8, against the defaults.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ak
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
run base_$rep --steps 20 --warmup 5
run occ6_$rep --steps 20 --warmup 5 --tuning primary_occ=6
run x8_$rep --steps 20 --warmup 5 --tuning xcd_chunk=8
done
