#!/bin/bash
# c3 at the driver's shape: XCD chunk sweep (tuning xcd_chunk 8 / 16 default / 32 / 64), interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4v
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
for x in 16 8 32 64; do
run x${x}_$rep --steps 20 --warmup 5 --tuning xcd_chunk=$x
done
done
