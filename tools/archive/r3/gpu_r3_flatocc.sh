#!/bin/bash
# c4 (FLAT) at 4 / 5 / 6 waves/SIMD (diagnostic codes 68 / 69 / 70; default = 5) and XCD chunks of
# 4 and 8 cells, two interleaved repeats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
b() {
  timeout -k 10 200 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for rep in 1 2; do
  b flat_$rep; b occ4_$rep --variant-code 68; b occ6_$rep --variant-code 70
  b ch4_$rep --tuning xcd_chunk=4; b ch8_$rep --tuning xcd_chunk=8
done
