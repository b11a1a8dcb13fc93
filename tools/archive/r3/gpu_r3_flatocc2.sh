#!/bin/bash
# c4 (FLAT) at 6 / 7 waves/SIMD (diagnostic codes 70 / 71), with XCD chunk 8; c5 at 6 vs 7.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3o2
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
b() {
  timeout -k 10 300 python3 bench.py --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for rep in 1 2; do
  b occ6_$rep --config c4 --variant-code 70; b occ7_$rep --config c4 --variant-code 71
  b occ6ch8_$rep --config c4 --variant-code 70 --tuning xcd_chunk=8; b occ7ch8_$rep --config c4 --variant-code 71 --tuning xcd_chunk=8
done
b c5occ6 --config c5 --steps 2 --warmup 1 --variant-code 70; b c5occ7 --config c5 --steps 2 --warmup 1 --variant-code 71
