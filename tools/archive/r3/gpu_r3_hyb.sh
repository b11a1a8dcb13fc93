#!/bin/bash
# HYBRID deal threshold (tuning hybrid_a / hybrid_b) re-swept at HEAD, c3 driver shape, two repeats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3hy
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
b() {
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for rep in $(seq 1 ${HY_REPS:-2}); do
  for ab in ${HY_SET:-2,1 1,1 3,1 2,0 2,3 4,2 1,0}; do
    a=${ab%,*}; bb=${ab#*,}
    b a${a}b${bb}_$rep --tuning hybrid_a=$a,hybrid_b=$bb
  done
done
