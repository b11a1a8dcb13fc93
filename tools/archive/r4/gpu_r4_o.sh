#!/bin/bash
# Refill kernel thresholds (experiment: refill min / pass min through hybrid_a / hybrid_b), c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady --no-orbit --config c4 --steps 4 --warmup 1 "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'])" || exit 1
}
run claim64 --tuning path_refill=1
for t in 16,16 32,16 48,48 64,64 8,1 32,1 64,1 16,64; do
  a=${t%,*}; b=${t#*,}
  run r_${a}_${b} --tuning hybrid_a=$a,hybrid_b=$b
done
run claim64b --tuning path_refill=1
