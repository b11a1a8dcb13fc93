#!/bin/bash
# c4: path-engine batches in flight -- 2 (default), 3 or 4 streams.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4al
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config']['launches'])" || exit 1
}
for rep in 1 2; do
run s2_$rep --config c4 --steps 8 --warmup 2
run s3_$rep --config c4 --steps 8 --warmup 2 --streams 3
run s4_$rep --config c4 --steps 8 --warmup 2 --streams 4
done
