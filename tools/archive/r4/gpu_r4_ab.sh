#!/bin/bash
# c3 8-way shards: tile order (grid vs heaviest first) under the graded cell order; every rank.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ab
mkdir -p $O
run() {  # name, args
  timeout -k 10 120 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady --steps 20 --warmup 5 "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for r in 0 1 2 3 4 5 6 7; do run grid_r$r --sim-world 8 --sim-rank $r --tile-order grid; done
for r in 0 1 2 3 4 5 6 7; do run cost_r$r --sim-world 8 --sim-rank $r; done
for r in 0 1 2 3 4 5 6 7; do run gridlist_r$r --sim-world 8 --sim-rank $r --tile-order grid --cell-order list; done
