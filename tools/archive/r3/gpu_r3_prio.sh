#!/bin/bash
# Raised wave priority (s_setprio) for the heaviest cells of the graded plan (--cell-prio FRAC) on
# c3 8-way shards and the full frame.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3pr
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
b() {
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], d['config']['launch_render_done_ms'])"
}
for rep in 1 2; do
for p in 0 0.02 0.05 0.2; do
  for r in 7 2; do b r${r}_p${p}_$rep --sim-world 8 --sim-rank $r --cell-prio $p; done
  b full_p${p}_$rep --cell-prio $p
done
done
