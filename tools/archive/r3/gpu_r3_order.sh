#!/bin/bash
# Graded heavy-first cell dispatch (--cell-order graded) on c3 8-way shards, the c3 full frame, and
# c4 shards / full frame.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3od
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
b() {
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], d['config']['launch_render_done_ms'])"
}
for rep in 1 2; do
for o in list graded; do
  for r in 7 0 3; do b c3r${r}_${o}_$rep --steps 20 --warmup 5 --sim-world 8 --sim-rank $r --cell-order $o; done
  b c3full_${o}_$rep --steps 20 --warmup 5 --cell-order $o
done
done
for o in list graded; do
  for r in 7 0; do b c4r${r}_$o --config c4 --steps 8 --warmup 2 --sim-world 8 --sim-rank $r --cell-order $o; done
  b c4full_$o --config c4 --steps 8 --warmup 2 --cell-order $o
done
