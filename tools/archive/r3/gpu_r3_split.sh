#!/bin/bash
# c3 8-way shards are tail-bound (one shard frame ~0.05 ms of work, its slowest cell ~0.3 ms): the
# heaviest cells split over P waves (--cell-split P:FRAC, atr_set_cell_plan) on two shards and the
# full frame.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
b() {
  timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], d['config']['launch_render_done_ms'])"
}
for sp in none 2:0.03 4:0.01 4:0.03 8:0.01 8:0.03; do
  A=""; [ $sp != none ] && A="--cell-split $sp"
  for r in 7 0; do b r${r}_${sp/:/_} --sim-world 8 --sim-rank $r $A; done
  b full_${sp/:/_} $A
done
