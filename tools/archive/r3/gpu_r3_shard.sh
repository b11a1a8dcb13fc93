#!/bin/bash
# c3 8-way shard launch shapes: 2 streams with / without stream priority, one stream, 5-frame launches.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3sh
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
b() {
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['config']['launches'], d['config']['launch_render_done_ms'])"
}
for rep in 1 2; do
for r in 7 2; do
  b r${r}_def_$rep --sim-world 8 --sim-rank $r
  b r${r}_noprio_$rep --sim-world 8 --sim-rank $r --stream-priority 0
  b r${r}_s1_$rep --sim-world 8 --sim-rank $r --streams 1
  b r${r}_f5_$rep --sim-world 8 --sim-rank $r --frames-per-launch 5
  b r${r}_s3_$rep --sim-world 8 --sim-rank $r --streams 3 --frames-per-launch 7
done
done
