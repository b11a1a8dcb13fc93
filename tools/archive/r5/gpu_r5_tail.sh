#!/bin/bash
# Round 5: how an 8-way c3 shard's two timed launches overlap (rank 4 of the 8-way plan, bench.py
# --sim-world 8 --sim-rank 4): launch completion times for several launch shapes and priorities.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-r5tail}
mkdir -p $O
run() {  # name, args
  timeout -k 10 120 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady --steps 20 --warmup 5 --sim-world 8 --sim-rank 4 "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); c=d['config']; print('$1', d['ms_per_step'], c['launches'], c['launch_render_done_ms'], d['single_frame']['latency_ms'])"
}
for i in 1 2; do
  run prio_$i
  run noprio_$i --stream-priority 0
  run one_stream_$i --streams 1
  run four_launch_$i --frames-per-launch 5
  run one_launch10_$i --streams 1 --frames-per-launch 10 --steps 10
  run list_grid_$i --cell-order list --tile-order grid
  run list_cost_$i --cell-order list
done
echo all done
