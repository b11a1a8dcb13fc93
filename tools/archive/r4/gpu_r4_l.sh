#!/bin/bash
# c3: HYBRID primary at 6 vs 7 waves/SIMD for frames in flight -- 8-way shard (rank 1) and full frame.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l2
mkdir -p $O
run() {  # name, args
  timeout -k 10 120 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady --steps 20 --warmup 5 "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); c=d['config']; print('$1', d['ms_per_step'], d['value'], c['launch_render_done_ms'])" || exit 1
}
for rep in 1 2 3; do
run s7_$rep --sim-world 8 --sim-rank 1
run s6_$rep --sim-world 8 --sim-rank 1 --tuning primary_occ=6
run s6r5_$rep --sim-world 8 --sim-rank 5 --tuning primary_occ=6
run s7r5_$rep --sim-world 8 --sim-rank 5
run f7_$rep
run f6_$rep --tuning primary_occ=6
done
