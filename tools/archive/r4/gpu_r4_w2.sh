#!/bin/bash
# c3 8-way shard balance, second look: 32-px tiles again, 32-px + 5 calibration frames; c4 with 32-px tiles.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4w2
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for v in "s32:--side 32" "base:" "s32c5:--side 32 --calib-frames 5"; do
  n=${v%%:*}; a=${v#*:}
  for r in 0 1 2 3 4 5 6 7; do run ${n}_r$r --steps 20 --warmup 5 --sim-world 8 --sim-rank $r $a; done
done
for r in 0 1 2 3 4 5 6 7; do run c4s32_r$r --config c4 --steps 8 --warmup 2 --sim-world 8 --sim-rank $r --side 32; done
