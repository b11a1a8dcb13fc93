#!/bin/bash
# c3 8-way shard balance: every rank with 32-px tiles, and with 5 calibration frames (0-4).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
run() {  # name, args
  timeout -k 10 120 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady --steps 20 --warmup 5 "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for v in "base:" "s32:--side 32" "cal5:--calib-frames 5"; do
  n=${v%%:*}; a=${v#*:}
  for r in 0 1 2 3 4 5 6 7; do run ${n}_r$r --sim-world 8 --sim-rank $r $a; done
done
