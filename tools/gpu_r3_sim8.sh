#!/bin/bash
# Round 3: the 8-GPU plan's per-rank render side on one GPU (bench.py --sim-world 8 --sim-rank r):
# each rank's shard of c3, c4 and c5 alone (its render + 3-byte pack; no exchange), plus the
# full-frame line of the same shape, for the N=8 projection.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3sim
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
run() {  # name, timeout, args
  timeout -k 10 $2 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:3}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d['config']['shard_pixels'][:1] if 'sim' not in d else d['sim'])"
}
run c3_full 120 --steps 20 --warmup 5
for r in 0 1 2 3 4 5 6 7; do run c3_sim8_r$r 120 --steps 20 --warmup 5 --sim-world 8 --sim-rank $r; done
run c4_full 300 --config c4 --steps 4 --warmup 1
for r in 0 1 2 3 4 5 6 7; do run c4_sim8_r$r 300 --config c4 --steps 8 --warmup 2 --sim-world 8 --sim-rank $r; done
run c5_full 600 --config c5 --steps 1 --warmup 1 --streams 1
for r in 0 1 2 3 4 5 6 7; do run c5_sim8_r$r 300 --config c5 --steps 2 --warmup 1 --sim-world 8 --sim-rank $r --streams 1; done
echo all done
