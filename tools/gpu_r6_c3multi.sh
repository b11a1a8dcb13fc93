#!/bin/bash
# Round 6: the c3 8-GPU render side, per rank on one MI355X (bench.py --sim-world N --sim-rank r),
# under launch shapes and decompositions: the 8-way tile plan with stream 0 at high priority (the
# round-5 default) or equal priorities, 4 streams; and frame groups x tile shards (G groups of the
# 20 timed frames, each frame split over 8/G GPUs: 2 x 4, 4 x 2, 8 x 1).
# usage: gpu_r6_c3multi.sh OUTDIR [sets]   sets: full p8 e8 s8 g2 g4 g8 (default: all)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
run() {  # name, args
  timeout -k 10 120 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['steps'])"
}
A="--warmup 5"
for set in ${2:-full p8 e8 s8 g2 g4 g8}; do
  case $set in
    full) run full $A --steps 20;;
    p8) for r in 0 1 2 3 4 5 6 7; do run p8_r$r $A --steps 20 --sim-world 8 --sim-rank $r; done;;
    e8) for r in 0 1 2 3 4 5 6 7; do run e8_r$r $A --steps 20 --sim-world 8 --sim-rank $r --stream-priority 0; done;;
    s8) for r in 0 1 2 3 4 5 6 7; do run s8_r$r $A --steps 20 --sim-world 8 --sim-rank $r --stream-priority 0 --streams 4; done;;
    g2) for r in 0 1 2 3; do run g2_r$r $A --steps 10 --sim-world 4 --sim-rank $r; done;;
    g4) for r in 0 1; do run g4_r$r $A --steps 5 --sim-world 2 --sim-rank $r; done;;
    g8) run g8_r0 $A --steps 3;;
  esac
done
echo all done
