#!/bin/bash
# Round 6: the c3 8-GPU render side, per rank on one MI355X (bench.py --sim-world N --sim-rank r:
# rank r's shard of the N-way cost plan alone, its masked stream encoded as in the real run), under
# launch shapes and decompositions. Sets (each = every rank of the plan):
#   full      the one-GPU line (20 frames)
#   p8 / e8   8-way tiles, stream 0 at high priority (round-5 default) / equal priorities
#   s8        8-way, 4 streams, equal priorities
#   e8s16     e8 with 16-px shard tiles;  e8cs2 / e8cs4: e8 with the top 2% cells split over 2 / 4 waves
#   e8prio    e8 with the top 2% cells' waves at raised issue priority
#   g2 g4 g8  frame groups x tile shards: 2 x 4-way (10 frames per rank), 4 x 2-way (5), 8 x whole (3)
# usage: gpu_r6_c3multi.sh OUTDIR "sets" [reps]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
run() {  # name, args
  timeout -k 10 120 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['steps'], d['config']['launch_render_done_ms'], (d.get('sim') or {}).get('stream_bytes_per_frame'))"
}
A="--warmup 5"
ranks8() {  # set name, extra args
  for r in 0 1 2 3 4 5 6 7; do run ${1}_r${r}_$i $A --steps 20 --sim-world 8 --sim-rank $r "${@:2}"; done
}
for i in $(seq 1 ${3:-1}); do
for set in $2; do
  case $set in
    full) run full_$i $A --steps 20;;
    p8) ranks8 p8 --stream-priority 1;;
    e8) ranks8 e8 --stream-priority 0;;
    s8) ranks8 s8 --stream-priority 0 --streams 4;;
    e8s16) ranks8 e8s16 --stream-priority 0 --side 16;;
    e8cs2) ranks8 e8cs2 --stream-priority 0 --cell-split 2:0.02;;
    e8cs4) ranks8 e8cs4 --stream-priority 0 --cell-split 4:0.02;;
    e8prio) ranks8 e8prio --stream-priority 0 --cell-prio 0.02;;
    g2) for r in 0 1 2 3; do run g2_r${r}_$i $A --steps 10 --sim-world 4 --sim-rank $r; done;;
    g4) for r in 0 1; do run g4_r${r}_$i $A --steps 5 --sim-world 2 --sim-rank $r; done;;
    g8) run g8_r0_$i $A --steps 3;;
  esac
done
done
echo all done
