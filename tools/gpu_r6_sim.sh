#!/bin/bash
# Round 6: every rank's shard of the N-way cost plans (N = 2, 4, 8) alone on one GPU, in the same
# timed shape as the full-frame line (bench.py --sim-world N --sim-rank r: render, per-tile
# counters and the masked stream's encoding, as that rank runs them), for tools/project_r6.py.
# usage: gpu_r6_sim.sh OUTDIR "c3 c4 c5" ["2 4 8"] [reps] [extra bench.py args, e.g. "--streams 2"]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
run() {  # name, timeout, args
  timeout -k 10 $2 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:3}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], (d.get('sim') or {}).get('stream_bytes_per_frame'))"
}
for i in $(seq 1 ${4:-1}); do
for cfg in $2; do
  case $cfg in
    c3) A="--steps 20 --warmup 5"; T=120;;
    c4) A="--config c4 --steps 8 --warmup 2"; T=300;;
    c5) A="--config c5 --steps 2 --warmup 1"; T=600;;
  esac
  run ${cfg}_full_$i $T $A $5
  for w in ${3:-2 4 8}; do
    for r in $(seq 0 $((w - 1))); do run ${cfg}_sim${w}_r${r}_$i $T $A --sim-world $w --sim-rank $r $5; done
  done
done
done
echo all done
