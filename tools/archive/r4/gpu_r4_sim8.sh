#!/bin/bash
# Round 4: the 8-GPU plan's per-rank render side on one GPU (bench.py --sim-world 8 --sim-rank r):
# each rank's shard of c3, c4 and c5 alone (its render + 3-byte pack; no exchange), plus the
# full-frame line of the same shape, for the N=8 projection.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4sim
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
run() {  # name, timeout, args
  timeout -k 10 $2 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:3}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d['config']['shard_pixels'][:1] if 'sim' not in d else d['sim'])"
}
CFGS=${1:-c3 c4 c5}
# the same timed shape for the full frame and the shards of a config
for cfg in $CFGS; do
  case $cfg in
    c3) A="--steps 20 --warmup 5"; T=120;;
    c4) A="--config c4 --steps 8 --warmup 2"; T=300;;
    c5) A="--config c5 --steps 2 --warmup 1"; T=600;;
  esac
  run ${cfg}_full $T $A
  for r in 0 1 2 3 4 5 6 7; do run ${cfg}_sim8_r$r $T $A --sim-world 8 --sim-rank $r; done
done
echo all done
