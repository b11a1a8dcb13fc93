#!/bin/bash
# Multi-rank rehearsals on one GPU (gloo, host-staged exchange): the N-rank plan, graded cell order,
# exchange, assembly and per-tile ray_casts, every frame checked against a one-launch render.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3mu
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
ATR_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 11 --warmup 3 --check --no-cpu-baseline --no-pmc > $O/gloo_n2.json 2> $O/gloo_n2.err || { tail -20 $O/gloo_n2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/gloo_n2.json').read().strip().splitlines()[-1]); print('n2', d['value'], d.get('check_mismatched_pixels'), d['config']['shard_pixels'])"
ATR_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 8 --steps 20 --warmup 5 --check --no-cpu-baseline --no-pmc > $O/gloo_n8.json 2> $O/gloo_n8.err || { tail -20 $O/gloo_n8.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/gloo_n8.json').read().strip().splitlines()[-1]); print('n8', d['value'], d.get('check_mismatched_pixels'), d['config']['shard_pixels'])"
