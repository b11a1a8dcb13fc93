#!/bin/bash
# Cluster size re-check with the round-4 kernels (tuning cluster_size 16 default / 12 / 8): c3, c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ai
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
for c in 16 12 8; do run c3_cs${c}_$rep --steps 20 --warmup 5 --tuning cluster_size=$c; done
done
for c in 16 12 8; do run c4_cs${c} --config c4 --steps 8 --warmup 2 --tuning cluster_size=$c; done
