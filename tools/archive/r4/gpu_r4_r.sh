#!/bin/bash
# Cluster screen: only the direction through the opaque copy (experiment build sdo) vs HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4r
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
run base_c3_$rep --steps 20 --warmup 5
ATRAY_LIB=atray_amd/_lib/exp/sdo.so run sdo_c3_$rep --steps 20 --warmup 5
done
for rep in 1 2; do
run base_c4_$rep --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/sdo.so run sdo_c4_$rep --config c4 --steps 8 --warmup 2
done
