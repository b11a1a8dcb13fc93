#!/bin/bash
# In-place candidate tests up to 2 x rounds - 1 per lane (experiment build ipw) vs HEAD: c3, c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ad
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
run base_c3_$rep --steps 20 --warmup 5
ATRAY_LIB=atray_amd/_lib/exp/ipw.so run ipw_c3_$rep --steps 20 --warmup 5
done
for rep in 1 2; do
run base_c4_$rep --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/ipw.so run ipw_c4_$rep --config c4 --steps 8 --warmup 2
done
