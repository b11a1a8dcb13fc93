#!/bin/bash
# c4: camera kernel at 7 (default) vs 6 waves/SIMD after the in-place candidate tests -- bench
# lines with the PMC passes (per-kernel bytes written).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4q
mkdir -p $O
run() {  # name, args
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); r=d['roofline']; pf=r.get('pmc_frames') or {}
print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], 'write/frame', pf.get('write_bytes_per_frame'), 'per kernel', pf.get('per_kernel_bytes_per_frame'), 'tpr', r.get('traffic_per_traced_ray'))" || exit 1
}
run cam7 --config c4 --steps 8 --warmup 2
run cam6 --config c4 --steps 8 --warmup 2 --tuning path_camera_occ=6
run cam7b --config c4 --steps 8 --warmup 2 --no-pmc
run cam6b --config c4 --steps 8 --warmup 2 --no-pmc --tuning path_camera_occ=6
# the next leaf's cluster range loaded during the current step (experiment build rpf)
run2() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
run2 base_c3_$rep --steps 20 --warmup 5
ATRAY_LIB=atray_amd/_lib/exp/rpf.so run2 rpf_c3_$rep --steps 20 --warmup 5
done
for rep in 1 2; do
run2 base_c4_$rep --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/rpf.so run2 rpf_c4_$rep --config c4 --steps 8 --warmup 2
done
