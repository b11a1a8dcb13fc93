#!/bin/bash
# Bounce kernel re-reads its ray after the query (intersect_models + scene_finish): spills 44 -> 33
# dwords. Parity subset, c4 with PMC (bytes written) against the previous build (exp/head.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4t
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); r=d['roofline']; pf=r.get('pmc_frames') or {}
print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], 'write/frame', pf.get('write_bytes_per_frame'), 'tpr', r.get('traffic_per_traced_ray'))" || exit 1
}
run new_pmc --config c4 --steps 8 --warmup 2
for rep in 1 2; do
run new_$rep --config c4 --steps 8 --warmup 2 --no-pmc
ATRAY_LIB=atray_amd/_lib/exp/head.so run head_$rep --config c4 --steps 8 --warmup 2 --no-pmc
done
