#!/bin/bash
# In-place candidate tests in lane-private steps: parity subset, c3 and c4 against the
# compacted-only build (experiment library noinp), interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cluster.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
run inp_c3_$rep --steps 20 --warmup 5
ATRAY_LIB=atray_amd/_lib/exp/noinp.so run noinp_c3_$rep --steps 20 --warmup 5
done
for rep in 1 2; do
run inp_c4_$rep --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/noinp.so run noinp_c4_$rep --config c4 --steps 8 --warmup 2
done
# launch shape of the driver's c3 command: 3 or 4 streams
for rep in 1 2; do
run s3_c3_$rep --steps 20 --warmup 5 --streams 3
run s4_c3_$rep --steps 20 --warmup 5 --streams 4
run s2_c3_$rep --steps 20 --warmup 5
done
