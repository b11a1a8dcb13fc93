#!/bin/bash
# Check at HEAD after an illegal-address fault with an uncommitted change (reverted): parity, then
# the driver's c3 command twice and c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4ag2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cluster.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
run c3_1 --steps 20 --warmup 5
run c3_2 --steps 20 --warmup 5
run c4 --config c4 --steps 8 --warmup 2
