#!/bin/bash
# Multi-frame camera cap 24: the c3 run as ONE 20-frame launch on one stream vs 10 + 10 on two --
# every rank of the 8-way plan and the full frame.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "cameras or frames" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 120 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady --steps 20 --warmup 5 "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['ms_per_step'], d['config']['launches'], d['config']['launch_render_done_ms'])" || exit 1
}
run full_base
run full_one --streams 1 --frames-per-launch 20
for r in 0 1 2 3 4 5 6 7; do run one_r$r --sim-world 8 --sim-rank $r --streams 1 --frames-per-launch 20; done
for r in 0 1 2 3 4 5 6 7; do run base_r$r --sim-world 8 --sim-rank $r; done
run full_base2
run full_one2 --streams 1 --frames-per-launch 20
