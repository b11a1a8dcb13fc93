#!/bin/bash
# Round 3: product FLAT (LDS leaf buffer, private path stash, 5 waves/SIMD, candidate compaction):
# full GPU suite, c4-shape probe (4/5/6 waves), c4 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 68 70 96 > $O/flat_probe.jsonl 2> $O/flat_probe.err || exit $?
grep -h '"bounces": 5' $O/flat_probe.jsonl | cut -c1-100
timeout -k 10 400 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
python3 -c "import json; d=json.loads(open('$O/bench_c4.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'])"
echo all done
