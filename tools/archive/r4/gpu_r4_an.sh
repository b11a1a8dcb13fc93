#!/bin/bash
# c4 at path_batch_log2 = 29 (one 531 M-path batch per 4-frame launch, 77 GB of queues per stream):
# outputs checked against one-frame launches (--check), and one stream vs two.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4an
mkdir -p $O
run() {  # name, args
  timeout -k 10 300 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['roofline'].get('launch_ms'), d.get('check_mismatched_pixels'))" || exit 1
}
run b29_check --config c4 --steps 8 --warmup 2 --tuning path_batch_log2=29 --check
run b29_s1 --config c4 --steps 8 --warmup 2 --tuning path_batch_log2=29 --streams 1
run b28_check --config c4 --steps 8 --warmup 2 --tuning path_batch_log2=28 --check
