#!/bin/bash
# c4: path batch size (atr_tuning.path_batch_log2) -- 2^27 paths (one c4 frame, default) vs
# smaller batches whose queues (144 B per path) fit the 256 MB MALL: 2^25, 2^23, 2^21, 2^20;
# `bash tools/archive/r4/gpu_r4_am.sh big`: 2^28 and 2^29 (2 and 4 c4 frames per batch).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4am
mkdir -p $O
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame'].get('latency_ms'))" || exit 1
}
for rep in 1 2; do
run b27_$rep --config c4 --steps 8 --warmup 2
BS="25 23 21 20"; [ "$1" = big ] && BS="28 29"
for b in $BS; do run b${b}_$rep --config c4 --steps 8 --warmup 2 --tuning path_batch_log2=$b; done
done
