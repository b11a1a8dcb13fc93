#!/bin/bash
# c5 (3840x2160, 256 spp, 5 bounces) on the path engine; c4 bench line.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python3 bench.py --config c5 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline --no-steady > $O/c5.json 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c5', d['value'], d['ms_per_step'], d['single_frame'])" $O/c5.json
timeout -k 10 300 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-steady > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'], d['single_frame'])" $O/c4.json
