#!/bin/bash
# c4 (FLAT) XCD chunk sweep: a larger chunk gives each XCD a compact region of the frame (its L2 then
# holds fewer distinct leaves for the secondary rays); two interleaved repeats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
b() {
  timeout -k 10 200 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; kill $HB; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame'])"
}
for rep in 1 2; do
  for ch in 16 64 256 1024 0; do b c4_ch${ch}_$rep --tuning xcd_chunk=$ch; done
done
kill $HB
echo done
