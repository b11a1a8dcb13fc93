#!/bin/bash
# Round 3 final measurement set, part B: the c5 line, then every rank's 8-way shard of c3, c4, c5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat_b; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 bench.py --config c5 --steps 2 --warmup 1 --cpu-seconds 10 > $O/bench_c5_full.json 2> $O/bench_c5_full.err || { tail -20 $O/bench_c5_full.err; exit 1; }
tail -c 300 $O/bench_c5_full.json; echo
bash tools/gpu_r3_sim8.sh "${@:-c3 c4 c5}"
