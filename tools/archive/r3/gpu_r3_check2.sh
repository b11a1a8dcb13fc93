#!/bin/bash
# gpu_r3_check.sh, then c4 and the c3 8-way shards at HEAD.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r3_check.sh || exit $?
O=gpurun_out/r3c
timeout -k 10 300 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
tail -c 400 $O/bench_c4.json; echo
bash tools/gpu_r3_sim8.sh c3
