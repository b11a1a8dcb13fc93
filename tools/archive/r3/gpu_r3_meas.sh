#!/bin/bash
# Round 3 measurement set for the multi-bounce configs: GPU suite, c4/c5 bench lines, c4 PMC groups
# (FLAT, 64 spp x 5 bounces, one frame per launch), then the 8-way shard simulation.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 bench.py --config c4 --steps 8 --warmup 1 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || { tail -20 $O/bench_c4.err; exit 1; }
tail -c 300 $O/bench_c4.json; echo
OUT_DIR=r3m/pmc_c4 PMC_SPP=64 PMC_BOUNCES=5 bash tools/gpu_pmc2.sh || exit $?
timeout -k 10 600 python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -c 300 $O/bench_c5.json; echo
bash tools/gpu_r3_sim8.sh
