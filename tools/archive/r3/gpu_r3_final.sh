#!/bin/bash
# Round 3 final measurement set, part A: GPU suite + smoke, the driver's c3 command (PMC child,
# CPU baseline) and its rocprofv3 trace (gpu_r3_check.sh), c4 line (PMC child + CPU baseline),
# c4 PMC counter groups. Part B (gpu_r3_final_b.sh): c5 line and the 8-way shard timings.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r3_check.sh || exit $?
O=gpurun_out/r3c
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python3 bench.py --config c4 --steps 8 --warmup 2 > $O/bench_c4_full.json 2> $O/bench_c4_full.err || { tail -20 $O/bench_c4_full.err; exit 1; }
tail -c 300 $O/bench_c4_full.json; echo
rm -rf gpurun_out/r3c/pmc_c4
OUT_DIR=r3c/pmc_c4 PMC_SPP=64 PMC_BOUNCES=5 bash tools/gpu_pmc2.sh || exit $?
echo part A done
