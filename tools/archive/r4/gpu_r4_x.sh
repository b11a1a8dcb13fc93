#!/bin/bash
# 32-px shard tiles by default: the multi-rank GPU tests (gloo, real kernels, --check), then the
# 8-way shard set of c3/c4/c5 (tools/gpu_r4_sim8.sh).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bench_multi.py -x -v --timeout 300 --timeout-method thread > $O/pytest_multi.log 2>&1 || { tail -30 $O/pytest_multi.log; exit 1; }
tail -1 $O/pytest_multi.log
bash tools/gpu_r4_sim8.sh "c3 c4 c5"
