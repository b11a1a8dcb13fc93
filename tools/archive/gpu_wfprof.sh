#!/bin/bash
# per-kernel timeline of one variant (kprof) under rocprofv3 --kernel-trace --stats
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wfprof -o wf -- python3 tools/kprof.py --config ${CFG:-c3} --rounds 1 --iters 2 --variants ${VAR:-wf} > gpurun_out/wfprof.log 2>&1
echo "wfprof_rc=$?"
