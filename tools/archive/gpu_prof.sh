#!/bin/bash
# GPU-box profiling pass: kprof A/B (c3 and a multi-bounce case) + rocprofv3 kernel stats of
# the bench. Each GPU step has its own limit; a crash-class exit stops the script.
export TMPDIR=/tmp
mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python tools/kprof.py --config c3 ${KPROF_ARGS} > gpurun_out/kprof_c3.json 2> gpurun_out/kprof_c3.err
rc=$?; echo "kprof_c3_rc=$rc"; if crash $rc; then exit $rc; fi
timeout -k 10 300 python tools/kprof.py --config c3 --spp 4 --bounces 5 --rounds 3 --iters 3 ${KPROF_MB_ARGS} > gpurun_out/kprof_c3_s4b5.json 2> gpurun_out/kprof_c3_s4b5.err
rc=$?; echo "kprof_mb_rc=$rc"; if crash $rc; then exit $rc; fi
if [ -n "$ROCPROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rocprof -o bench -- python3 bench.py --steps 20 --warmup 3 --streams 1 --no-cpu-baseline --no-pmc ${BENCH_EXTRA} > gpurun_out/rocprof_bench.log 2>&1
  rc=$?; echo "rocprof_rc=$rc"
fi
