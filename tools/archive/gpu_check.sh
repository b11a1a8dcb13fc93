#!/bin/bash
# GPU-box validation: smoke -> pytest -m gpu -> short bench. Every GPU step has its own time
# limit; a crash-class exit (abort/segfault/timeout/kill) ends the script before the next GPU step.
export TMPDIR=/tmp
mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m gpu ${PYTEST_X--x} -q -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; if crash $rc; then exit $rc; fi
if [ -n "$BENCH_ARGS" ]; then
  timeout -k 10 ${BENCH_TIMEOUT:-400} python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench_rc=$rc"; tail -2 gpurun_out/bench.log
fi
