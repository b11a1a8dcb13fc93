#!/bin/bash
# Round-2 GPU check: host CPU facts, the GPU test suite, smoke, and the c3 bench at the driver's
# step count and at 48 steps (steps-independence). Each GPU step has its own time limit.
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-r2}
mkdir -p $O
python - > $O/cpu.txt 2>&1 <<'PY'
import os
print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for f in ("/sys/fs/cgroup/cpu.max", "/proc/cpuinfo"):
    try:
        txt = open(f).read()
        print(f, txt if f.endswith("max") else [l for l in txt.splitlines() if "model name" in l][:1])
    except OSError as e:
        print(f, e)
PY
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > $O/bench_c3_s20.log 2>&1 || { tail -20 $O/bench_c3_s20.log; exit 1; }
grep '^{' $O/bench_c3_s20.log | tail -1
timeout -k 10 300 python bench.py --steps 48 --warmup 8 --no-cpu-baseline --no-pmc ${BENCH_ARGS} > $O/bench_c3_s48.log 2>&1 || exit 1
grep '^{' $O/bench_c3_s48.log | tail -1 | cut -c1-400
echo done
