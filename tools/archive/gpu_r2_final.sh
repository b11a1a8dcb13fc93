#!/bin/bash
# Round-2 measurement set at HEAD (copied into profiles/r02/ afterwards): the GPU test suite and
# smoke, the default bench line (PMC traffic passes + CPU baseline), the driver's command, the
# default bench under a rocprofv3 kernel trace, c4/c5 lines, a 2-rank gloo rehearsal with the
# frame check, and every rank's shard of the 8-GPU plan alone (--sim-world 8).
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
step() { echo "== $1"; }
if [ -z "$SKIP_TESTS" ]; then
step tests
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
fi
step bench_default
timeout -k 10 600 python bench.py > $O/bench_c3_default.log 2>&1 || { tail -20 $O/bench_c3_default.log; exit 1; }
grep '^{' $O/bench_c3_default.log > $O/bench_c3_default.json; cut -c1-250 $O/bench_c3_default.json
step bench_driver_shape
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/bench_c3_s20.log 2>&1 || exit 1
grep '^{' $O/bench_c3_s20.log > $O/bench_c3_s20.json; cut -c1-250 $O/bench_c3_s20.json
step trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o bench -- \
  python3 bench.py --no-cpu-baseline --no-pmc > $O/bench_c3_traced.log 2>&1 || exit 1
grep '^{' $O/bench_c3_traced.log > $O/bench_c3_traced.json
python tools/trace_summary.py $O/trace_c3 $(python -c "import json; print(json.load(open('$O/bench_c3_traced.json'))['config']['frames_per_launch'])") > $O/trace_c3_summary.json || exit 1
step c4
timeout -k 10 400 python bench.py --config c4 --steps 8 --warmup 1 > $O/bench_c4.log 2>&1 || exit 1
grep '^{' $O/bench_c4.log > $O/bench_c4.json; cut -c1-250 $O/bench_c4.json
step c5
timeout -k 10 500 python bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5.log 2>&1 || exit 1
grep '^{' $O/bench_c5.log > $O/bench_c5.json; cut -c1-250 $O/bench_c5.json
step gloo2
ATR_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 11 --warmup 3 --check --no-pmc --no-cpu-baseline > $O/bench_gloo_n2.log 2>&1 || exit 1
grep '^{' $O/bench_gloo_n2.log > $O/bench_gloo_n2.json
step sim8
for r in 0 1 2 3 4 5 6 7; do
  timeout -k 10 120 python bench.py --sim-world 8 --sim-rank $r --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep > $O/sim8_$r.log 2>&1 || exit 1
  grep '^{' $O/sim8_$r.log > $O/sim8_$r.json
done
echo done
