export TMPDIR=/tmp
O=gpurun_out/r2e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline --no-prep > $O/bench_c4.log 2>&1 || { tail $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log | cut -c1-600
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline --no-prep --variant cl > $O/bench_c4_cl.log 2>&1 || exit 1
grep '^{' $O/bench_c4_cl.log | cut -c1-400
timeout -k 10 400 python bench.py --config c5 --steps 1 --warmup 1 --frames-per-launch 1 --streams 1 --no-pmc --no-cpu-baseline --no-prep > $O/bench_c5.log 2>&1 || { tail $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log | cut -c1-600
