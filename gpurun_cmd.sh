export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_gpu_parity.py tests/test_gpu_cluster.py -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python tools/kprof.py --variants cl,hyb4,hyb5 --rounds 7 > $O/kp_c3.json || exit 1
for v in 84 85 36 37; do
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --variant-code $v > $O/bench_c3_$v.json || exit 1
done
echo done
