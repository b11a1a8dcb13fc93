export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --steps 20 --warmup 3 > $O/bench_c3_s20w3.json || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --steps 20 --warmup 5 > $O/bench_c3_s20w5.json || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --steps 20 --warmup 0 > $O/bench_c3_s20w0.json || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc > $O/bench_c3.json || exit 1
echo done
