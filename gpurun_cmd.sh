export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_c3_default.json || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --no-pmc --steps 20 --warmup 5 > $O/bench_c3_s20.json || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o run -- python3 bench.py --no-cpu-baseline --no-pmc > $O/bench_c3_traced.json 2> $O/trace_c3.err || exit 1
python tools/trace_summary.py $O/trace_c3 4 > $O/trace_c3_summary.json || exit 1
OUT_DIR=r02/pmc bash tools/gpu_pmc2.sh > $O/pmc.log 2>&1 || exit 1
python tools/pmc_summary2.py $O/pmc > $O/pmc_summary.json || exit 1
timeout -k 10 400 python bench.py --config c4 --steps 8 --warmup 1 > $O/bench_c4.json || exit 1
timeout -k 10 500 python bench.py --config c5 --steps 2 --warmup 1 > $O/bench_c5.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o run -- python3 bench.py --config c4 --steps 4 --warmup 1 --no-cpu-baseline --no-pmc --no-prep > $O/bench_c4_traced.json 2> $O/trace_c4.err || exit 1
python tools/trace_summary.py $O/trace_c4 4 > $O/trace_c4_summary.json || exit 1
for ab in "2 2" "3 1" "1 1" "2 0"; do set -- $ab
ATR_HYB_A=$1 ATR_HYB_B=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc > $O/sweep_c3_$1_$2.json || exit 1
done
echo done
