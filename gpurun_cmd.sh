export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
for ab in "2 2" "2 1" "2 0" "3 1" "2 3" "3 2" "1 1"; do set -- $ab
  ATR_HYB_A=$1 ATR_HYB_B=$2 timeout -k 10 120 python tools/kprof.py --variants cl,hyb --rounds 7 > $O/kp_c3_$1_$2.json || exit 1
done
for ab in "2 2" "4 4" "8 8" "1 0"; do set -- $ab
  ATR_HYB_A=$1 ATR_HYB_B=$2 timeout -k 10 200 python tools/kprof.py --config c4 --variants flat,hyb --rounds 2 --iters 1 > $O/kp_c4_$1_$2.json || exit 1
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --variant cl > $O/bench_c3_cl.json || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --variant hyb > $O/bench_c3_hyb.json || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --variant cl > $O/bench_c3_cl2.json || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --variant hyb > $O/bench_c3_hyb2.json || exit 1
echo done
