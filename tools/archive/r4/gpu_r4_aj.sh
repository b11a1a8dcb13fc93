#!/bin/bash
# 32-slot clusters (experiment build c32: 256-B cluster blocks, 32-bit candidate masks): parity on
# c32, then c3 / c4 against HEAD (16), and c32 at cluster_size 24.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4aj
mkdir -p $O
ATRAY_LIB=atray_amd/_lib/exp/c32.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cluster.py -x -q --timeout 200 --timeout-method thread -k "not test_tuning_changes_no_output" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() {  # name, args
  timeout -k 10 200 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])" || exit 1
}
for rep in 1 2 3; do
run h16_c3_$rep --steps 20 --warmup 5
ATRAY_LIB=atray_amd/_lib/exp/c32.so run c32_c3_$rep --steps 20 --warmup 5
ATRAY_LIB=atray_amd/_lib/exp/c32.so run c24_c3_$rep --steps 20 --warmup 5 --tuning cluster_size=24
done
run h16_c4 --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/c32.so run c32_c4 --config c4 --steps 8 --warmup 2
ATRAY_LIB=atray_amd/_lib/exp/c32.so run c24_c4 --config c4 --steps 8 --warmup 2 --tuning cluster_size=24
