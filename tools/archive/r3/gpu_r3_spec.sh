#!/bin/bash
# Speculative leaf steps: GPU suite on the new build, then A/B against the same build without them
# (ATRAY_LIB=atray_amd/_lib/exp/nospec.so): c3 driver shape + single-frame latency, two c3 8-way
# shards, c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3sp
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
b() {
  timeout -k 10 300 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:2}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
for rep in 1 2; do
  for lib in spec nospec; do
    L=""; [ $lib = nospec ] && L=atray_amd/_lib/exp/nospec.so
    export ATRAY_LIB=$L
    b c3_${lib}_$rep --steps 20 --warmup 5
    b c3s7_${lib}_$rep --steps 20 --warmup 5 --sim-world 8 --sim-rank 7
    b c3s2_${lib}_$rep --steps 20 --warmup 5 --sim-world 8 --sim-rank 2
    [ $rep = 1 ] && b c4_${lib} --config c4 --steps 8 --warmup 2
  done
done
