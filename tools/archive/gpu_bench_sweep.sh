#!/bin/bash
# bench.py throughput sweep on one GPU: schedule x frames in flight (no PMC / CPU legs).
# Settings from the environment or build/bench_sweep.env: BS_VARIANTS, BS_STREAMS, BS_CONFIG.
export TMPDIR=/tmp
[ -f build/bench_sweep.env ] && . build/bench_sweep.env
mkdir -p gpurun_out/bsweep
for F in ${BS_FPL:-1}; do
for q in ${BS_QUEUES:-0}; do
for v in ${BS_VARIANTS:-cl ps}; do
  for s in ${BS_STREAMS:-1 2 3}; do
    L=gpurun_out/bsweep/${BS_CONFIG:-c3}_${v}_s${s}_q${q}_f$F.log
    timeout -k 10 300 python bench.py --config ${BS_CONFIG:-c3} --variant $v --streams $s --hw-queues $q --frames-per-launch $F --steps 48 \
      --warmup 3 --no-pmc --no-cpu-baseline > $L 2>&1 || exit 1
    grep '^{' $L | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 's=$s', 'q=$q', 'F=$F', d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'kernel', d['roofline']['kernel_ms'])"
  done
done
done
done
