#!/bin/bash
# bench.py throughput sweep on one GPU: schedule x frames in flight (no PMC / CPU legs).
# Settings from the environment or build/bench_sweep.env: BS_VARIANTS, BS_STREAMS, BS_CONFIG.
export TMPDIR=/tmp
[ -f build/bench_sweep.env ] && . build/bench_sweep.env
mkdir -p gpurun_out/bsweep
for v in ${BS_VARIANTS:-cl ps}; do
  for s in ${BS_STREAMS:-1 2 3}; do
    timeout -k 10 300 python bench.py --config ${BS_CONFIG:-c3} --variant $v --streams $s --steps 30 --warmup 3 \
      --no-pmc --no-cpu-baseline > gpurun_out/bsweep/${BS_CONFIG:-c3}_${v}_s$s.log 2>&1 || exit 1
    grep '^{' gpurun_out/bsweep/${BS_CONFIG:-c3}_${v}_s$s.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', 's=$s', d['value'], 'Mrays/s', d['ms_per_step'], 'ms/frame', 'kernel', d['roofline']['kernel_ms'])"
  done
done
