#!/bin/bash
# bench.py launch-shape sweep: per-step time at the driver's 20 steps and at 48 for a set of
# (streams, frames per launch) shapes; no PMC / CPU legs.
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-sweep}
mkdir -p $O
for shape in ${SHAPES:-1x1 1x8 2x8 2x4 4x4 1x16 2x16}; do
  set -- ${shape/x/ }
  for K in ${STEPS:-20 48}; do
    timeout -k 10 120 python bench.py --steps $K --warmup 8 --streams $1 --frames-per-launch $2 --no-cpu-baseline --no-pmc --no-prep ${BENCH_ARGS} > $O/s$1_f$2_k$K.log 2>&1 || exit 1
    python -c "import json,sys,os; d=[json.loads(l) for l in open('$O/s$1_f$2_k$K.log') if l.startswith('{')][-1]; print('R='+os.environ.get('ATR_FRAME_ROTATE','')+' S=$1 F=$2 K=$K', d['ms_per_step'], d['value'], d['single_frame']['kernel_ms'])"
  done
done
