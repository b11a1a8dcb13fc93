#!/bin/bash
# PERSIST tuning sweep (GPU box): the default build and the experiment builds of
# tools/build_exp.sh on c3 (primary) and c4-shaped multi-bounce (kprof, CLUSTER beside PERSIST).
# Settings: SWEEP_NAME, SWEEP_LIBS, SWEEP_MB from the environment or build/sweep.env.
[ -f build/sweep.env ] && . build/sweep.env
EXP_NAME=${SWEEP_NAME:-sweep} EXP_VARIANTS=${SWEEP_VARIANTS:-cl,ps} EXP_PMC=$SWEEP_PMC EXP_LIBS="$SWEEP_LIBS" bash tools/gpu_exp.sh || exit 1
if [ -n "$SWEEP_MB" ]; then
  mkdir -p gpurun_out/${SWEEP_NAME:-sweep}_mb
  for L in "" $SWEEP_LIBS; do
    lib=${L:+$PWD/build/$L.so}
    ATRAY_LIB=$lib timeout -k 10 300 python tools/kprof.py --config c3 --spp 4 --bounces 5 --rounds 3 --iters 2 \
      --variants cl,ps > gpurun_out/${SWEEP_NAME:-sweep}_mb/${L:-base}.json 2> gpurun_out/${SWEEP_NAME:-sweep}_mb/${L:-base}.err || exit 1
  done
fi
echo done
