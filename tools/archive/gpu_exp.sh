#!/bin/bash
# Kernel experiment pass: kprof of the default build and of an experiment build (EXP_LIB), then
# two PMC passes of the default cluster kernel (one counter group per rocprofv3 run).
export TMPDIR=/tmp
OUT=gpurun_out/${EXP_NAME:-exp}
mkdir -p $OUT
VAR=${EXP_VARIANTS:-cl}
timeout -k 10 200 python tools/kprof.py --config ${EXP_CONFIG:-c3} --variants $VAR --rounds 5 > $OUT/base.json 2> $OUT/base.err || exit 1
for L in $EXP_LIBS; do
  ATRAY_LIB=$PWD/build/$L.so timeout -k 10 200 python tools/kprof.py --config ${EXP_CONFIG:-c3} --variants $VAR --rounds 5 > $OUT/$L.json 2> $OUT/$L.err || exit 1
done
for EV in $EXP_ENVS; do
  env $EV timeout -k 10 200 python tools/kprof.py --config ${EXP_CONFIG:-c3} --variants $VAR --rounds 5 > $OUT/$EV.json 2> $OUT/$EV.err || exit 1
done
if [ -n "$EXP_PMC" ]; then
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES --kernel-trace --output-format csv -d $OUT/pmc1 -o p -- python3 tools/kprof.py --config c3 --rounds 1 --iters 2 --variants $VAR > $OUT/pmc1.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $OUT/pmc2 -o p -- python3 tools/kprof.py --config c3 --rounds 1 --iters 2 --variants $VAR > $OUT/pmc2.log 2>&1 || exit 1
fi
echo done
