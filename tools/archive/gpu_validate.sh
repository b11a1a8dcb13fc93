#!/bin/bash
# GPU-box validation of a kernel change: the full -m gpu parity suite, then kernel timings of the
# CLUSTER and PERSIST schedules on c3 (primary) and c3 at 4 spp x 5 bounces. Each GPU step has
# its own time limit; a failing step ends the script.
export TMPDIR=/tmp
mkdir -p gpurun_out/val
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/val/pytest_gpu.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/val/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/kprof.py --config c3 --variants cl,cl4,ps > gpurun_out/val/kprof_c3.json 2> gpurun_out/val/kprof_c3.err || exit 1
timeout -k 10 300 python tools/kprof.py --config c3 --spp 4 --bounces 5 --rounds 3 --iters 2 --variants cl,ps \
  > gpurun_out/val/kprof_c3_s4b5.json 2> gpurun_out/val/kprof_c3_s4b5.err || exit 1
python tools/show_kprof.py gpurun_out/val
