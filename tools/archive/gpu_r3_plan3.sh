#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frame_plan or tuning" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in prod s2 s4a; do
  L=""; [ $lib != prod ] && L=atray_amd/_lib/exp/$lib.so
  ATRAY_LIB=$L timeout -k 10 300 python3 -u tools/plan_probe.py > $O/plan_$lib.jsonl 2> $O/plan_$lib.err || { tail $O/plan_$lib.err; exit 1; }
  echo $lib; grep '"frame_plan": 1' $O/plan_$lib.jsonl | cut -c1-120
done
grep '"frame_plan": 0' $O/plan_prod.jsonl | cut -c1-120
echo all done
