#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "frame_plan or tuning or bgr" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u tools/plan_probe.py > $O/plan.jsonl 2> $O/plan.err || { tail $O/plan.err; exit 1; }
cat $O/plan.jsonl
echo all done
