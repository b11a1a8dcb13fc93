#!/bin/bash
# The whole GPU suite and smoke at HEAD.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4full
mkdir -p $O
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAIL|Error|error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
grep -E "PASSED|FAILED" $O/pytest_gpu.log | awk '{print $NF, $0}' | sort | tail -3
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
