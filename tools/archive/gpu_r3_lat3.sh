#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "cell_plan or packed or bgr or frames" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python3 -u tools/latency_probe.py > $O/latency.jsonl 2> $O/latency.err || { tail $O/latency.err; exit 1; }
grep plan $O/latency.jsonl; head -1 $O/latency.jsonl
echo all done
