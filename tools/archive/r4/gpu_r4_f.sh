#!/bin/bash
# Register-stack near-first passes: multi-bounce parity, c4 kernel times, per-level counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread \
  -k "multibounce or ragged or spheres or variants_agree or tuning or c4_full" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o c4 -- python3 tools/path_probe.py c4 0 3 > $O/trace_c4.log 2>&1 || { tail -20 $O/trace_c4.log; exit 1; }
grep "^frame" $O/trace_c4.log | tail -2
find $O/trace_c4 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-130 | head -4 | tail -3
timeout -k 10 200 python3 tools/path_counters.py > $O/counters.jsonl 2> $O/counters.err || { tail -20 $O/counters.err; exit 1; }
cut -c1-300 $O/counters.jsonl
