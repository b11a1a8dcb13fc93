#!/bin/bash
# c4 after the coalesced resolve; per-level work counters of the path engine (product COUNT build,
# then the diagnostic build's phase clocks).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o c4 -- python3 tools/path_probe.py c4 0 3 > $O/trace_c4.log 2>&1 || { tail -20 $O/trace_c4.log; exit 1; }
grep "^frame" $O/trace_c4.log
find $O/trace_c4 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-160 | head -5
timeout -k 10 200 python3 tools/path_counters.py > $O/counters.jsonl 2> $O/counters.err || { tail -20 $O/counters.err; exit 1; }
cat $O/counters.jsonl
ATRAY_LIB=atray_amd/_lib/diag/libatray_hip.so timeout -k 10 300 python3 tools/path_counters.py > $O/counters_diag.jsonl 2> $O/counters_diag.err || { tail -20 $O/counters_diag.err; exit 1; }
cat $O/counters_diag.jsonl
