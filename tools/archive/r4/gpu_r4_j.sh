#!/bin/bash
# Diagnostic build: per-level work, phase clocks and SIMD counters of the path engine on c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
ATRAY_LIB=atray_amd/_lib/diag/libatray_hip.so timeout -k 10 300 python3 tools/path_counters.py > $O/counters_diag.jsonl 2> $O/counters_diag.err || { tail -20 $O/counters_diag.err; exit 1; }
cat $O/counters_diag.jsonl
