#!/bin/bash
# Near-first passes for bounce rays: multi-bounce parity, c4 frame times per bounce occupancy,
# per-level counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "multibounce or ragged or spheres or variants_agree" > $O/pytest_mb.log 2>&1 || { tail -40 $O/pytest_mb.log; exit 1; }
tail -1 $O/pytest_mb.log
for occ in 7 6 5; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4_$occ -o c4 -- python3 tools/path_probe.py c4 0 3 "path_bounce_occ=$occ" > $O/trace_c4_$occ.log 2>&1 || { tail -20 $O/trace_c4_$occ.log; exit 1; }
  echo "bounce occ $occ"; grep "^frame" $O/trace_c4_$occ.log
  find $O/trace_c4_$occ -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-130 | head -4
done
ATRAY_LIB=atray_amd/_lib/diag/libatray_hip.so timeout -k 10 300 python3 tools/path_counters.py > $O/counters_diag.jsonl 2> $O/counters_diag.err || { tail -20 $O/counters_diag.err; exit 1; }
cat $O/counters_diag.jsonl | cut -c1-400
