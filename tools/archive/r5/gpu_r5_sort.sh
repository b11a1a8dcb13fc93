#!/bin/bash
# Round 5: the queue sort (tuning path_sort_bits). The tuning parity test, c4 A/B of the sort
# settings (tools/gpu_r5_ab2.sh), then the path engine's per-level work counters with and without
# the sort (diagnostic build).
# usage: gpu_r5_sort.sh OUTDIR "variant ..." [counters]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "tuning_changes_no_output" --timeout 300 --timeout-method thread > $O/pytest_sort.log 2>&1 || { tail -40 $O/pytest_sort.log; exit 1; }
tail -1 $O/pytest_sort.log
bash tools/gpu_r5_ab2.sh $1 "$2" "c4" || exit 1
if [ "${3:-}" = "counters" ]; then
  for b in 0 4; do
    SORT=$b ATRAY_LIB=atray_amd/_lib/diag/libatray_hip.so timeout -k 10 300 python3 -u tools/path_counters.py > $O/counters_sort$b.jsonl 2> $O/counters_sort$b.err || { tail -5 $O/counters_sort$b.err; exit 1; }
    echo "counters sort $b done"
  done
fi
echo all done
