#!/bin/bash
# Direction binning A/B on c4 (path_bin 0 / 1), parity of the tuning test (includes path_bin=1).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "tuning_changes or multibounce" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for t in "path_bin=0" "path_bin=1" "path_bin=0" "path_bin=1"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$t -o c4 -- python3 tools/path_probe.py c4 0 3 "$t" > $O/trace_$t.log 2>&1 || { tail -20 $O/trace_$t.log; exit 1; }
  echo "$t"; grep "^frame" $O/trace_$t.log | tail -2
  find $O/trace_$t -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-130 | head -5 | tail -4
done
