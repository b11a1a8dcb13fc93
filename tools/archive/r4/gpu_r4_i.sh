#!/bin/bash
# Mirror-once examine (bounce 7-wave spills 58 -> 43 dwords): parity subset, c4 kernel times at
# bounce occupancy 7 / 6 / 5.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread \
  -k "multibounce or ragged or spheres or variants_agree" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for occ in 7 6 5; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4_$occ -o c4 -- python3 tools/path_probe.py c4 0 3 "path_bounce_occ=$occ" > $O/trace_c4_$occ.log 2>&1 || { tail -20 $O/trace_c4_$occ.log; exit 1; }
  echo "bounce occ $occ"; grep "^frame" $O/trace_c4_$occ.log | tail -1
  find $O/trace_c4_$occ -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-130 | head -3 | tail -2
done
