#!/bin/bash
# Round 3: FLAT_LO (LDS leaf buffer + private-memory path stash: 22.5 KB LDS) at 4/5/6 waves/SIMD
# against the product FLAT on the c4 shape; parity of FLAT_LO.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
ATR_TEST_VARIANTS=101,102,103 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
  --timeout-method thread -k "multibounce or tuning or frames or axis or spheres or ragged" > $O/pytest_lo.log 2>&1 || { tail -30 $O/pytest_lo.log; exit 1; }
tail -2 $O/pytest_lo.log
for rep in 1 2; do
timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 101 102 103 > $O/flat_probe_$rep.jsonl 2> $O/flat_probe_$rep.err || exit $?
grep -h '"bounces": 5' $O/flat_probe_$rep.jsonl | cut -c1-100
done
echo all done
