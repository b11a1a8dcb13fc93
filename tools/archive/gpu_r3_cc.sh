#!/bin/bash
# Round 3: candidate compaction (CC) and slot-record (AoS) A/B -- parity of the CC schedules
# (96 FLAT_CC, 97 HYBRID_CC), FLAT vs FLAT_CC on the c4 shape, HYBRID vs HYBRID_CC on c3 (one
# frame and the driver's shape), each with the product library and the AoS experiment build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
ATR_TEST_VARIANTS=96,97 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cluster.py \
  -x -q --timeout 200 --timeout-method thread > $O/pytest_cc.log 2>&1 || { tail -30 $O/pytest_cc.log; exit 1; }
tail -2 $O/pytest_cc.log
timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 96 > $O/flat_probe.jsonl 2> $O/flat_probe.err || exit $?
ATRAY_LIB=atray_amd/_lib/exp/aos.so timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 96 > $O/flat_probe_aos.jsonl 2> $O/flat_probe_aos.err || exit $?
grep -h '"bounces": 5' $O/flat_probe.jsonl $O/flat_probe_aos.jsonl | cut -c1-140
for lib in prod aos prod aos; do
  for v in 9 97 98; do
    L=""; [ $lib = aos ] && L=atray_amd/_lib/exp/aos.so
    ATRAY_LIB=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --variant-code $v > $O/bench_c3_${lib}_v$v.json 2> $O/bench_c3_${lib}_v$v.err || exit $?
    python3 -c "import json,sys; d=json.loads(open('$O/bench_c3_${lib}_v$v.json').read().strip().splitlines()[-1]); print('$lib $v', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d.get('steady_state'))"
  done
done
PHASES=1 ATRAY_LIB=atray_amd/_lib/exp/phase.so timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 > $O/flat_probe_phase.jsonl 2> $O/flat_probe_phase.err || exit $?
echo all done
