#!/bin/bash
# Round 5 set B: the bounce rays' bounding-sphere gate. Parity (every multi-bounce test of the
# suite), then c4 A/B against the experiment build without the gate (ATRAY_LIB), interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${2:-r5b}
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
if [ "${1:-full}" = "full" ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head -20; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
fi
run() {  # name, timeout, lib, args
  ATRAY_LIB=$3 timeout -k 10 $2 python3 bench.py --no-pmc --no-cpu-baseline --no-prep --no-steady "${@:4}" > $O/$1.json 2> $O/$1.err || { tail -5 $O/$1.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
}
X=atray_amd/_lib/exp/nosphere.so
P=atray_amd/_lib/libatray_hip.so
for i in 1 2; do
  run c4_sph_$i 300 $P --config c4 --steps 8 --warmup 2
  run c4_nosph_$i 300 $X --config c4 --steps 8 --warmup 2
done
run c5_sph 600 $P --config c5 --steps 2 --warmup 1
run c3_sph 120 $P --steps 20 --warmup 5
echo all done
