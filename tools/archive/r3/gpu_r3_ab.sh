#!/bin/bash
# Quick A/B of the current build: GPU suite, then c3 at the driver's shape (PMC child for VALU) and c4.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3ab
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in $(seq 1 ${AB_C3_REPS:-2}); do
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-prep --no-steady > $O/c3_$rep.json 2> $O/c3_$rep.err || { tail -20 $O/c3_$rep.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c3_$rep.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c3', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'], r.get('valu',{}).get('wave_insts_per_frame'), r.get('frac'))"
done
timeout -k 10 300 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady > $O/c4.json 2> $O/c4.err || { tail -20 $O/c4.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/c4.json').read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
if [ -n "$AB_C4_VARIANTS" ]; then
  for v in $AB_C4_VARIANTS; do
    timeout -k 10 300 python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady --variant-code $v > $O/c4_$v.json 2> $O/c4_$v.err || { tail -20 $O/c4_$v.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c4_$v.json').read().strip().splitlines()[-1]); print('c4 variant $v', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
  done
fi
if [ -n "$AB_SIM_RANKS" ]; then
  for r in $AB_SIM_RANKS; do
    timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep --no-steady --sim-world 8 --sim-rank $r > $O/c3sim_$r.json 2> $O/c3sim_$r.err || { tail -20 $O/c3sim_$r.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c3sim_$r.json').read().strip().splitlines()[-1]); print('c3 shard $r', d['value'], d['ms_per_step'], d['single_frame']['latency_ms'])"
  done
fi
