#!/bin/bash
# Round 3: one-frame latency probe (HYBRID, c3) + the default bench with its PMC passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 300 python3 -u tools/latency_probe.py > $O/latency.jsonl 2> $O/latency.err || { tail $O/latency.err; exit 1; }
cat $O/latency.jsonl | cut -c1-400
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 --cpu-seconds 4 > $O/bench_c3.json 2> $O/bench_c3.err || { tail $O/bench_c3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/bench_c3.json').read().strip().splitlines()[-1]); print(json.dumps(d['roofline'])); print(d['value'], d.get('steady_state'))"
echo all done
