#!/bin/bash
# c4 with the path workspace sized for the multi-frame batches; kernel trace of c4 frames; the
# bench's PMC passes on the path engine.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
B="python3 bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline --no-prep --no-steady"
timeout -k 10 200 $B --no-pmc > $O/c4_paths.json 2> $O/c4_paths.err || { tail -20 $O/c4_paths.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('c4', d['value'], d['ms_per_step'], d['single_frame'], d['roofline']['launch_ms'])" $O/c4_paths.json
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o c4 -- python3 tools/path_probe.py c4 0 3 > $O/trace_c4.log 2>&1 || { tail -20 $O/trace_c4.log; exit 1; }
cat $O/trace_c4.log | tail -4
find $O/trace_c4 -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-220
timeout -k 10 500 $B > $O/c4_pmc.json 2> $O/c4_pmc.err || { tail -20 $O/c4_pmc.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('c4 pmc', d['value'], {k: r.get(k) for k in ('traffic_per_frame','traffic_per_traced_ray','frac','pmc_frames','valu','l2_hit_rate','pmc_note')})" $O/c4_pmc.json
cp gpurun_out/bench_pmc/rows_c4.json $O/ || true
