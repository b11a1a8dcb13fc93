#!/bin/bash
# Round 4, first look at the sample-parallel path engine: the multi-bounce parity goldens on every
# variant, then c4 bench lines (PATHS default, FLAT for comparison) and an occupancy A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "multibounce or ragged or frames_per_launch or spheres" > $O/pytest_mb.log 2>&1 || { tail -40 $O/pytest_mb.log; exit 1; }
tail -1 $O/pytest_mb.log
B="python3 bench.py --config c4 --steps 8 --warmup 2 --no-pmc --no-cpu-baseline --no-prep --no-steady"
timeout -k 10 200 $B > $O/c4_paths.json 2> $O/c4_paths.err || { tail -20 $O/c4_paths.err; exit 1; }
tail -c 600 $O/c4_paths.json
for t in "path_camera_occ=6,path_bounce_occ=6" "path_camera_occ=5,path_bounce_occ=5" "path_camera_occ=7,path_bounce_occ=5"; do
  timeout -k 10 200 $B --tuning $t > $O/c4_paths_$t.json 2> $O/c4_paths_$t.err || { tail -20 $O/c4_paths_$t.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['single_frame'])" $O/c4_paths_$t.json $t
done
timeout -k 10 300 $B --variant flat > $O/c4_flat.json 2> $O/c4_flat.err || { tail -20 $O/c4_flat.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('flat', d['value'], d['ms_per_step'], d['single_frame'])" $O/c4_flat.json
