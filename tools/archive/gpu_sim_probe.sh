#!/bin/bash
# Per-rank render side of N-GPU runs (bench.py --sim-world) and N=1 tile-list variants.
# RUNS: "name|args" lines (default set below).
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-simp}
mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 120 python bench.py --no-pmc --no-cpu-baseline --no-prep "$@" > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$n', d['value'], d['ms_per_step'], c['launches'], c['plan'], d['single_frame']['kernel_ms'])"
}
if [ -n "$RUNS" ]; then
  while IFS='|' read -r n a; do [ -n "$n" ] && run $n $a; done <<< "$RUNS"
else
for r in 0 1 2 3 4 5 6 7; do run s8r$r --sim-world 8 --sim-rank $r --steps 20 --warmup 5; done
for r in 0 1 2 3 4 5 6 7; do run s8r${r}_f5 --sim-world 8 --sim-rank $r --steps 20 --warmup 5 --frames-per-launch 5; done
run s2r0 --sim-world 2 --sim-rank 0 --steps 20 --warmup 5
run s2r1 --sim-world 2 --sim-rank 1 --steps 20 --warmup 5
run s2r0_f5 --sim-world 2 --sim-rank 0 --steps 20 --warmup 5 --frames-per-launch 5
run s2r1_f5 --sim-world 2 --sim-rank 1 --steps 20 --warmup 5 --frames-per-launch 5
fi
echo done
