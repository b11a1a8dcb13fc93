#!/bin/bash
# A/B of runtime knobs on the c3 bench: AB="name|ENV=.. ENV2=..|bench args" lines. Optional
# pytest pass first (PYTEST_K, PYTEST_ENV).
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-ab}
mkdir -p $O
if [ -n "$PYTEST_K" ]; then
env $PYTEST_ENV timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$PYTEST_K" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
fi
while IFS='|' read -r n e a; do
  [ -z "$n" ] && continue
  env $e timeout -k 10 200 python bench.py --no-pmc --no-cpu-baseline --no-prep $a > $O/$n.log 2>&1 || { tail -20 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$n', d['value'], d['ms_per_step'], c['launches'], d['single_frame']['kernel_ms'], c.get('launch_render_done_ms'))"
done <<< "${AB:-$(cat ${AB_FILE:-/dev/null})}"
echo done
