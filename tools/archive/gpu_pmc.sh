#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) over a short kprof run.
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1
VAR=${PMC_VARIANT:-occ6}
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d gpurun_out/pmc/g$i -o p -- python3 tools/kprof.py --config ${PMC_CONFIG:-c3} --rounds 1 --iters 2 --variants $VAR > gpurun_out/pmc/g$i.log 2>&1
  rc=$?; echo "group $i ($grp) rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
done <<< "$PMC_GROUPS"
