#!/bin/bash
# Round 6: the 2^29-path batch cliff. c4, 4 frames in one launch: 2^28-path batches
# (two batches) against 2^29 (one batch, a 77-GB workspace), experiment library b29
# (tools/build_exp.sh "b29:-DATR_MAX_BATCH_LOG2=29"). Kernel traces, then one PMC pass of the
# address-translation counters this rocprofv3 lists for the TCP/UTCL blocks, for each batch size.
# usage: gpu_r6_cliff.sh OUTDIR
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
( while sleep 30; do date +%s >> $O/heartbeat; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o -E "TCP_UTCL1_[A-Z_]+(_sum)?|UTCL2_[A-Z_]+|TCP_TCP_TA_DATA_STALL_CYCLES_sum|TD_TD_BUSY_sum" $O/counters.txt | sort -u > $O/tlb_counters.txt || true
C=$(grep -E "^TCP_UTCL1_TRANSLATION_MISS_sum$|^TCP_UTCL1_TRANSLATION_HIT_sum$|^TCP_UTCL1_PERMISSION_MISS_sum$|^TCP_UTCL1_REQUEST_sum$" $O/tlb_counters.txt | head -4 | tr '\n' ' ')
echo "counters: $C"
for lg in 28 29; do
  A="--config c4 --steps 4 --warmup 1 --frames-per-launch 4 --streams 1 --no-pmc --no-cpu-baseline --no-prep --no-steady --tuning path_batch_log2=$lg"
  ATRAY_LIB=atray_amd/_lib/exp/b29.so timeout -k 10 300 python3 bench.py $A > $O/b$lg.json 2> $O/b$lg.err || { tail -5 $O/b$lg.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/b$lg.json').read().strip().splitlines()[-1]); print('b$lg', d['value'], d['ms_per_step'])"
  ATRAY_LIB=atray_amd/_lib/exp/b29.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_b$lg -o run -- python3 bench.py $A > $O/trace_b$lg.log 2>&1 || { tail -5 $O/trace_b$lg.log; exit 1; }
  if [ -n "$C" ]; then
    ATRAY_LIB=atray_amd/_lib/exp/b29.so timeout -s KILL 300 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_b$lg -o run -- python3 bench.py $A --pmc-child > $O/pmc_b$lg.log 2>&1 || { tail -5 $O/pmc_b$lg.log; exit 1; }
  fi
done
echo all done
