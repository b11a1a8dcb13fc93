#!/bin/bash
# Round 3, first look at the multi-bounce kernel: FLAT lane use / work counters / bounce-limit
# timings (tools/flat_probe.py) and PMC groups of one c4-shaped launch (4 spp x 5 bounces).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3a
mkdir -p $O
timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 > $O/flat_probe.jsonl 2> $O/flat_probe.err || exit $?
OUT_DIR=r3a/pmc_c4 PMC_SPP=4 PMC_BOUNCES=5 PMC_VARIANT=8 bash tools/gpu_pmc2.sh || exit $?
# the same launch at 3 waves/SIMD (FLAT without scratch): FETCH/WRITE difference = spill traffic
for c in FETCH_SIZE WRITE_SIZE; do
  PMC_SPP=4 PMC_BOUNCES=5 PMC_VARIANT=67 timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace --output-format csv \
    -d $O/pmc_c4_occ3/$c -o p -- python3 tools/pmc_probe.py > $O/pmc_c4_occ3_$c.log 2>&1 || exit $?
done
echo probe done
