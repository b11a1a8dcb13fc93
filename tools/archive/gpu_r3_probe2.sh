#!/bin/bash
# Round 3: SIMD-efficiency counters of FLAT (c4 shape) and HYBRID (c3), plus phase clocks.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3b
mkdir -p $O
timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 > $O/flat_probe.jsonl 2> $O/flat_probe.err || exit $?
PHASES=1 ATRAY_LIB=atray_amd/_lib/exp/phase.so timeout -k 10 300 python3 -u tools/flat_probe.py 4 8 > $O/flat_probe_phase.jsonl 2> $O/flat_probe_phase.err || exit $?
echo probe2 done
