#!/bin/bash
# FLAT diagnostics at HEAD (tools/flat_probe.py): work per ray, bounce-loop lane use, SIMD counters.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 300 python3 -u tools/flat_probe.py ${1:-16} > $O/flat_probe.jsonl 2> $O/flat_probe.err || { tail $O/flat_probe.err; exit 1; }
cat $O/flat_probe.jsonl
