#!/bin/bash
# Kernel traces of the N=1 bench and of one rank's shard (--sim-world 2) in the benched shape.
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-simtr}
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/n1 -o t -- python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep > $O/n1.log 2>&1 || { tail $O/n1.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/s2 -o t -- python3 bench.py --sim-world 2 --sim-rank 0 --steps 20 --warmup 5 --no-pmc --no-cpu-baseline --no-prep > $O/s2.log 2>&1 || { tail $O/s2.log; exit 1; }
grep '^{' $O/n1.log | cut -c1-200
grep '^{' $O/s2.log | cut -c1-200
echo done
