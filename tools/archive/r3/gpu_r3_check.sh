#!/bin/bash
# Round 3 check at HEAD: GPU suite + smoke, the driver's bench command (PMC child + CPU baseline),
# and a rocprofv3 kernel trace of the same command. Output under gpurun_out/r3c.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
tail -c 600 $O/bench_driver.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_driver -o t -- python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/bench_traced.json 2> $O/bench_traced.err || { tail -20 $O/bench_traced.err; exit 1; }
echo done
