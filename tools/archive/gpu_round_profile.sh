#!/bin/bash
# The committed measurement set (GPU box): the default bench line (roofline PMC passes and the
# CPU baseline included), rocprofv3 kernel stats of the same bench with one frame in flight (so
# each launch's duration is its own), the multi-bounce bench (c4 shape), and a 2-rank gloo
# rehearsal of the multi-GPU path with the frame check. Each GPU step has its own time limit.
export TMPDIR=/tmp
O=gpurun_out/prof
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || exit 1
grep '^{' $O/bench_c3.log > $O/bench_c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rocprof -o bench -- \
  python3 bench.py --steps 20 --warmup 3 --streams 1 --frames-per-launch 1 --no-cpu-baseline --no-pmc > $O/rocprof_bench.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --config c4 --steps 3 --warmup 1 --no-pmc --no-cpu-baseline > $O/bench_c4.log 2>&1 || exit 1
grep '^{' $O/bench_c4.log > $O/bench_c4.json
ATR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --check --no-pmc \
  --no-cpu-baseline > $O/bench_gloo_n2.log 2>&1 || exit 1
grep '^{' $O/bench_gloo_n2.log > $O/bench_gloo_n2.json
echo done
