#!/bin/bash
# One-GPU rehearsal of the multi-GPU bench path: N=1 bench with the frame check, an N-rank
# gloo run on the same GPU (host-staged gather) with the frame check, and the shard balance
# measurement (each rank's shard timed alone). Each GPU step has its own limit.
export TMPDIR=/tmp
mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --check --no-pmc --no-cpu-baseline > gpurun_out/bench_n1_check.log 2>&1
rc=$?; echo "bench_n1_rc=$rc"; tail -1 gpurun_out/bench_n1_check.log; if crash $rc; then exit $rc; fi
for N in ${REHEARSE:-2 4}; do
  ATR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 5 --warmup 2 --check --no-pmc --no-cpu-baseline > gpurun_out/bench_gloo_n$N.log 2>&1
  rc=$?; echo "bench_gloo_n${N}_rc=$rc"; grep '^{' gpurun_out/bench_gloo_n$N.log | tail -1; if crash $rc; then exit $rc; fi
done
timeout -k 10 400 python tools/shard_balance.py ${BAL_ARGS} > gpurun_out/shard_balance.json 2> gpurun_out/shard_balance.err
rc=$?; echo "balance_rc=$rc"
