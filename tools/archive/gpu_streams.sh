#!/bin/bash
# Frames in flight: N=1 bench at 1/2/3 streams (frame check on), shard balance with 1 and 3
# streams (per-rank shard time when S frames overlap), gloo N=2 rehearsal with the check.
export TMPDIR=/tmp
mkdir -p gpurun_out
crash() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for S in 1 2 3 4; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --streams $S --check --no-pmc --no-cpu-baseline > gpurun_out/bench_s$S.log 2>&1
  rc=$?; echo "bench_s${S}_rc=$rc"; grep '^{' gpurun_out/bench_s$S.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('check_mismatched_pixels'))"; if crash $rc; then exit $rc; fi
done
ATR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 6 --warmup 2 --streams 3 --check --no-pmc --no-cpu-baseline > gpurun_out/bench_gloo_s3.log 2>&1
rc=$?; echo "gloo_rc=$rc"; grep '^{' gpurun_out/bench_gloo_s3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('check', d.get('check_mismatched_pixels'))"; if crash $rc; then exit $rc; fi
for S in 1 3; do
  timeout -k 10 300 python tools/shard_balance.py --plans lpt --sides 64 --streams $S > gpurun_out/shard_balance_s$S.json 2> gpurun_out/shard_balance_s$S.err
  rc=$?; echo "balance_s${S}_rc=$rc"; if crash $rc; then exit $rc; fi
done
