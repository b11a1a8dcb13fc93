#!/bin/bash
# Multi-GPU path on one GPU (round 2): N=1 bench with the frame check, gloo rehearsals of the
# exact-size gather + per-tile ray_casts reduction (2 and 4 ranks on one GPU, frame check), the
# spawn path (bench.py --gpus 2 without a launcher), and every rank's shard of the N = 2, 4, 8
# plans rendered alone in the benched launch shape (--sim-world: the render side of an N-GPU run).
export TMPDIR=/tmp
O=gpurun_out/${OUT_DIR:-multi}
mkdir -p $O
if [ -n "$PYTEST_K" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$PYTEST_K" > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --check --no-pmc --no-cpu-baseline > $O/bench_n1_check.log 2>&1 || { tail -20 $O/bench_n1_check.log; exit 1; }
grep '^{' $O/bench_n1_check.log | cut -c1-300
for N in 2 4; do
  ATR_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 11 --warmup 3 --check --no-pmc --no-cpu-baseline > $O/bench_gloo_n$N.log 2>&1 || { tail -30 $O/bench_gloo_n$N.log; exit 1; }
  grep '^{' $O/bench_gloo_n$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('gloo', d['n_gpus'], d['check_mismatched_pixels'], d['total_ray_casts_per_frame'], d['config']['launches'])"
done
ATR_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --check --no-pmc --no-cpu-baseline > $O/bench_spawn_n2.log 2>&1 || { tail -30 $O/bench_spawn_n2.log; exit 1; }
grep '^{' $O/bench_spawn_n2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('spawn', d['n_gpus'], d['check_mismatched_pixels'])"
for N in ${SIM_WORLDS:-8 4 2}; do
  for ((r = 0; r < N; r++)); do
    timeout -k 10 120 python bench.py --sim-world $N --sim-rank $r --steps ${SIM_STEPS:-20} --warmup 5 --no-pmc --no-cpu-baseline --no-prep > $O/sim_${N}_$r.log 2>&1 || { tail -20 $O/sim_${N}_$r.log; exit 1; }
    grep '^{' $O/sim_${N}_$r.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('sim', $N, $r, d['value'], d['ms_per_step'], d['config']['launches'], d['config']['shard_pixels'][$r])"
  done
done
echo done
