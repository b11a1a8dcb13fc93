export TMPDIR=/tmp
O=gpurun_out/r2h
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --check --no-pmc --no-cpu-baseline > $O/n1.log 2>&1 || { tail $O/n1.log; exit 1; }
grep '^{' $O/n1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N1', d['value'], d['ms_per_step'], d.get('check_mismatched_pixels'), d['config']['frames_per_launch'], d['total_ray_casts_per_frame'])"
for N in 2 4; do
  ATR_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus $N --steps 12 --warmup 4 --check --no-pmc --no-cpu-baseline > $O/gloo_n$N.log 2>&1 || { tail -20 $O/gloo_n$N.log; exit 1; }
  grep '^{' $O/gloo_n$N.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('N$N', d['n_gpus'], d['value'], d['check_mismatched_pixels'], d['config']['frames_per_launch'], d['total_ray_casts_per_frame'], d['config']['shard_pixels'])"
done
