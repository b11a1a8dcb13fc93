export TMPDIR=/tmp
O=gpurun_out/r02s
mkdir -p $O
for K in 20 48 20 48; do
timeout -k 10 120 python bench.py --steps $K --warmup 5 --no-cpu-baseline --no-pmc > $O/b_k$K.json || exit 1
python -c "
import json; d=json.load(open('$O/b_k$K.json')); print('K=$K', d['value'], d['ms_per_step'], d['config']['launches'])"
done
echo done
