export TMPDIR=/tmp
O=gpurun_out/r2g
mkdir -p $O
for cfg in "c4 67 4" "c4 68 4" "c4 66 4" "c5 67 1" "c5 68 1"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --config $1 --variant flat --variant-code $2 --frames-per-launch $3 --steps 2 --warmup 1 --no-pmc --no-cpu-baseline --no-prep > $O/b_$1_$2_$3.log 2>&1 || { tail -3 $O/b_$1_$2_$3.log; exit 1; }
  python -c "import json; d=[json.loads(l) for l in open('$O/b_$1_$2_$3.log') if l.startswith('{')][-1]; print('$cfg', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'])"
done
