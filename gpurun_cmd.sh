export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python tools/kprof.py --variants cl5,hyb5 --rounds 7 > $O/kp_c3.json || exit 1
python -c "
import json; d=json.load(open('$O/kp_c3.json')); print({k:(v['ms_median'],v['ms_min']) for k,v in d.items() if isinstance(v,dict)})"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3.json || exit 1
python -c "
import json; d=json.load(open('$O/bench_c3.json')); print('c3', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'], d['roofline']['traffic'])"
timeout -k 10 300 python bench.py --config c4 --steps 8 --warmup 1 --no-cpu-baseline --no-pmc --no-prep > $O/bench_c4.json || exit 1
python -c "
import json; d=json.load(open('$O/bench_c4.json')); print('c4', d['value'], d['ms_per_step'], d['single_frame']['kernel_ms'])"
echo done
