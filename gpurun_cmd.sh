export TMPDIR=/tmp
mkdir -p gpurun_out/r2d
timeout -k 10 120 python tools/out_probe.py || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2d/pytest.log 2>&1 || { tail -30 gpurun_out/r2d/pytest.log; exit 1; }
tail -2 gpurun_out/r2d/pytest.log
OUT_DIR=r2d SHAPES="2x4 2x8 1x1" STEPS="20 48" bash tools/gpu_bench_sweep2.sh || exit 1
