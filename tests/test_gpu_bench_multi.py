"""bench.py's N-rank path on the real kernels (one GPU, gloo, host-staged exchange): the cost plan,
the graded cell order (atr_set_cell_plan classes), the packed shard renders, the frame exchange --
3 bytes per pixel (atr_pack_bgr on each rank, atr_scatter_bgr on rank 0: the code the 8-GPU RCCL run
uses, with the bytes staged through the host) or the u32 framebuffer --, frame assembly and the
per-tile ray_casts reduction, on c3 (HYBRID) and c4 (the path engine). Round 6: the masked exchange
(the default: atr_pack_bgr_masked streams, their sizes sent first, atr_scatter_bgr_masked on rank 0). --check renders every timed frame again as one full-frame launch and
counts mismatching pixels and tile sums: it must be 0 (the reordered block list once broke the
per-tile counters). Two ranks, one subprocess tree (bench.py starts its ranks itself).
Needs an MI355X (-m gpu)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("config,order,exchange", [("c3", "graded", "masked"), ("c3", "list", "bgr"),
                                                   ("c3", "graded", "bgrx"), ("c4", "graded", "masked"),
                                                   ("c3", "graded", "bgr")])
def test_bench_two_ranks_frames_exact(config, order, exchange):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, ATR_DIST_BACKEND="gloo")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    steps, warm = ("6", "2") if config == "c3" else ("2", "1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", config,
                        "--steps", steps, "--warmup", warm, "--check", "--cell-order", order, "--exchange", exchange,
                        "--no-pmc", "--no-cpu-baseline", "--no-prep", "--no-steady"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert d["n_gpus"] == 2 and d["check_mismatched_pixels"] == 0
    assert d["config"]["exchange"].startswith(exchange + " ")
    assert sum(d["config"]["shard_pixels"]) == 1920 * 1080
