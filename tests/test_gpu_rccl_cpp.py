"""The reference-side multi-GPU flow in C++ over RCCL (tests/c/multi_gpu_exchange.cpp, built by
atray_amd/csrc/Makefile against include/atray.h and <rccl/rccl.h> only): rank 0's cost
calibration broadcast with ncclBroadcast, the balanced shard plan, a PACKED render of the rank's
tiles, per-tile ray_casts on the device, grouped ncclSend/ncclRecv of the pixels (u32 through
atr_unpack, or the masked stream through atr_scatter_bgr_masked after a sizes-first exchange) and
of the tile sums, assembly on rank 0 -- the renderer.cpp:403-471 surface without Python. At world
size 1 (one GPU per box here) rank 0 sends to itself through the same calls. The assembled C4 frame
must equal the oracle's whole frame (tests/golden/fullframe.json) and total_ray_casts the oracle's
sum; --check also compares it with a one-launch render on the same GPU.
The binary's usage path is CPU-only (test_multi_gpu_exchange_builds); the renders need an MI355X."""
import json
import os
import subprocess

import numpy as np
import pytest

from atray_amd.assets import asset_path
from tests.goldens import frame_digest, fullframe

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "atray_amd", "_lib", "multi_gpu_exchange")


def test_multi_gpu_exchange_builds():
    """Built and linked (make -C atray_amd/csrc); without arguments it prints its usage (exit 2)
    before touching a GPU."""
    assert os.path.exists(EXE), "make -C atray_amd/csrc"
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("exchange", ["u32", "masked"])
def test_cpp_rccl_flow_c4_matches_oracle(tmp_path, exchange):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    g = fullframe()["c4"]
    out = tmp_path / "frame.u32"
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    r = subprocess.run([EXE, asset_path("Dragon"), "1920", "1080", "64", "5", "--exchange", exchange,
                        "--out", str(out), "--check"], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr[-3000:] + r.stdout[-1000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["world"] == 1 and d["exchange"] == exchange
    assert d["check_mismatched_pixels"] == 0
    assert d["total_ray_casts"] == d["check_total_ray_casts"] == g["casts_sum"]
    img = np.fromfile(out, np.uint32).reshape(1080, 1920)
    assert frame_digest(img) == g["fb"]  # the oracle's whole C4 frame, every pixel
    if exchange == "masked":  # the sky and the blurred background: far below 4 B per pixel
        assert d["rank0_stream_bytes"] < 3 * 1920 * 1080
