"""The engine's fast reciprocal of the culled test's det (trace.h recip_det) equals IEEE division,
1.0f / x, bit for bit for every f32 x in [2^-14, 2^64) -- 654 M values, every mantissa of every
exponent the fast path takes (det >= kTol = 1e-4). tests/c/recip_check.hip, built in-tree by
atray_amd/csrc/Makefile. Needs an MI355X (-m gpu)."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_fast_reciprocal_is_correctly_rounded():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    exe = os.path.join(ROOT, "atray_amd", "_lib", "recip_check")
    assert os.path.exists(exe), "build first: make -C atray_amd/csrc"
    # never a stale binary: it must be newer than every source it is built from
    for src in ("tests/c/recip_check.hip", "atray_amd/csrc/trace.h", "atray_amd/csrc/engine.h"):
        assert os.path.getmtime(exe) >= os.path.getmtime(os.path.join(ROOT, src)), f"recip_check older than {src}"
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "recip mismatches 0 checked 654311424" in r.stdout, r.stdout
