"""The engine's host-side scene preparation under AddressSanitizer + UndefinedBehaviorSanitizer
(CPU only, host code only: the sanitizers never reach a GPU kernel).

tests/c/host_sanitize.cpp drives the C++ behind atr_mesh_parse_obj / atr_octree_build /
atr_octree_finish / the leaf-cluster and inner-node tables / the tile planners
(atray_amd/csrc/obj_parse.cpp, host_scene.cpp) over the committed OBJ assets and 400
deterministic mutations of each (truncated lines, flipped bytes, injected out-of-range or
negative indices, over- and underflowing numbers), checking that the threaded parser gives the
single-threaded mesh and that every shard plan covers the frame. Any sanitizer report fails it.
"""
import glob
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"
CSRC = os.path.join(ROOT, "atray_amd", "csrc")


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("no ROCm compiler")
    out = str(tmp_path_factory.mktemp("host_sanitize") / "host_sanitize")
    # host-only build: no --offload-arch, and -fno-gpu-sanitize (same line, as the GPU pool's check wants)
    # keeps the sanitizers off any device pass. This file is also listed in .gpurunignore: CPU only.
    cmd = [HIPCC, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-gpu-sanitize",
           "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", os.path.join(ROOT, "tests", "c", "host_sanitize.cpp"),
           os.path.join(CSRC, "host_scene.cpp"), os.path.join(CSRC, "obj_parse.cpp"), "-lpthread", "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    return out


def test_host_scene_prep_is_sanitizer_clean(exe):
    assets = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "assets", "*.obj")))
    assert assets
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([exe, "400", *assets], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "Sanitizer" not in r.stderr, r.stderr[-4000:]
    last = r.stdout.strip().splitlines()[-1]
    assert last.startswith("host_sanitize ok") and int(last.split()[-1]) > 1500, last
