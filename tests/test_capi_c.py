"""The C-ABI from a C compiler: tests/c/abi_check.c is built by gcc against include/atray.h and
linked to libatray_hip.so (atray_amd/csrc/Makefile). Its struct layouts must equal the ctypes
mirrors in atray_amd/engine.py, its host calls must agree with the Python binding, and on the GPU
its render (atr_create -> atr_scene_upload -> atr_render_start -> atr_render_wait, the
renderer.h flow) must reproduce the reference's Cube hash."""
import ctypes as C
import json
import os
import subprocess

import pytest

from atray_amd import engine as E
from atray_amd.assets import CENTERS, asset_path

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "atray_amd", "_lib", "abi_check")


def run(*args):
    if not os.path.exists(EXE):
        pytest.fail(f"{EXE} not built (make -C atray_amd/csrc)")
    r = subprocess.run([EXE, *args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_struct_layouts_match_ctypes_mirrors():
    lay = run("layout")
    for name in ["atr_vec3", "atr_material", "atr_model", "atr_sphere", "atr_plane", "atr_camera", "atr_tile",
                 "atr_frame", "atr_tuning"]:
        cls = getattr(E, name)
        assert lay[f"sizeof({name})"] == C.sizeof(cls), name
        for field, _ in cls._fields_:
            assert lay[f"{name}.{field}"] == getattr(cls, field).offset, (name, field)
        # every C field is mirrored (no field missing from the ctypes side)
        c_fields = {k.split(".", 1)[1] for k in lay if k.startswith(name + ".")}
        assert c_fields == {f for f, _ in cls._fields_}, name


def test_host_calls_from_c_agree_with_the_binding():
    h = run("host", asset_path("Cube"))
    m = E.Mesh.load_obj(asset_path("Cube"))
    box = m.translate_to(m.aabb(), CENTERS["Cube"])
    t = E.Octree.build(m, 300)
    assert (h["nv"], h["nn"], h["nf"]) == m.info()
    assert h["nodes"] == t.stats()["nodes"] and h["leaf_refs"] == t.stats()["leaf_prim_refs"]
    assert [float(C.c_float(x).value) for x in h["aabb"]] == [float(x) for x in box]
    cam = E.camera(256, 256)
    assert h["aspect"] == pytest.approx(cam.aspect_ratio, rel=0, abs=0)
    assert h["tiles_1280x720_8"] == len(E.make_tiles(1280, 720, 8)) == 40
    assert h["version"] == E.lib().atr_version().decode()


@pytest.mark.gpu
def test_c_caller_renders_the_reference_cube_hash():
    g = run("gpu", asset_path("Cube"))
    assert g["hash"] == "ccc1a886254060ba" and g["hits"] == 7155
    assert g["traced"] == 256 * 256 and g["tiles_done"] == g["ntiles"] == 64
