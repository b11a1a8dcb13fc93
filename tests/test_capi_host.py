"""C-ABI library: loads, exports every symbol include/atray.h declares, and its host-side
prerequisites (OBJ parse, AABB, translate, octree build, camera, tiles) are bit-identical to
the oracle. CPU only: no compute call touches a GPU here."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from atray_amd import engine as E
from atray_amd.assets import CENTERS, asset_path
from oracle import oracle as O

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "atray.h")


def header_symbols():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(atr_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = E.lib()
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(L, s), s
    assert sorted(E.EXPORTS) == syms
    assert b"gfx950" in L.atr_version()


def test_ctypes_fixed_arrays_match_header():
    """Every fixed-size array parameter of a prototype (e.g. counters_out[10]) has the same
    length in the ctypes signature table, so no call can under-allocate an output."""
    txt = re.sub(r"/\*.*?\*/", "", open(HDR).read(), flags=re.S)
    sig = E.signatures()
    checked = 0
    for name, params in re.findall(r"\b(atr_[a-z0-9_]+)\s*\(([^;{]*?)\)\s*;", txt):
        for i, p in enumerate(x.strip() for x in params.split(",")):
            m = re.search(r"\[(\d+)\]$", p)
            if not m or name not in sig:
                continue
            at = sig[name][0][i]
            if isinstance(at, type) and issubclass(at, C.Array):
                assert at._length_ == int(m.group(1)), (name, p, at._length_)
                checked += 1
    assert checked >= 1


def _engine_tree(asset, leaf=300):
    m = E.Mesh.load_obj(asset_path(asset))
    box = m.aabb()
    box = m.translate_to(box, CENTERS[asset])
    return m, box, E.Octree.build(m, leaf)


@pytest.mark.parametrize("asset", ["Cube", "Monkey", "Deer", "Dragon"])
def test_octree_bit_identical_to_oracle(asset):
    m, box, t = _engine_tree(asset)
    s = O.Scene(asset_path(asset), center=CENTERS[asset])
    assert np.array_equal(box.view(np.uint32), s.surrounding_aabb.view(np.uint32))
    st = t.stats()
    os_ = s.tree_stats()
    for k in ["nodes", "inner", "leaves", "empty_leaves", "leaf_prim_refs", "max_leaf"]:
        assert st[k] == os_[k], k
    assert st["depth"] < 16
    bounds, children, first, count, verts, face = t.export()
    nodes, otri, oface = s.tree_arrays()
    assert np.array_equal(bounds[:, :3].view(np.uint32), nodes["bmin"].view(np.uint32))
    assert np.array_equal(bounds[:, 3:].view(np.uint32), nodes["bmax"].view(np.uint32))
    assert np.array_equal(children, nodes["children"])
    leaf = children == 0
    assert np.array_equal(first[leaf], nodes["prim_off"][leaf])
    assert np.array_equal(count[leaf], nodes["prim_cnt"][leaf])
    assert np.array_equal(verts.view(np.uint32), otri.view(np.uint32))
    assert np.array_equal(face, oface)


def test_octree_from_nodes_roundtrip():
    s = O.Scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    nodes, tri, face = s.tree_arrays()
    bounds = np.concatenate([nodes["bmin"], nodes["bmax"]], 1)
    t = E.Octree.from_nodes(bounds, nodes["children"], nodes["prim_off"], nodes["prim_cnt"], tri, face)
    assert t.stats()["nodes"] == len(nodes)
    with pytest.raises(E.AtrError):  # leaf range past the primitive array
        bad = nodes["prim_cnt"].copy()
        bad[nodes["children"] == 0] += 10**6
        E.Octree.from_nodes(bounds, nodes["children"], nodes["prim_off"], bad, tri, face)


QUIRKY = ("# c\nv 0.1 0.2 0.3\nv 1e1 -2.5E-1 +3\nv 1 1 1\nv 2 2 2\nvt 0.5 0.5\nvn 0 0 1\n"
          "f 1/1/1 2/1/1 3/1/1 4/1/1\nf -4//1 -3//1 -2//1\nusemtl x\r\nv\t3 4 5\nvn 0 1 0\r\n"
          "f 1 2 3\nf 5//-1 -2//2 1//1\nf 1/1 2/-1 3/1")


def _bits(a):
    return a.view(np.uint32) if a.dtype == np.float32 else a


def _mesh_equal(a, b):
    return all(x.shape == y.shape and np.array_equal(_bits(x), _bits(y)) for x, y in zip(a, b))


def test_mesh_parser_matches_oracle_on_quirky_text():
    m = E.Mesh.parse_obj(QUIRKY)
    assert m.info() == (4, 2, 5)
    s = O.Scene(obj_text=QUIRKY, center=None, use_tree=False)
    V, N, FV, FN = s.mesh_arrays()
    ev, en, _, efv, _, efn = m.arrays()
    assert np.array_equal(ev.view(np.uint32), V.view(np.uint32)) and np.array_equal(en.view(np.uint32), N.view(np.uint32))
    assert np.array_equal(efv, FV) and np.array_equal(efn, FN)
    assert np.array_equal(m.aabb().view(np.uint32), s.surrounding_aabb.view(np.uint32))


@pytest.mark.parametrize("asset", ["Cube", "Monkey", "Deer", "Dragon"])
def test_parallel_obj_load_bit_identical(asset):
    """f3: load_model_data's chunked parallel parse (OBJ_loader.cpp:298-340) gives the
    single-threaded mesh for every chunk count, and both equal the oracle's parse."""
    one = E.Mesh.load_obj(asset_path(asset), threads=1).arrays()
    for th in (2, 3, 7, 16, 0):
        assert _mesh_equal(E.Mesh.load_obj(asset_path(asset), threads=th).arrays(), one), th
    if asset != "Dragon":  # the Dragon surrogate is checked through the octree test above
        s = O.Scene(asset_path(asset), center=None, use_tree=False)
        V, N, FV, FN = s.mesh_arrays()
        assert np.array_equal(one[0].view(np.uint32), V.view(np.uint32)) and np.array_equal(one[3], FV)
        assert np.array_equal(one[1].view(np.uint32), N.view(np.uint32)) and np.array_equal(one[5], FN)


@pytest.mark.parametrize("text", [QUIRKY, QUIRKY + "\n", "v 1 2 3", "", "\n\n", "f 1 2 3\nv 1 1 1\0 junk\nv 2\0 2 2\n",
                                  "v 1 2 3\r\n" * 50 + "f 1 2 3\r\n" * 40])
def test_parallel_parse_edge_texts(text):
    """No trailing newline, CRLF, empty input, NUL bytes (read as blanks), chunks smaller than a
    line: every thread count gives the one-thread mesh."""
    one = E.Mesh.parse_obj(text, threads=1).arrays()
    for th in (2, 3, 5, 64):
        assert _mesh_equal(E.Mesh.parse_obj(text, threads=th).arrays(), one), th


def test_scene_upload_rejects_bad_sphere_and_plane_materials():
    """atr_scene_upload validates every material index the device shading reads (mats[material])
    before touching the context, so this runs without a GPU."""
    L = E.lib()
    fake_ctx = C.create_string_buffer(64)  # never dereferenced: validation fails first
    mats = (E.atr_material * 2)()
    for sph, pln in [([((0, 0, 0), 1.0, 2)], []), ([((0, 0, 0), 1.0, -1)], []), ([], [((0, 1, 0), 0.0, 7)]),
                     ([], [((0, 1, 0), 0.0, -3)])]:
        sa = (E.atr_sphere * max(1, len(sph)))(*[E.atr_sphere(E.vec3(c), r, m) for c, r, m in sph])
        pa = (E.atr_plane * max(1, len(pln)))(*[E.atr_plane(E.vec3(n), d, m) for n, d, m in pln])
        rc = L.atr_scene_upload(C.cast(fake_ctx, C.c_void_p), C.cast(mats, C.c_void_p), 2, None, 0,
                                C.cast(sa, C.c_void_p), len(sph), C.cast(pa, C.c_void_p), len(pln))
        assert rc == -1, (sph, pln, rc)


def test_camera_matches_oracle():
    for (w, h, aa, spp, b) in [(1920, 1080, 0, 1, 1), (256, 256, 1, 4, 5), (7, 3, 0, 2, 2)]:
        ce = E.camera(w, h, spp, b, aa)
        co = O.Camera(w, h, spp=spp, bounces=b, aa=aa).c
        assert bytes(ce) == bytes(co)


@pytest.mark.parametrize("wht", [(1280, 720, 8), (1920, 1080, 8), (256, 256, 1), (100, 30, 8), (5, 5, 8)])
def test_reference_tiles_match_oracle(wht):
    w, h, t = wht
    assert np.array_equal(E.make_tiles(w, h, t), O.make_tiles(w, h, t))


def test_shard_tiles_partition_the_image():
    W, H = 1920, 1080
    cover = np.zeros((H, W), np.int32)
    for r in range(3):
        for x0, y0, x1, y1 in E.make_shard_tiles(W, H, 64, r, 3):
            cover[y0:y1 + 1, x0:x1 + 1] += 1
    assert (cover == 1).all()


def test_packed_size_counts_union_of_overlapping_tiles():
    tiles = E.make_tiles(1280, 720, 8)  # inclusive tiles overlapping by one pixel
    assert E.packed_size(tiles) == 1280 * 720
    assert E.packed_size([[0, 0, 9, 9], [5, 5, 14, 14]]) == 100 + 100 - 25


def test_write_bmp_layout_and_naming(tmp_path):
    """texture.cpp:66-115: 14 + 56 byte headers, BI_BITFIELDS masks, the BGRX rows as stored
    (row 0 = bottom, positive height), and the first free <name>_<id>.bmp."""
    import struct
    W, H = 5, 3
    px = (np.arange(W * H, dtype=np.uint32) * 0x010203 + 0x00112233).reshape(H, W)
    base = str(tmp_path / "render")
    p0 = E.write_bmp(px, base)
    p1 = E.write_bmp(px, base)
    assert (p0, p1) == (base + "_0.bmp", base + "_1.bmp")
    b = open(p0, "rb").read()
    assert len(b) == 70 + W * H * 4
    assert b[:2] == b"BM" and struct.unpack_from("<iHHI", b, 2) == (70 + W * H * 4, 0, 0, 70)
    dib = struct.unpack_from("<IIIhhIIIIIIIIII", b, 14)
    assert dib == (56, W, H, 1, 32, 3, W * H * 4, 197, 39, 0, 0, 0x00FF0000, 0x0000FF00, 0x000000FF, 0)
    assert np.array_equal(np.frombuffer(b[70:], np.uint32).reshape(H, W), px)


def test_write_bmp_id_limit_and_errors(tmp_path):
    """The reference formats into strlen(name) + 8 bytes, so ids 0..99 fit; past them, and for
    a path that cannot be created, the writer reports ATR_E_IO instead of writing nothing."""
    px = np.zeros((1, 1), np.uint32)
    base = str(tmp_path / "f")
    for i in range(100):
        open(f"{base}_{i}.bmp", "wb").close()
    with pytest.raises(E.AtrError):
        E.write_bmp(px, base)
    with pytest.raises(E.AtrError):
        E.write_bmp(px, str(tmp_path / "missing_dir" / "x"))
    with pytest.raises(ValueError):
        E.write_bmp(np.zeros(4, np.uint32), base)
    assert E.lib().atr_write_bmp(None, 1, 1, b"x", None, 0) == -1  # ATR_E_INVALID


def test_default_tuning_is_the_measured_schedule():
    """atr_default_tuning (host-only): the knobs a context starts with."""
    import ctypes as C
    t = E.atr_tuning()
    E.lib().atr_default_tuning(C.byref(t))
    got = {f: getattr(t, f) for f, _ in E.atr_tuning._fields_ if f != "reserved"}
    assert got == {"xcd_chunk": 16, "frame_rotate": 0, "hybrid_a": 2, "hybrid_b": 0, "path_batch_log2": 28,
                   "cluster_size": 16, "frame_plan": 1, "path_camera_occ": 0, "path_bounce_occ": 0,
                   "primary_occ": 0, "path_sort_bits": 5, "path_split": 0}
