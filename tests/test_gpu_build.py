"""f3: the octree build on the GPU (atray_amd/csrc/build.hip) against the host
restatement of build_oct_kd_tree (kd_tree.cpp:67-288), which tests/test_capi_host.py pins to the
oracle. Every exported array -- node boxes, children, leaf ranges, leaf primitives' vertices
and face ids -- must be bit-identical, on the asset meshes at the reference leaf size and at
small leaf sizes (deeper trees, more duplication), and on random soups with duplicated and
zero-area triangles (area sum 0: the split point is not inside, the node stays a leaf)."""
import numpy as np
import pytest

from atray_amd import engine as E
from atray_amd.assets import CENTERS, asset_path

pytestmark = pytest.mark.gpu


def _same(a, b):
    ea, eb = a.export(), b.export()
    names = ["bounds", "children", "leaf_first", "leaf_count", "prim_vertices", "prim_face"]
    for n, x, y in zip(names, ea, eb):
        assert x.shape == y.shape, n
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), n
    assert a.stats() == b.stats()


def _mesh(asset):
    m = E.Mesh.load_obj(asset_path(asset))
    m.translate_to(m.aabb(), CENTERS[asset])
    return m


@pytest.mark.parametrize("asset,leaf", [("Cube", 300), ("Cube", 4), ("Monkey", 300), ("Monkey", 64),
                                        ("Monkey", 16), ("Deer", 300), ("Deer", 32),
                                        ("Dragon", 300), ("Dragon", 64)])
def test_device_build_bit_identical(asset, leaf):
    m = _mesh(asset)
    tm = {}
    g = E.Octree.build_device(m, leaf, timings=tm)
    _same(g, E.Octree.build(m, leaf))
    assert tm["wall_ms"] > 0 and tm["device_ms"] > 0


def _soup(n, seed, dup=0.2, flat=0.1):
    rng = np.random.default_rng(seed)
    c = rng.normal(size=(n, 3)) * rng.choice([0.5, 4.0], (n, 1))
    tri = c[:, None, :] + rng.normal(scale=0.2, size=(n, 3, 3))
    k = int(n * dup)
    tri[rng.integers(0, n, k)] = tri[rng.integers(0, n, k)]      # exact duplicates
    z = rng.integers(0, n, int(n * flat))
    tri[z, 1] = tri[z, 0]                                       # zero-area triangles
    tri[z, 2] = tri[z, 0]
    v = tri.reshape(-1, 3).astype(np.float32)
    lines = [f"v {x:.9g} {y:.9g} {w:.9g}" for x, y, w in v]
    lines += [f"f {3 * i + 1} {3 * i + 2} {3 * i + 3}" for i in range(n)]
    return E.Mesh.parse_obj("\n".join(lines))


@pytest.mark.parametrize("n,seed,leaf", [(5000, 1, 40), (20000, 2, 300), (3000, 3, 8)])
def test_device_build_soups(n, seed, leaf):
    m = _soup(n, seed)
    _same(E.Octree.build_device(m, leaf), E.Octree.build(m, leaf))


def test_device_build_degenerate():
    # every triangle collapsed onto one point: areas 0, split point 0/0 = NaN, never inside
    txt = "v 1 1 1\n" + "f 1 1 1\n" * 500
    m = E.Mesh.parse_obj(txt)
    g = E.Octree.build_device(m, 10)
    _same(g, E.Octree.build(m, 10))
    assert g.stats()["nodes"] == 1
    # no faces at all
    m0 = E.Mesh.parse_obj("v 0 0 0\nv 1 0 0\n")
    _same(E.Octree.build_device(m0, 300), E.Octree.build(m0, 300))


def test_device_build_rejects_bad_input():
    m = E.Mesh.parse_obj("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 9\n")
    with pytest.raises(E.AtrError):
        E.Octree.build_device(m, 300)
