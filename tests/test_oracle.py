"""The CPU oracle against the reference's own recorded outputs and the
committed golden vectors. CPU only."""
import numpy as np
import pytest

from atray_amd.assets import CENTERS, asset_path
from oracle import oracle as O
from tests.goldens import GOLD, SEED, hits, render

M = 0xFFFFFFFF


@pytest.mark.parametrize("name", ["cube_256_tree", "monkey_1280x720_tree", "monkey_1280x720_bf",
                                  "deer_640x360_tree", "dragon_480x270_tree"])
def test_oracle_primary_hits_match_goldens(name):
    g = GOLD["hits"][name]
    s = O.Scene(asset_path(g["asset"]), center=CENTERS[g["asset"]], use_tree=g["tree"])
    f, t, ctr = s.primary_hits(O.Camera(g["W"], g["H"]))
    gf, gt = hits(name)
    assert np.array_equal(f, gf)
    assert np.array_equal(t.view(np.uint32), gt.view(np.uint32))
    assert f"{O.fnv_hits(f, t):016x}" == g["hash"]
    assert ctr == g["counters"]


def test_survey_pins():
    """Hashes/hit counts the survey recorded from the reference itself."""
    assert GOLD["hits"]["cube_256_tree"]["hash"] == "ccc1a886254060ba"
    assert GOLD["hits"]["cube_256_tree"]["hits"] == 7155
    assert GOLD["hits"]["monkey_1280x720_tree"]["hash"] == "679cb71ac9b3db1d"
    assert GOLD["hits"]["monkey_1280x720_tree"]["hits"] == 64597
    assert GOLD["hits"]["monkey_1280x720_bf"]["hits"] == 64606
    assert GOLD["hits"]["dragon_1920x1080_tree"]["hash"] == "43ad95dbe7a70300"
    st = GOLD["hits"]["dragon_1920x1080_tree"]["tree_stats"]
    assert (st["nodes"], st["inner"], st["leaves"], st["empty_leaves"], st["leaf_prim_refs"],
            st["max_leaf"]) == (2857, 357, 2500, 73, 234665, 297)


def test_tree_vs_bruteforce_monkey_difference():
    """99 different faces + 9 tree-missed pixels (first-leaf break etc)."""
    ft, _ = hits("monkey_1280x720_tree")
    fb, _ = hits("monkey_1280x720_bf")
    assert int(((ft != fb) & (ft != M) & (fb != M)).sum()) == 99
    assert int(((ft == M) & (fb != M)).sum()) == 9
    assert int(((ft != M) & (fb == M)).sum()) == 0


@pytest.mark.parametrize("name", list(GOLD["render"].keys()))
def test_oracle_render_matches_goldens(name):
    g = GOLD["render"][name]
    s = O.Scene(asset_path(g["asset"]), center=CENTERS[g["asset"]], use_tree=g["tree"])
    rgb, fb, casts, ctr = s.render(O.Camera(g["W"], g["H"], spp=g["spp"], bounces=g["bounces"],
                                            aa=g["aa"]), SEED)
    grgb, gfb, gcasts = render(name)
    assert np.array_equal(rgb.view(np.uint32), grgb.view(np.uint32))
    assert np.array_equal(fb, gfb) and np.array_equal(casts, gcasts)
    assert ctr == g["counters"]


def test_pcg_reference_sequence():
    """PCG-XSH-RR 64/32 (PL_math.h:506-516): pcg-random.org's demo vector for
    state 42 / seq 54 after pcg32_srandom: 0xa15c02b7 0x7b47f409 0xba1d3330 ..."""
    # pcg32_srandom_r(42, 54): inc = 54<<1|1; state=0; step; state+=42; step
    inc = (54 << 1) | 1
    st = 0
    st = (st * 6364136223846793005 + inc) & (2**64 - 1)
    st = (st + 42) & (2**64 - 1)
    st = (st * 6364136223846793005 + inc) & (2**64 - 1)
    out = O.pcg_sequence(st, inc, 6)
    assert out == [0xa15c02b7, 0x7b47f409, 0xba1d3330, 0x83d2f293, 0xbfa4784b, 0xcbed606e]


def test_tiles_match_reference_grid():
    """renderer.cpp:403-445: 1280x720 on 8 threads -> 160 px inclusive tiles, 8x5 = 40."""
    t = O.make_tiles(1280, 720, 8)
    assert len(t) == 40
    assert t[0].tolist() == [0, 0, 160, 160]
    assert t[-1].tolist() == [1120, 640, 1279, 719]
    t = O.make_tiles(1920, 1080, 8)
    assert len(t) == 40 and t[0].tolist() == [0, 0, 240, 240]


def test_obj_parser_quirks():
    """parse_f64 (parser.h:113-191) multiplies a u64 mantissa by a f64 power of ten; faces
    keep only the first triangle of a polygon; negative indices are relative."""
    txt = "v 0.1 0.2 0.3\nv 1e1 -2.5E-1 +3\nv 1 1 1\nv 2 2 2\nvn 0 0 1\nf 1//1 2//1 3//1 4//1\nf -4 -3 -2\n"
    s = O.Scene(obj_text=txt, center=None, use_tree=False)
    V, N, FV, FN = s.mesh_arrays()
    assert V.dtype == np.float32
    # 0.1 = (f32)((f64)1 * 1.0e-1)
    assert V[0, 0] == np.float32(np.float64(1) * 1.0e-1)
    assert V[1].tolist() == [np.float32(10.0), np.float32(-0.25), np.float32(3.0)]
    assert FV.tolist() == [[0, 1, 2], [0, 1, 2]]
    assert FN.tolist() == [[0, 0, 0], [-1, -1, -1]]
