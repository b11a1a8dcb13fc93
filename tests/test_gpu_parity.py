"""GPU parity: the HIP engine (through the C-ABI) against the pinned oracle and the committed
golden vectors. Bit-exact face index and t bits for primary hits; framebuffer and ray_casts
bit-exact and RGB within 1e-5 relative (north star) for multi-bounce renders -- in practice the
RGB is bit-exact too and the test reports it. Needs an MI355X (-m gpu)."""
import ctypes as C
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from atray_amd import engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.goldens import GOLD, SEED, hits, render  # noqa: E402

pytestmark = pytest.mark.gpu
SKY, MODEL = O.SKY, O.MODEL_MAT
# Every variant of the shipping library: LANE (the reference's exact per-triangle work), the cell
# kernels HYBRID (primary-only default) and FLAT (multi-bounce megakernel), and the sample-parallel
# path engine PATHS (multi-bounce default).
VARIANTS = list(E.VARIANTS)
# ATR_TEST_VARIANTS=a,b,...: exactly these kernel codes (experiment builds)
if os.environ.get("ATR_TEST_VARIANTS"):
    VARIANTS = [int(v) for v in os.environ["ATR_TEST_VARIANTS"].split(",")]
RGB_RTOL = 1e-5


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = E.Engine(0)
    yield e
    e.close()


_scenes = {}


def upload(eng, asset, tree=True, spheres=(), planes=(), materials=(SKY, MODEL)):
    key = (asset, tree)
    if key not in _scenes:
        m = E.Mesh.load_obj(asset_path(asset))
        box = m.translate_to(m.aabb(), CENTERS[asset])
        _scenes[key] = (m, E.Octree.build(m, 300) if tree else None, box)
    m, t, box = _scenes[key]
    eng.upload(list(materials), [(m, t, box, 1)], spheres, planes)


def run(eng, cam, tiles=None, layout=E.ATR_LAYOUT_IMAGE, variant=E.ATR_KERNEL_AUTO, seed=SEED, progressive=0):
    W, H = cam.width, cam.height
    if tiles is None:
        tiles = [[0, 0, W - 1, H - 1]]
    n = W * H if layout == E.ATR_LAYOUT_IMAGE else max(1, E.packed_size(tiles))
    dev = torch.device("cuda", 0)
    fb = torch.full((n,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
    face = torch.full((n,), -7, dtype=torch.int32, device=dev)
    t = torch.zeros(n, dtype=torch.float32, device=dev)
    rgb = torch.zeros(3 * n, dtype=torch.float32, device=dev)
    casts = torch.full((n,), -1, dtype=torch.int32, device=dev)
    traced = torch.zeros(1, dtype=torch.int64, device=dev)
    fr = E.atr_frame(layout, fb.data_ptr(), face.data_ptr(), t.data_ptr(), rgb.data_ptr(),
                     casts.data_ptr(), traced.data_ptr())
    stream = torch.cuda.current_stream().cuda_stream
    if progressive:
        eng.render_start_progressive(cam, tiles, fr, seed, progressive, stream=stream, variant=variant)
    else:
        eng.render_start(cam, tiles, fr, seed, stream=stream, variant=variant)
    rc, done = eng.wait()
    assert rc == 0 and done == len(tiles)
    torch.cuda.synchronize()
    out = {"fb": fb.cpu().numpy().view(np.uint32), "face": face.cpu().numpy().view(np.uint32),
           "t": t.cpu().numpy(), "rgb": rgb.cpu().numpy().reshape(-1, 3),
           "casts": casts.cpu().numpy().view(np.uint32), "traced": int(traced.item())}
    if layout == E.ATR_LAYOUT_IMAGE:
        for k in ["fb", "face", "t", "casts"]:
            out[k] = out[k].reshape(H, W)
        out["rgb"] = out["rgb"].reshape(H, W, 3)
    return out


def assert_rgb(got, want):
    both_exact = np.array_equal(got.view(np.uint32), want.view(np.uint32))
    if not both_exact:
        np.testing.assert_allclose(got, want, rtol=RGB_RTOL, atol=1e-7)
    return both_exact


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", ["cube_256_tree", "monkey_1280x720_tree", "monkey_1280x720_bf",
                                  "deer_640x360_tree", "dragon_480x270_tree"])
def test_primary_hits_bit_exact(eng, name, variant):
    g = GOLD["hits"][name]
    upload(eng, g["asset"], g["tree"])
    o = run(eng, E.camera(g["W"], g["H"]), variant=variant)
    gf, gt = hits(name)
    bad = np.argwhere(o["face"] != gf)
    assert len(bad) == 0, f"{len(bad)} face mismatches, first {bad[:5].tolist()}"
    assert np.array_equal(o["t"].view(np.uint32), gt.view(np.uint32))
    assert o["traced"] == g["counters"]["n_rays"]


@pytest.mark.parametrize("variant", VARIANTS)
def test_dragon_1920x1080_matches_reference_hash(eng, variant):
    """Config 3 at full size: per-pixel (face, t) hash equals the reference's own output
    recorded by the survey probe (43ad95dbe7a70300, 284,360 hits)."""
    upload(eng, "Dragon", True)
    o = run(eng, E.camera(1920, 1080), variant=variant)
    assert int((o["face"] != E.MISS).sum()) == 284360
    assert f"{O.fnv_hits(o['face'], o['t']):016x}" == "43ad95dbe7a70300"


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", list(GOLD["render"].keys()))
def test_multibounce_render_matches_golden(eng, name, variant):
    g = GOLD["render"][name]
    upload(eng, g["asset"], g["tree"])
    o = run(eng, E.camera(g["W"], g["H"], g["spp"], g["bounces"], g["aa"]), variant=variant)
    grgb, gfb, gcasts = render(name)
    assert np.array_equal(o["fb"], gfb)
    assert np.array_equal(o["casts"], gcasts)
    assert_rgb(o["rgb"], grgb)
    assert o["traced"] == g["counters"]["n_rays"]


def test_packed_shards_unpack_to_the_image(eng):
    """Multi-GPU path on one GPU: R virtual ranks render interleaved shard tiles into packed
    buffers; unpacking them reproduces the single-render image byte for byte."""
    upload(eng, "Dragon", True)
    W, H = 480, 270
    cam = E.camera(W, H, 2, 3)
    full = run(eng, cam)
    img = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    for r in range(3):
        tiles = E.make_shard_tiles(W, H, 40, r, 3)
        o = run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED)
        p = torch.from_numpy(o["fb"].view(np.int32).copy()).cuda()
        eng.unpack(tiles, W, p.data_ptr(), img.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy().view(np.uint32).reshape(H, W), full["fb"])


def test_reference_tiles_and_ray_cast_counts(eng):
    """Overlapping reference tiles (renderer.cpp:429-442) trace every pixel once; per-tile
    ray_casts are the reference's sums over the inclusive rects (overlaps twice)."""
    name = "monkey_320x180_s4_b5"
    g = GOLD["render"][name]
    upload(eng, "Monkey", True)
    tiles = E.make_tiles(g["W"], g["H"], 8)
    o = run(eng, E.camera(g["W"], g["H"], g["spp"], g["bounces"]), tiles=tiles)
    _, gfb, gcasts = render(name)
    assert np.array_equal(o["fb"], gfb)
    casts = torch.from_numpy(o["casts"].view(np.int32).ravel().copy()).cuda()
    per = torch.zeros(len(tiles), dtype=torch.int64, device="cuda")
    eng.tile_ray_casts(tiles, g["W"], casts.data_ptr(), per.data_ptr())
    want = [int(gcasts[y0:y1 + 1, x0:x1 + 1].astype(np.int64).sum()) for x0, y0, x1, y1 in tiles]
    assert per.cpu().numpy().tolist() == want


@pytest.mark.parametrize("kind", ["shard", "reference"])
@pytest.mark.parametrize("planned", [False, True])
def test_packed_tile_ray_casts(eng, kind, planned):
    """atr_packed_tile_ray_casts (the multi-GPU bench's per-tile counters): per-tile sums of a
    PACKED multi-frame ray_casts buffer equal the sums of the golden per-pixel ray_casts over each
    tile's pixels -- shard tiles (disjoint), and the reference's overlapping tiles, where a pixel
    counts in the first tile holding it (the packed layout traces it once). planned: a cell plan
    with dispatch classes and splits reorders the block list, not the packed slots (the bench's
    graded order; the slot-to-tile map once followed the list order)."""
    name = "monkey_320x180_s4_b5"
    g = GOLD["render"][name]
    upload(eng, "Monkey", True)
    W, H = g["W"], g["H"]
    cam = E.camera(W, H, g["spp"], g["bounces"])
    tiles = E.make_shard_tiles(W, H, 32, 1, 3) if kind == "shard" else E.make_tiles(W, H, 8)
    if planned:
        rng = np.random.default_rng(11)
        ncell = ((W + 7) // 8) * ((H + 7) // 8)
        plan = rng.choice(np.array([0, 2, E.plan_class(7), E.plan_class(4) | 4, E.plan_class(1)], np.uint8),
                          size=ncell)
        eng.set_cell_plan(W, H, plan)
    try:
        o = run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED)
        _check_packed_tile_casts(eng, name, W, H, tiles, o)
    finally:
        if planned:
            eng.set_cell_plan(W, H, None)


def _check_packed_tile_casts(eng, name, W, H, tiles, o):
    n = E.packed_size(tiles)
    F, stride = 3, n + 11
    casts = torch.full((F * stride,), 5, dtype=torch.int32, device="cuda")
    for f in range(F):  # frame f holds the render's ray_casts + f per pixel
        casts[f * stride:f * stride + n] = torch.from_numpy(o["casts"].view(np.int32) + f).cuda()
    out = torch.full((F * len(tiles),), -3, dtype=torch.int64, device="cuda")
    eng.packed_tile_ray_casts(tiles, W, H, casts.data_ptr(), F, stride, out.data_ptr(),
                              stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    _, _, gcasts = render(name)
    owner = np.full((H, W), -1, np.int64)
    for k, (x0, y0, x1, y1) in enumerate(tiles):
        blk = owner[y0:y1 + 1, x0:x1 + 1]
        blk[blk < 0] = k
    got = out.cpu().numpy().reshape(F, len(tiles))
    for f in range(F):
        want = [int((gcasts.astype(np.int64) + f)[owner == k].sum()) for k in range(len(tiles))]
        assert got[f].tolist() == want


@pytest.mark.parametrize("variant", VARIANTS)
def test_cell_plan_changes_no_output(eng, variant):
    """atr_set_cell_plan: cells split over 2, 4 or 8 waves (the measured heaviest and some at
    random) leave every output identical, image and packed layouts, primary and multi-bounce."""
    upload(eng, "Dragon", True)
    W, H = 480, 270
    rng = np.random.default_rng(3)
    try:
        for spp, bounces in ((1, 1), (2, 3)):
            cam = E.camera(W, H, spp, bounces)
            tiles = E.make_shard_tiles(W, H, 64, 0, 2)
            want = [run(eng, cam, variant=variant), run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED,
                                                         variant=variant)]
            cost = eng.cell_costs(E.camera(W, H), SEED).ravel()
            plan = rng.choice(np.array([0, 1, 2, 4, 8], np.uint8), size=cost.size, p=[0.6, 0.1, 0.1, 0.1, 0.1])
            plan[np.argsort(-cost)[:40]] = 4
            # dispatch-first and priority flags on random cells (scheduling only)
            plan |= rng.choice(np.array([0, E.plan_class(7), E.plan_class(3), E.ATR_PLAN_PRIO,
                                         E.plan_class(5) | E.ATR_PLAN_PRIO], np.uint8), size=cost.size,
                               p=[0.6, 0.1, 0.1, 0.1, 0.1])
            eng.set_cell_plan(W, H, plan)
            got = [run(eng, cam, variant=variant), run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED,
                                                        variant=variant)]
            eng.set_cell_plan(W, H, None)
            for a, b in zip(want, got):
                for k in ("fb", "face", "t", "casts", "rgb"):
                    assert np.array_equal(np.asarray(a[k]).view(np.uint32), np.asarray(b[k]).view(np.uint32)), k
                assert a["traced"] == b["traced"]
    finally:
        eng.set_cell_plan(W, H, None)
    with pytest.raises(E.AtrError):
        eng.set_cell_plan(W, H, np.full(((W + 7) // 8) * ((H + 7) // 8), 3, np.uint8))
    with pytest.raises(E.AtrError):
        eng.set_cell_plan(W, H, np.full(((W + 7) // 8) * ((H + 7) // 8), 0x45, np.uint8))


@pytest.mark.parametrize("variant", [E.ATR_KERNEL_HYBRID, E.ATR_KERNEL_FLAT])
def test_cell_plan_under_frame_plan_changes_no_output(eng, variant):
    """A user cell plan with 2/4/8-way splits and classes, the single-frame plan on top of it
    (frame_plan=1 re-plans the split list launch after launch, plan.hip): the same tiles rendered
    three times equal the frame_plan=0 render, image and packed layouts."""
    upload(eng, "Dragon", True)
    W, H = 480, 270
    rng = np.random.default_rng(11)
    base = eng.tuning()
    ncell = ((W + 7) // 8) * ((H + 7) // 8)
    plan = rng.choice(np.array([0, 2, 4, 8], np.uint8), size=ncell, p=[0.7, 0.1, 0.1, 0.1])
    plan |= rng.choice(np.array([0, E.plan_class(7), E.plan_class(2)], np.uint8), size=ncell, p=[0.6, 0.2, 0.2])
    try:
        for spp, bounces in ((1, 1), (2, 3)):
            cam = E.camera(W, H, spp, bounces)
            tiles = E.make_shard_tiles(W, H, 64, 0, 2)
            eng.set_cell_plan(W, H, plan)
            eng.set_tuning(frame_plan=0)
            want = [run(eng, cam, variant=variant), run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED,
                                                         variant=variant)]
            eng.set_tuning(frame_plan=1)
            for _ in range(3):  # the same block set each time: the planned list is dispatched
                got = [run(eng, cam, variant=variant), run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED,
                                                            variant=variant)]
                for a, b in zip(want, got):
                    for k in ("fb", "face", "t", "casts", "rgb"):
                        assert np.array_equal(np.asarray(a[k]).view(np.uint32), np.asarray(b[k]).view(np.uint32)), k
                    assert a["traced"] == b["traced"]
    finally:
        eng.set_cell_plan(W, H, None)
        eng.set_tuning(**base)


@pytest.mark.parametrize("variant", VARIANTS)
def test_tuning_changes_no_output(eng, variant):
    """atr_set_tuning: XCD chunking, the HYBRID deal rule forced to always / never deal, the path
    engine's batch size (2^12 paths: dozens of batches per frame), occupancies, queue sort and the
    two-stream split of one-batch launches,
    the HYBRID primary's occupancy and the cluster size (re-upload) change scheduling only -- every output identical, primary and multi-bounce."""
    W, H = 480, 270
    base = eng.tuning()
    settings = [{"xcd_chunk": 0}, {"xcd_chunk": 3}, {"hybrid_a": -4096, "hybrid_b": -4096},
                {"hybrid_a": 4096, "hybrid_b": 4096}, {"path_batch_log2": 12}, {"cluster_size": 7},
                {"frame_plan": 0}, {"primary_occ": 7}, {"primary_occ": 8}, {"path_camera_occ": 5, "path_bounce_occ": 6},
                {"path_camera_occ": 7}, {"path_sort_bits": 0}, {"path_sort_bits": 4}, {"path_sort_bits": 7}, {"path_split": 1},
                {"path_split": 1, "path_sort_bits": 0},
                {"path_sort_bits": 2, "path_batch_log2": 12}, {"path_sort_bits": 5, "path_bounce_occ": 5}]
    try:
        for spp, bounces in ((1, 1), (2, 3)):
            upload(eng, "Dragon", True)
            cam = E.camera(W, H, spp, bounces)
            want = run(eng, cam, variant=variant)
            for kw in settings:
                eng.set_tuning(**kw)
                upload(eng, "Dragon", True)  # cluster_size applies at upload
                got = run(eng, cam, variant=variant)
                eng.set_tuning(**base)
                for k in ("fb", "face", "t", "casts", "rgb"):
                    assert np.array_equal(np.asarray(want[k]).view(np.uint32), np.asarray(got[k]).view(np.uint32)), (kw, k)
                assert want["traced"] == got["traced"], kw
    finally:
        eng.set_tuning(**base)
        upload(eng, "Dragon", True)
    with pytest.raises(E.AtrError):
        eng.set_tuning(cluster_size=17)
    with pytest.raises(E.AtrError):
        eng.set_tuning(xcd_chunk=-1)
    with pytest.raises(E.AtrError):
        eng.set_tuning(path_batch_log2=29)
    for bits in (1, 8, -1):
        with pytest.raises(E.AtrError):
            eng.set_tuning(path_sort_bits=bits)
    with pytest.raises(E.AtrError):
        eng.set_tuning(path_split=2)
    t = E.atr_tuning()  # ABI 2: the reserved words must stay zero
    assert E.lib().atr_get_tuning(eng.h, C.byref(t)) == 0
    t.reserved[1] = 3
    assert E.lib().atr_set_tuning(eng.h, C.byref(t)) == -1  # ATR_E_INVALID
    assert eng.tuning() == base


def test_queue_sort_at_scale(eng):
    """The path engine's queue sort at a c4-like shape -- 960x540 at 16 spp, 5
    bounces: 8.3 M paths, ~2 M per bounce level over the 2^23 bins -- in one batch and in 2^20-path
    batches (a sort per level per batch), at the default and the largest key: every output and the
    traced-ray count identical to queue order; framebuffer, hit records and ray counts also equal
    FLAT's (the cell megakernel)."""
    upload(eng, "Dragon", True)
    cam = E.camera(960, 540, 16, 5)
    base = eng.tuning()
    try:
        flat = run(eng, cam, variant=E.ATR_KERNEL_FLAT)
        eng.set_tuning(path_sort_bits=0)
        want = run(eng, cam, variant=E.ATR_KERNEL_PATHS)
        for k in ("fb", "face", "t", "casts"):
            assert np.array_equal(flat[k].view(np.uint32), want[k].view(np.uint32)), k
        for kw in ({"path_sort_bits": base["path_sort_bits"]}, {"path_sort_bits": 6},
                   {"path_sort_bits": base["path_sort_bits"], "path_batch_log2": 20}):
            eng.set_tuning(**kw)
            got = run(eng, cam, variant=E.ATR_KERNEL_PATHS)
            eng.set_tuning(**base)
            for k in ("fb", "face", "t", "casts", "rgb"):
                assert np.array_equal(want[k].view(np.uint32), got[k].view(np.uint32)), (kw, k)
            assert want["traced"] == got["traced"], kw
    finally:
        eng.set_tuning(**base)


@pytest.mark.parametrize("variant", VARIANTS)
def test_frame_plan_changes_no_output(eng, variant):
    """The single-frame plan (tuning frame_plan, plan.hip): consecutive one-frame launches of a
    tile list dispatch the cells by the previous launch's cost, heaviest first, the heaviest 1 %
    split over two row-band waves -- image and packed layouts, primary and multi-bounce, every
    output identical to the plain list order, launch after launch."""
    upload(eng, "Dragon", True)
    W, H = 480, 270
    base = eng.tuning()
    try:
        for spp, bounces in ((1, 1), (2, 3)):
            cam = E.camera(W, H, spp, bounces)
            tiles = E.make_shard_tiles(W, H, 64, 1, 2)
            eng.set_tuning(frame_plan=0)
            want = [run(eng, cam, variant=variant), run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED,
                                                         variant=variant)]
            eng.set_tuning(frame_plan=1)
            for _ in range(5):  # the first two measure, the later ones dispatch by a plan (one per parity)
                got = [run(eng, cam, variant=variant), run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED,
                                                            variant=variant)]
                for a, b in zip(want, got):
                    for k in ("fb", "face", "t", "casts", "rgb"):
                        assert np.array_equal(np.asarray(a[k]).view(np.uint32), np.asarray(b[k]).view(np.uint32)), k
                    assert a["traced"] == b["traced"]
        # costs that jump between launches (a sky view, then the dragon): the previous plan's
        # thresholds would split far more cells than the list holds -- that plan splits none
        sky = E.camera(W, H, 1, 1, facing=(0.0, 1.0, 0.0))
        drag = E.camera(W, H, 1, 1)
        eng.set_tuning(frame_plan=0)
        want_sky, want_drag = run(eng, sky, variant=variant), run(eng, drag, variant=variant)
        eng.set_tuning(frame_plan=1)
        for cam, want in ((sky, want_sky), (drag, want_drag), (drag, want_drag), (sky, want_sky), (drag, want_drag)):
            got = run(eng, cam, variant=variant)
            for k in ("fb", "face", "t", "casts"):
                assert np.array_equal(np.asarray(want[k]).view(np.uint32), np.asarray(got[k]).view(np.uint32)), k
    finally:
        eng.set_tuning(**base)


@pytest.mark.parametrize("variant", [E.ATR_KERNEL_AUTO, E.ATR_KERNEL_FLAT])
def test_frame_plan_back_to_back_launches(eng, variant):
    """Single-frame launches issued back to back with no wait between them (the live view's
    pattern, several in flight): the plan kernels run on the context's plan stream beside the next
    launch, double-buffered (launch n renders from the plan of launch n - 2's costs, capi.cpp
    launch_planned), so each launch must wait for exactly the plan and cleared cost half it uses.
    Eight launches over two alternating cameras, every output equal to the plain list order's."""
    upload(eng, "Dragon", True)
    W, H = 480, 270
    cams = [E.camera(W, H, 1, 1), E.camera(W, H, 1, 1, eye=(0.3, 2.0, 0.6))]
    base = eng.tuning()
    try:
        eng.set_tuning(frame_plan=0)
        want = [run(eng, c, variant=variant) for c in cams]
        eng.set_tuning(frame_plan=1)
        n = W * H
        fb = torch.zeros(8, n, dtype=torch.int32, device="cuda")
        casts = torch.zeros(8, n, dtype=torch.int32, device="cuda")
        traced = torch.zeros(8, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream().cuda_stream
        for i in range(8):
            fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb[i].data_ptr(), None, None, None, casts[i].data_ptr(),
                             traced[i:i + 1].data_ptr())
            eng.render_start(cams[i % 2], [[0, 0, W - 1, H - 1]], fr, SEED, stream=s, variant=variant)
        assert eng.wait()[0] == 0
        torch.cuda.synchronize()
        for i in range(8):
            w = want[i % 2]
            assert np.array_equal(fb[i].cpu().numpy().view(np.uint32), w["fb"].ravel()), i
            assert np.array_equal(casts[i].cpu().numpy().view(np.uint32), w["casts"].ravel()), i
            assert int(traced[i].item()) == w["traced"], i
    finally:
        eng.set_tuning(**base)


def test_renderer_api_start_wait(eng):
    """renderer.h's start/wait pair over the engine, app-scene materials (app.cpp:91-131)."""
    from atray_amd import renderer as R
    scene = R.app_scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    R.prep_scene(scene, eng)
    rs = R.RenderSettings(resolution=(320, 180), samples_per_pixel=4, bounce_limit=5)
    info = R.RenderInfo(camera=R.set_camera((0.1, 2.0, 0.0), (-0.1, -0.5, -1.0), rs, 1.0),
                        scene=scene, seed=SEED)
    R.start_render_from_camera(info, eng)
    while R.wait_for_render_from_camera_to_finish(info, eng, 33):
        pass
    _, gfb, gcasts = render("monkey_320x180_s4_b5")
    assert np.array_equal(info.camera_tex, gfb)
    tiles = E.make_tiles(320, 180, 8)
    assert info.total_ray_casts == sum(int(gcasts[y0:y1 + 1, x0:x1 + 1].sum()) for x0, y0, x1, y1 in tiles)
    assert info.jobs_done == len(tiles) == 40


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("bounces", [1, 3])
def test_frames_per_launch_equal_single_renders(eng, variant, bounces):
    """atr_render_start_frames: every frame of a multi-frame launch (outputs frame_stride apart,
    image and packed layouts) equals the single-frame render."""
    upload(eng, "Monkey", True)
    W, H = 96, 56
    cam = E.camera(W, H, 2, bounces)
    tiles = E.make_tiles(W, H, 4)
    for layout in (E.ATR_LAYOUT_IMAGE, E.ATR_LAYOUT_PACKED):
        want = run(eng, cam, tiles=tiles, layout=layout, variant=variant)
        n = W * H if layout == E.ATR_LAYOUT_IMAGE else E.packed_size(tiles)
        F, stride = 3, n + 37
        fb = torch.full((F * stride,), 0x7F7F7F7F, dtype=torch.int32, device="cuda")
        face = torch.full((F * stride,), -7, dtype=torch.int32, device="cuda")
        t = torch.zeros(F * stride, dtype=torch.float32, device="cuda")
        rgb = torch.zeros(3 * F * stride, dtype=torch.float32, device="cuda")
        casts = torch.full((F * stride,), -1, dtype=torch.int32, device="cuda")
        traced = torch.zeros(1, dtype=torch.int64, device="cuda")
        fr = E.atr_frame(layout, fb.data_ptr(), face.data_ptr(), t.data_ptr(), rgb.data_ptr(), casts.data_ptr(),
                         traced.data_ptr())
        torch.cuda.synchronize()
        eng.render_start_frames(cam, tiles, fr, F, stride, SEED, stream=torch.cuda.current_stream().cuda_stream,
                                variant=variant)
        rc, _ = eng.wait()
        assert rc == 0
        torch.cuda.synchronize()
        assert int(traced.item()) == F * want["traced"]
        for f in range(F):
            sl = slice(f * stride, f * stride + n)
            assert np.array_equal(fb[sl].cpu().numpy().view(np.uint32), want["fb"].ravel())
            assert np.array_equal(face[sl].cpu().numpy().view(np.uint32), want["face"].ravel())
            assert np.array_equal(t[sl].cpu().numpy().view(np.uint32), want["t"].ravel().view(np.uint32))
            assert np.array_equal(casts[sl].cpu().numpy().view(np.uint32), want["casts"].ravel())
            got_rgb = rgb[3 * f * stride:3 * f * stride + 3 * n].cpu().numpy()
            assert np.array_equal(got_rgb.view(np.uint32), want["rgb"].ravel().view(np.uint32))
            if f + 1 < F:  # the gap between frames is untouched
                assert (fb[f * stride + n:(f + 1) * stride].cpu().numpy() == 0x7F7F7F7F).all()


def test_renderer_api_progressive_live_view(eng):
    """Live view (app.cpp:162-186): tiles finish in groups while the render runs; every pixel
    of a tile reported done is final, and the finished frame equals the one-shot render."""
    from atray_amd import renderer as R
    scene = R.app_scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    R.prep_scene(scene, eng)
    rs = R.RenderSettings(resolution=(320, 180), samples_per_pixel=4, bounce_limit=5)
    info = R.RenderInfo(camera=R.set_camera((0.1, 2.0, 0.0), (-0.1, -0.5, -1.0), rs, 1.0),
                        scene=scene, seed=SEED)
    _, gfb, gcasts = render("monkey_320x180_s4_b5")
    tiles = E.make_tiles(320, 180, 8)
    R.start_render_from_camera(info, eng, tiles_per_launch=3)
    seen = []
    while R.wait_for_render_from_camera_to_finish(info, eng, 0):
        if not seen or info.jobs_done != seen[-1]:
            seen.append(info.jobs_done)
            for x0, y0, x1, y1 in tiles[:info.jobs_done]:
                assert np.array_equal(info.camera_tex[y0:y1 + 1, x0:x1 + 1], gfb[y0:y1 + 1, x0:x1 + 1])
    assert seen == sorted(seen) and all(v % 3 == 0 for v in seen)
    assert np.array_equal(info.camera_tex, gfb) and info.jobs_done == 40
    assert info.total_ray_casts == sum(int(gcasts[y0:y1 + 1, x0:x1 + 1].sum()) for x0, y0, x1, y1 in tiles)


@pytest.mark.parametrize("variant", VARIANTS)
def test_progressive_start_equals_one_shot(eng, variant):
    """Tile groups with overlapping reference tiles: each pixel traced once (first tile owns it)."""
    upload(eng, "Monkey", True)
    W, H = 160, 90
    tiles = E.make_tiles(W, H, 8)
    cam = E.camera(W, H, 3, 4)
    want = run(eng, cam, tiles=tiles, variant=variant)
    for per in (1, 7, 1000):
        got = run(eng, cam, tiles=tiles, variant=variant, progressive=per)
        for k in ("fb", "casts", "face", "rgb", "traced"):
            assert np.array_equal(got[k], want[k]), (per, k)
        assert np.array_equal(got["t"].view(np.uint32), want["t"].view(np.uint32))


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("wh", [(1, 1), (37, 23), (8, 8), (65, 9)])
def test_ragged_sizes_match_oracle(eng, wh, variant):
    W, H = wh
    upload(eng, "Monkey", True)
    s = O.Scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    f, t, _ = s.primary_hits(O.Camera(W, H))
    rgb, fb, casts, _ = s.render(O.Camera(W, H, spp=3, bounces=4), SEED)
    o = run(eng, E.camera(W, H), variant=variant)
    assert np.array_equal(o["face"], f) and np.array_equal(o["t"].view(np.uint32), t.view(np.uint32))
    o = run(eng, E.camera(W, H, 3, 4), variant=variant)
    assert np.array_equal(o["fb"], fb) and np.array_equal(o["casts"], casts)
    assert_rgb(o["rgb"], rgb)


def test_empty_tile_list_is_a_noop(eng):
    upload(eng, "Cube", True)
    o = run(eng, E.camera(16, 16), tiles=np.zeros((0, 4), np.int32))
    assert (o["fb"] == 0x7F7F7F7F).all() and o["traced"] == 0


@pytest.mark.parametrize("variant", VARIANTS)
def test_axis_parallel_rays_match_oracle(eng, variant):
    """Camera looking straight down -z from a box-plane coordinate: 1/0 = inf in the slab test,
    (b - o) * inf = NaN comparisons (renderer.cpp:43, aabb.h:29-93)."""
    upload(eng, "Cube", True)
    s = O.Scene(asset_path("Cube"), center=CENTERS["Cube"])
    for eye, facing in [((-0.256, 0.22, 0.0), (0.0, 0.0, -1.0)), ((0.744, 1.2200999, 0.0), (0.0, 0.0, -1.0)),
                        ((-0.256, 3.0, -3.56), (0.0, -1.0, 0.0))]:
        oc = O.Camera(33, 17, eye=eye, facing=facing)
        f, t, _ = s.primary_hits(oc)
        o = run(eng, E.camera(33, 17, eye=eye, facing=facing), variant=variant)
        assert np.array_equal(o["face"], f)
        assert np.array_equal(o["t"].view(np.uint32), t.view(np.uint32))


@pytest.mark.parametrize("variant", VARIANTS)
def test_spheres_and_planes_match_oracle(eng, variant):
    """get_intersection_data's sphere/plane branches (renderer.cpp:86-121) with the app's
    spheres and planes (app.cpp:114-129) next to the model."""
    sph = [((-1.0, 1.0, -7.0), 1.0, 2), ((1.0, 1.0, -7.0), 1.0, 3)]
    pln = [((0.0, 1.0, 0.0), 0.0, 4), ((1.0, 0.0, 0.0), -7.0, 5)]
    mats = [SKY, MODEL, ((0, 0, 0), (0.2, 0.8, 0.2), 0.3), ((0, 0, 0), (0.4, 0.8, 0.9), 0.9),
            ((0, 0, 0), (0.5, 0.5, 0.5), 0.0), ((0, 0.4, 0.6), (0.2, 0.3, 0.2), 0.0)]
    upload(eng, "Monkey", True, spheres=sph, planes=pln, materials=mats)
    s = O.Scene(asset_path("Monkey"), center=CENTERS["Monkey"], materials=mats, spheres=sph, planes=pln)
    rgb, fb, casts, ctr = s.render(O.Camera(96, 54, spp=2, bounces=5), SEED)
    o = run(eng, E.camera(96, 54, 2, 5), variant=variant)
    assert np.array_equal(o["fb"], fb) and np.array_equal(o["casts"], casts)
    assert_rgb(o["rgb"], rgb)
    assert o["traced"] == ctr["n_rays"]


def test_variants_agree_at_full_size_multibounce(eng):
    """Size-independent properties at the config-4 resolution (1920x1080, 4 spp, 5 bounces): the
    reference-work cell kernel (LANE) and the sample-parallel path engine agree bit for bit, and a
    re-render is identical (determinism: the path queues' order varies between runs, the outputs
    do not)."""
    upload(eng, "Dragon", True)
    cam = E.camera(1920, 1080, 4, 5)
    a = run(eng, cam, variant=E.ATR_KERNEL_LANE)
    b = run(eng, cam, variant=E.ATR_KERNEL_PATHS)
    c = run(eng, cam, variant=E.ATR_KERNEL_PATHS)
    for k in ["fb", "casts", "face"]:
        assert np.array_equal(a[k], b[k]) and np.array_equal(b[k], c[k])
    assert np.array_equal(a["rgb"].view(np.uint32), b["rgb"].view(np.uint32))
    assert a["traced"] == b["traced"] == c["traced"]


@pytest.mark.parametrize("variant", VARIANTS)
@pytest.mark.parametrize("name", ["monkey_1280x720_tree", "dragon_1920x1080_tree", "cube_256_tree",
                                  "monkey_1280x720_bf"])
def test_gpu_work_counters_equal_reference_work(eng, name, variant):
    """The instrumented kernel's reference-equivalent work (box tests, triangle tests, leaves)
    equals the oracle's counts of the reference algorithm on the same input -- the N_* of the
    roofline byte model."""
    g = GOLD["hits"][name]
    upload(eng, g["asset"], g["tree"])
    c = eng.counters(E.camera(g["W"], g["H"]), [[0, 0, g["W"] - 1, g["H"] - 1]], SEED, variant)
    for k in ["n_rays", "n_box", "n_leaf"]:
        assert c[k] == g["counters"][k], (k, c[k], g["counters"][k])
    exact_work = (E.ATR_KERNEL_LANE,)
    if variant not in exact_work and g["tree"]:
        # the clustered scan visits the same leaves but skips provably irrelevant triangles
        assert 0 < c["n_tri"] <= g["counters"]["n_tri"], (c["n_tri"], g["counters"]["n_tri"])
    else:
        assert c["n_tri"] == g["counters"]["n_tri"], (c["n_tri"], g["counters"]["n_tri"])


def test_bgr_exchange_reassembles_frames(eng):
    """The multi-GPU 3-byte exchange on one GPU: 3 ranks' packed shard frames (2 frames per
    launch) packed by atr_pack_bgr into one byte buffer laid out as rank 0 receives it
    (shard.frame_offsets), expanded and scattered by atr_scatter_bgr through the assembly index:
    every frame equals the full-frame render, and the bytes equal the host reference."""
    from atray_amd import shard as S
    upload(eng, "Dragon", True)
    W, H, F, world = 480, 270, 2, 3
    cams = [E.camera(W, H, 1, 1, eye=(0.1 + 0.05 * f, 2.0, 0.0)) for f in range(F)]
    plan = S.ShardPlan(W, H, world, 64)
    off = S.frame_offsets(plan, F)
    big = torch.zeros(3 * F * W * H, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    for r in range(world):
        n = plan.sizes[r]
        fb = torch.zeros(F * n, dtype=torch.int32, device="cuda")
        fr = E.atr_frame(E.ATR_LAYOUT_PACKED, fb.data_ptr(), None, None, None, None, None)
        eng.render_start_cameras(cams, plan.tiles[r], fr, n, SEED, stream=s)
        eng.pack_bgr(fb.data_ptr(), F * n, big[3 * off[r]:].data_ptr(), stream=s)
        torch.cuda.synchronize()
        want = S.pack_bgr_host(fb.cpu().numpy().view(np.uint32))
        assert np.array_equal(big[3 * off[r]:3 * off[r] + 3 * F * n].cpu().numpy(), want)
    dst = torch.from_numpy(S.frames_assembly_index(plan, F)).cuda()
    img = torch.zeros(F * W * H, dtype=torch.int32, device="cuda")
    eng.scatter_bgr(big.data_ptr(), F * W * H, dst.data_ptr(), img.data_ptr(), stream=s)
    torch.cuda.synchronize()
    for f in range(F):
        full = run(eng, cams[f])
        assert np.array_equal(img[f * W * H:(f + 1) * W * H].cpu().numpy().view(np.uint32).reshape(H, W), full["fb"])


@pytest.mark.parametrize("bgsel", ["sky", "first", "absent"])
def test_masked_exchange_reassembles_frames(eng, bgsel):
    """The masked exchange (atr_pack_bgr_masked / atr_scatter_bgr_masked / atr_unpack_masked /
    atr_unpack_masked_ranks, round 6): 3 ranks' packed
    shard frames (2 per launch) encoded against a background value -- the frame's common sky value,
    rank 0's first pixel, or a value no pixel has (every pixel then travels) -- decoded through the
    assembly index: every frame equals the full-frame render, the device stream equals the host
    reference byte for byte, and its device byte count is the stream's length."""
    from atray_amd import shard as S
    upload(eng, "Dragon", True)
    W, H, F, world = 480, 270, 2, 3
    cams = [E.camera(W, H, 1, 1, eye=(0.1 + 0.05 * f, 2.0, 0.0)) for f in range(F)]
    plan = S.ShardPlan(W, H, world, 64)
    off = S.frame_offsets(plan, F)
    dst = torch.from_numpy(S.frames_assembly_index(plan, F)).cuda()
    img = torch.zeros(F * W * H, dtype=torch.int32, device="cuda")
    img2 = torch.full((F * (W * H + 5),), 0x7F7F7F7F, dtype=torch.int32, device="cuda")
    img3 = torch.full((F * (W * H + 5),), 0x7F7F7F7F, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    bg = None
    streams = []
    for r in range(world):
        n = plan.sizes[r]
        fb = torch.zeros(F * n, dtype=torch.int32, device="cuda")
        fr = E.atr_frame(E.ATR_LAYOUT_PACKED, fb.data_ptr(), None, None, None, None, None)
        eng.render_start_cameras(cams, plan.tiles[r], fr, n, SEED, stream=s)
        torch.cuda.synchronize()
        if r == 0:
            fb0 = fb
        host = fb.cpu().numpy().view(np.uint32)
        if bg is None:
            bg = {"sky": S.background_value(host), "first": int(host[0]), "absent": 0x01000000}[bgsel]
        out = torch.full((E.pack_bgr_masked_bound(F * n),), 0xA5, dtype=torch.uint8, device="cuda")
        nbytes = torch.zeros(1, dtype=torch.int64, device="cuda")
        eng.pack_bgr_masked(fb.data_ptr(), F * n, bg, out.data_ptr(), nbytes.data_ptr(), stream=s)
        torch.cuda.synchronize()
        want = S.pack_bgr_masked_host(host, bg)
        assert int(nbytes.item()) == want.size
        assert np.array_equal(out[:want.size].cpu().numpy(), want)
        if bgsel == "sky":
            assert want.size < 0.3 * 3 * F * n  # mostly sky: far below the 3-byte exchange
        eng.scatter_bgr_masked(out.data_ptr(), F * n, dst[off[r]:].data_ptr(), img.data_ptr(), stream=s)
        # and straight from the tile list's blocks (atr_unpack_masked), frames W * H + 5 apart
        eng.unpack_masked(plan.tiles[r], W, H, out.data_ptr(), F, img2.data_ptr(), W * H + 5, stream=s)
        streams.append(out)
    # and all ranks' streams in one call (atr_unpack_masked_ranks); then ranks 1.. as streams and
    # rank 0 as its raw packed frames
    eng.unpack_masked_ranks(plan.tiles, W, H, [o.data_ptr() for o in streams], F, img3.data_ptr(), W * H + 5, stream=s)
    img4 = torch.full_like(img3, 0x7F7F7F7F)
    eng.unpack_masked_ranks(plan.tiles[1:] + [plan.tiles[0]], W, H, [o.data_ptr() for o in streams[1:]] + [fb0.data_ptr()],
                            F, img4.data_ptr(), W * H + 5, stream=s, raw=[0] * (world - 1) + [1])
    torch.cuda.synchronize()
    assert torch.equal(img3, img2) and torch.equal(img4, img2)
    for f in range(F):
        full = run(eng, cams[f])
        assert np.array_equal(img[f * W * H:(f + 1) * W * H].cpu().numpy().view(np.uint32).reshape(H, W), full["fb"])
        o = f * (W * H + 5)
        assert np.array_equal(img2[o:o + W * H].cpu().numpy().view(np.uint32).reshape(H, W), full["fb"])
        assert (img2[o + W * H:o + W * H + 5] == 0x7F7F7F7F).all()


def test_unpack_masked_ranks_batches_past_sixteen_sources(eng):
    """atr_unpack_masked_ranks with 20 sources (two launch pairs: 16 + 4), one of them holding no
    pixel: the assembled frame equals the full-frame render."""
    from atray_amd import shard as S
    upload(eng, "Dragon", True)
    W, H, world = 256, 160, 20
    cam = E.camera(W, H, 1, 1)
    plan = S.ShardPlan(W, H, world, 32)
    full = run(eng, cam)
    bg = S.background_value(full["fb"].ravel())
    s = torch.cuda.current_stream().cuda_stream
    tiles, outs = [], []
    for r in range(world):
        n = plan.sizes[r]
        if not n:
            continue
        fb = torch.zeros(n, dtype=torch.int32, device="cuda")
        eng.render_start(cam, plan.tiles[r], E.atr_frame(E.ATR_LAYOUT_PACKED, fb.data_ptr(), None, None, None, None,
                                                         None), SEED, stream=s)
        out = torch.zeros(E.pack_bgr_masked_bound(n), dtype=torch.uint8, device="cuda")
        nb = torch.zeros(1, dtype=torch.int64, device="cuda")
        eng.pack_bgr_masked(fb.data_ptr(), n, bg, out.data_ptr(), nb.data_ptr(), stream=s)
        torch.cuda.synchronize()
        tiles.append(plan.tiles[r])
        outs.append(out)
    assert len(tiles) > 16
    tiles.append([[0, 0, -1, -1]])  # a source without pixels (an empty rect): skipped
    outs.append(outs[0])
    img = torch.full((W * H,), 0x7F7F7F7F, dtype=torch.int32, device="cuda")
    eng.unpack_masked_ranks(tiles, W, H, [o.data_ptr() for o in outs], 1, img.data_ptr(), W * H, stream=s)
    torch.cuda.synchronize()
    assert np.array_equal(img.cpu().numpy().view(np.uint32).reshape(H, W), full["fb"])


def test_block_cache_eviction_waits_for_every_stream(eng):
    """A tile list's cached block set read by launches on two streams is rewritten only after both
    have finished (round-2 advice: the slot's event once covered only the later stream): a long
    PACKED multi-bounce render on stream A, a short render of the same tiles on stream B, then
    more distinct tile lists on B than the cache holds (24), which evicts the set while A may
    still run. A's frame must equal the same render on an idle GPU."""
    upload(eng, "Dragon", True)
    W, H = 480, 270
    cam = E.camera(W, H, 16, 5)
    tiles = E.make_shard_tiles(W, H, 64, 0, 2)
    want = run(eng, cam, tiles=tiles, layout=E.ATR_LAYOUT_PACKED)
    n = E.packed_size(tiles)
    dev = torch.device("cuda", 0)
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    fa = torch.full((n,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
    ca = torch.full((n,), -1, dtype=torch.int32, device=dev)
    eng.render_start(cam, tiles, E.atr_frame(E.ATR_LAYOUT_PACKED, fa.data_ptr(), None, None, None, ca.data_ptr(),
                                             None), SEED, stream=sa.cuda_stream)
    fb = torch.zeros(W * H, dtype=torch.int32, device=dev)
    frb = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, None, None)
    small = E.camera(W, H)
    eng.render_start(small, tiles, frb, SEED, stream=sb.cuda_stream)
    for k in range(30):
        eng.render_start(small, [[k, 0, W - 1 - k, H - 1]], frb, SEED, stream=sb.cuda_stream)
    torch.cuda.synchronize()
    rc, _ = eng.wait()
    assert rc == 0
    assert np.array_equal(fa.cpu().numpy().view(np.uint32), want["fb"])
    assert np.array_equal(ca.cpu().numpy().view(np.uint32), want["casts"])
