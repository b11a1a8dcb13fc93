"""Engine API behaviour on the GPU: argument validation before any state changes, and the path
engine's workspace bound (atr_workspace_info) with its out-of-memory fallback (capi.cpp
path_workspace / launch_paths / launch_kernels). Outputs are compared with a plain render of the
same camera: the schedule and batch size never change an output bit. Needs an MI355X (-m gpu)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from atray_amd import engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.goldens import SEED  # noqa: E402

pytestmark = pytest.mark.gpu


def make_engine():
    e = E.Engine(0)
    m = E.Mesh.load_obj(asset_path("Monkey"))
    box = m.translate_to(m.aabb(), CENTERS["Monkey"])
    e.upload([O.SKY, O.MODEL_MAT], [(m, E.Octree.build(m, 300), box, 1)])
    return e


@pytest.fixture(scope="module")
def eng():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    e = make_engine()
    yield e
    e.close()


def render(eng, cam, variant, stream=None, wait=True):
    W, H = cam.width, cam.height
    dev = torch.device("cuda", 0)
    fb = torch.full((W * H,), 0x7F7F7F7F, dtype=torch.int32, device=dev)
    casts = torch.full((W * H,), -1, dtype=torch.int32, device=dev)
    fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, casts.data_ptr(), None)
    s = stream or torch.cuda.current_stream()
    eng.render_start(cam, [[0, 0, W - 1, H - 1]], fr, SEED, stream=s.cuda_stream, variant=variant)
    if wait:
        assert eng.wait()[0] == 0
        torch.cuda.synchronize()
    return fb, casts


def test_invalid_schedules_rejected_before_any_state(eng):
    """Kernel codes outside the shipping set (the removed schedules 2-7 among them) and PATHS past its
    64 bounce launches are ATR_E_INVALID at every render entry point (atray.h), and a valid render
    afterwards is unaffected."""
    W, H = 64, 40
    want = render(eng, E.camera(W, H, 2, 3), E.ATR_KERNEL_AUTO)
    fb = torch.zeros(2 * W * H, dtype=torch.int32, device="cuda")
    fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, None, None)
    tiles = [[0, 0, W - 1, H - 1]]
    bad = [(v, E.camera(W, H, 2, 3)) for v in (2, 3, 4, 5, 6, 7, 11, 99)]
    bad.append((E.ATR_KERNEL_PATHS, E.camera(W, H, 1, 65)))
    for v, cam in bad:
        with pytest.raises(E.AtrError):
            eng.render_start(cam, tiles, fr, SEED, variant=v)
        with pytest.raises(E.AtrError):
            eng.render_start_cameras([cam, cam], tiles, fr, W * H, SEED, variant=v)
        with pytest.raises(E.AtrError):
            eng.render_start_progressive(cam, tiles, fr, SEED, 1, variant=v)
        with pytest.raises(E.AtrError):
            eng.cell_costs(cam, SEED, v)
    got = render(eng, E.camera(W, H, 2, 3), E.ATR_KERNEL_AUTO)
    assert all(torch.equal(a, b) for a, b in zip(want, got))
    # AUTO beyond PATHS' bounce launches renders on FLAT (the same outputs as LANE)
    deep = E.camera(W, H, 1, 65)
    a, b = render(eng, deep, E.ATR_KERNEL_AUTO), render(eng, deep, E.ATR_KERNEL_LANE)
    assert all(torch.equal(x, y) for x, y in zip(a, b))


def test_path_workspaces_bounded_over_many_streams(eng):
    """PATHS renders on 7 streams at once hold at most 4 workspaces (a stream without one takes an
    idle or the least recently used one after a GPU-side wait), and every render equals the
    one-stream render."""
    W, H = 160, 96
    cam = E.camera(W, H, 4, 3)
    want = render(eng, cam, E.ATR_KERNEL_PATHS)
    streams = [torch.cuda.Stream() for _ in range(7)]
    outs = []
    for rep in range(2):
        for s in streams:
            outs.append(render(eng, cam, E.ATR_KERNEL_PATHS, stream=s, wait=False))
    torch.cuda.synchronize()
    assert eng.wait()[0] == 0
    info = eng.workspace_info()
    assert 1 <= info["workspaces"] <= 4, info
    for fb, casts in outs:
        assert torch.equal(fb, want[0]) and torch.equal(casts, want[1])


def test_path_workspace_grows_once_to_a_whole_batch():
    """A workspace holds its first launch's paths rounded up to 2^24 (within one batch); a later
    launch that needs more grows it straight to a whole batch, so launches after that never regrow
    (round 6: a regrow inside a timed multi-frame run cost a c4 line 4x). 2^26-path batches;
    128x128 at 64 spp, 1 bounce (no queue sort: 144 B per path): 1, 17 and 24 frames per launch, and
    every frame of the 24-frame launch equals the one-frame render."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    W, H = 128, 128
    cam = E.camera(W, H, 64, 1)
    e = make_engine()
    try:
        e.set_tuning(path_batch_log2=26)
        want = render(e, cam, E.ATR_KERNEL_PATHS)  # 1.05 M paths
        b1 = e.workspace_info()["device_bytes"]
        assert (1 << 24) * 144 <= b1 < (1 << 24) * 144 + (1 << 20), b1
        sizes = []
        for n in (17, 24, 17):  # 17.8 M paths: past 2^24 -> one 2^26 batch; then no change
            fb = torch.zeros(n * W * H, dtype=torch.int32, device="cuda")
            casts = torch.zeros(n * W * H, dtype=torch.int32, device="cuda")
            fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, casts.data_ptr(), None)
            e.render_start_cameras([cam] * n, [[0, 0, W - 1, H - 1]], fr, W * H, SEED,
                                   variant=E.ATR_KERNEL_PATHS)
            assert e.wait()[0] == 0
            torch.cuda.synchronize()
            info = e.workspace_info()
            assert info["workspaces"] == 1, info
            sizes.append(info["device_bytes"])
            for f in (0, n - 1):
                assert torch.equal(fb[f * W * H:(f + 1) * W * H], want[0])
                assert torch.equal(casts[f * W * H:(f + 1) * W * H], want[1])
        assert (1 << 26) * 144 <= sizes[0] < (1 << 26) * 144 + (1 << 20), sizes
        assert sizes[1] == sizes[0] == sizes[2], sizes
    finally:
        e.close()
        torch.cuda.empty_cache()


def test_path_workspace_out_of_memory_halves_the_batch():
    """With most of the device memory taken (a torch allocation of all but ~600 MB), a PATHS render
    whose default batch needs a 1.2-GB workspace (480x270 at 64 spp: 2^23 paths) halves its batch
    until the workspace fits (then drops the queue sort's buffers): same outputs as the render with
    memory, no error. (Below 2^16 paths the engine renders on FLAT; not forced here: the kernels'
    scratch needs memory too.)"""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    W, H = 480, 270
    cam = E.camera(W, H, 64, 3)
    e = make_engine()
    hog = None
    try:
        want = render(e, cam, E.ATR_KERNEL_FLAT)  # block lists, counters, scratch: before the hog
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        free, _ = torch.cuda.mem_get_info()
        hog = torch.empty(max(0, free - (600 << 20)), dtype=torch.uint8, device="cuda")
        got = render(e, cam, E.ATR_KERNEL_PATHS)
        assert torch.equal(got[0], want[0]) and torch.equal(got[1], want[1])
        info = e.workspace_info()
        # smaller than the default batch's queues alone (2^23 paths x 144 B): the batch was halved
        assert info["workspaces"] == 1 and 0 < info["device_bytes"] < (1 << 23) * 144, info
        del hog
        hog = None
        torch.cuda.empty_cache()
    finally:
        del hog
        e.close()
        torch.cuda.empty_cache()
