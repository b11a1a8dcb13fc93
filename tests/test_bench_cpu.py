"""bench.py on CPU: `--gpus N` starts N ranks itself (torch.distributed.run child, gloo here) and
the shard plan + gather + frame assembly reproduce every frame; the launch split does not depend
on the step count beyond rounding. The render kernel itself runs only on the GPU box (-m gpu);
here --selftest puts a synthetic fill (pixel index) in its place."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert lines, out[-2000:]
    return json.loads(lines[-1])


@pytest.mark.parametrize("n,exchange,plan", [(2, "bgr", "cost"), (2, "bgrx", "cost"), (3, "bgr", "cost"), (8, "bgr", "cost"),
                                            (2, "masked", "cost"), (3, "masked", "cost"), (8, "masked", "cost"),
                                            (3, "masked", "curve")])
def test_bench_gpus_n_spawns_n_ranks_and_assembles_frames(n, exchange, plan):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--selftest",
                        "--steps", "11", "--warmup", "1", "--frames-per-launch", "4", "--exchange", exchange, "--plan", plan],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == n and d["selftest"] is True and d["config"]["exchange"] == exchange
    assert d["frames_checked"] == 11
    assert d["check_mismatched_pixels"] == 0 and d["total_ray_casts_ok"] is True
    assert sum(d["config"]["shard_pixels"]) == 480 * 272


def test_bench_rejects_world_size_mismatch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--selftest"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


@pytest.mark.parametrize("k,f", [(20, 8), (48, 8), (7, 8), (1, 1), (17, 16), (0, 8)])
@pytest.mark.parametrize("streams", [1, 2, 3])
def test_launch_sizes_are_balanced(k, f, streams):
    s = bench.launch_sizes(k, f, streams)
    assert sum(s) == k and all(1 <= x <= f for x in s)
    assert (max(s) - min(s) <= 1) if s else k == 0
    n = (k + f - 1) // f
    # fewest launches that is a multiple of the streams (or one launch per frame)
    assert len(s) == min(k, -(-n // streams) * streams)
    if k >= streams:  # round-robin: every stream gets the same frames, to one
        per = [sum(s[q::streams]) for q in range(streams)]
        assert max(per) - min(per) <= 1


def test_curve_plan_is_compact_and_balanced():
    """ShardPlan.curve: every grid tile owned once, the recursive bisection balanced within about a
    tile's cost per cut (rank 0 lighter by its assembly share), and each rank's tiles compact (a
    near-rectangle: its bounding box at most twice its tiles' area)."""
    import numpy as np
    from atray_amd import shard as S
    W, H, side = 1920, 1080, 32
    grid = S.E.shard_grid(W, H, side)
    costs = (np.arange(len(grid)) * 7919) % 97 + 1
    for world in (2, 4, 8):
        p = S.ShardPlan.curve(costs, W, H, world, side, 0.1)
        assert sorted(np.concatenate([np.asarray(t).reshape(-1, 4)[:, 0] + W * np.asarray(t).reshape(-1, 4)[:, 1]
                                      for t in p.tiles])) == sorted(grid[:, 0] + W * grid[:, 1])
        loads = np.array([costs[p.owner == r].sum() for r in range(world)], np.float64)
        extra = 0.1 * costs.sum() / world
        share = (costs.sum() + extra) / world
        assert abs(loads[0] - (share - extra)) <= 3 * costs.max()
        assert np.all(np.abs(loads[1:] - share) <= 3 * costs.max())
        for t in p.tiles:
            t = np.asarray(t).reshape(-1, 4)
            area = (t[:, 2].max() - t[:, 0].min() + 1) * (t[:, 3].max() - t[:, 1].min() + 1)
            own = ((t[:, 2] - t[:, 0] + 1) * (t[:, 3] - t[:, 1] + 1)).sum()
            assert area <= 2 * own, (world, area, own)


def test_orbit_cameras_are_distinct():
    eyes = {bench.orbit_eye(k) for k in range(bench.ORBIT_PERIOD)}
    assert len(eyes) == bench.ORBIT_PERIOD
    assert bench.orbit_eye(0) == bench.APP_EYE


def test_path_dispatches_count_the_queue_sort():
    """The PMC selection of the path engine's timed dispatches (bench.path_dispatches): per batch one
    camera, bounces - 1 bounce and one resolve launch, and with the queue sort four sort kernels
    per bounce launch; a c4 launch of 8 frames at 2^28-path batches is 4 batches."""
    class A:
        steps, frames_per_launch, streams = 8, 8, 1
    tiles = [[0, 0, 1919, 1079]]
    d = bench.path_dispatches(A, tiles, 1920, 1080, 64, 5, 28, sort_bits=5)
    assert d["path_camera_kernel"] == 4 and d["path_bounce_kernel"] == 16 and d["path_resolve_kernel"] == 4
    for k in ("path_sort_sums", "path_sort_part_scan", "path_sort_scan", "path_sort_rank"):
        assert d[k] == 16
    d0 = bench.path_dispatches(A, tiles, 1920, 1080, 64, 5, 28, sort_bits=0)
    assert set(d0) == {"path_camera_kernel", "path_bounce_kernel", "path_resolve_kernel"}
    assert bench.path_dispatches(A, tiles, 1920, 1080, 64, 1, 28, sort_bits=5).keys() == d0.keys()


def test_streams_default_per_config():
    """bench.py --streams 0 (default): one for the path-engine configs; for the 1-spp configs one
    while a single launch holds every timed frame (the driver's 20), else two."""
    assert {c: bench.default_streams(c, 20) for c in bench.CONFIGS} == {"c1": 1, "c2": 1, "c3": 1, "c4": 1, "c5": 1}
    assert {c: bench.default_streams(c, 48) for c in bench.CONFIGS} == {"c1": 2, "c2": 2, "c3": 2, "c4": 1, "c5": 1}
    assert bench.launch_sizes(20, bench.MAX_FRAME_CAMS, 1) == [20]
    assert {c: bench.default_streams(c, 20, 8) for c in bench.CONFIGS} == {"c1": 2, "c2": 2, "c3": 2, "c4": 1, "c5": 1}
