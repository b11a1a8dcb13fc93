"""Does the GPU overlap small render launches? Full frame as one kernel vs the same frame as 8
shard kernels on 1 or 8 streams, one shard repeated with S frames in flight, and the host-side
cost of a render_start call.

python tools/concurrency_probe.py [--config c3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import atray_amd.engine as E  # noqa: E402
from atray_amd import shard as S  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from bench import CONFIGS, SEED  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=12)
    args = ap.parse_args()
    asset, W, H, spp, bounces, use_tree = CONFIGS[args.config]
    mesh = E.Mesh.load_obj(asset_path(asset))
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = E.Octree.build(mesh, 300) if use_tree else None
    eng = E.Engine(0)
    eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)],
               [(mesh, tree, box, 1)])
    cam = E.camera(W, H, spp, bounces)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(7)]
    buf = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    fr = E.atr_frame(E.ATR_LAYOUT_PACKED, buf.data_ptr(), None, None, None, None, None)
    costs = S.tile_costs(eng, cam, W, H, 64, SEED)
    plan = S.ShardPlan.balanced(costs, W, H, 8, 64)
    shard_tiles = [E.tiles_array(t) for t in plan.tiles]
    full = E.tiles_array([[0, 0, W - 1, H - 1]])

    def run(jobs):
        """jobs: list of (tiles, stream index); returns ms for all of them, repeated iters times."""
        for t, q in jobs:
            eng.render_start(cam, t, fr, SEED, stream=streams[q].cuda_stream)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        h0 = time.perf_counter()
        for _ in range(args.iters):
            for t, q in jobs:
                eng.render_start(cam, t, fr, SEED, stream=streams[q].cuda_stream)
        host = (time.perf_counter() - h0) / (args.iters * len(jobs)) * 1e3
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.iters * 1e3, host

    out = {}
    out["full_1kernel_ms"], out["host_ms_per_call_full"] = run([(full, 0)])
    out["full_as_8_shards_1stream_ms"], _ = run([(shard_tiles[r], 0) for r in range(8)])
    out["full_as_8_shards_8streams_ms"], out["host_ms_per_call_shard"] = run([(shard_tiles[r], r) for r in range(8)])
    for nstr in (1, 4, 8):
        ms, _ = run([(shard_tiles[0], q) for q in range(nstr)])
        out[f"shard0_x{nstr}_streams_ms_per_frame"] = ms / nstr
    print(json.dumps({k: round(v, 4) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
