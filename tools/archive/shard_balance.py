"""Load balance of the multi-GPU tile sharding, measured on ONE GPU: each rank's shard of a
frame (atr_make_shard_tiles, or a cost-balanced plan) is rendered alone and timed with HIP
events; the predicted N-GPU frame time is the slowest shard.

python tools/shard_balance.py [--config c3] [--worlds 2,4,8] [--sides 32,64] [--plans rr,lpt]
Prints JSON: per (plan, side, world): per-rank ms, max, mean, ideal (full frame / N), balance.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from atray_amd import shard as S  # noqa: E402
from bench import CONFIGS, SEED  # noqa: E402


STREAMS = [None]


def timed(eng, cam, tiles, fr, stream, iters):
    """ms per frame with len(STREAMS) frames in flight (one stream each), as bench.py runs."""
    eng.render_start(cam, tiles, fr, SEED, stream=stream)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record()
    for k in range(iters * len(STREAMS)):
        s = STREAMS[k % len(STREAMS)]
        eng.render_start(cam, tiles, fr, SEED, stream=s.cuda_stream)
    ends = []
    for s in STREAMS:
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        ends.append(e)
    torch.cuda.synchronize()
    return max(t0.elapsed_time(e) for e in ends) / (iters * len(STREAMS))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--sides", default="32,64")
    ap.add_argument("--plans", default="rr,lpt")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--streams", type=int, default=1)
    args = ap.parse_args()
    STREAMS[:] = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(args.streams - 1)]
    asset, W, H, spp, bounces, use_tree = CONFIGS[args.config]
    mesh = E.Mesh.load_obj(asset_path(asset))
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = E.Octree.build(mesh, 300) if use_tree else None
    eng = E.Engine(0)
    eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)],
               [(mesh, tree, box, 1)])
    cam = E.camera(W, H, spp, bounces)
    stream = torch.cuda.current_stream().cuda_stream
    packed = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    fr = E.atr_frame(E.ATR_LAYOUT_PACKED, packed.data_ptr(), None, None, None, None, None)
    full = timed(eng, cam, [[0, 0, W - 1, H - 1]], fr, stream, args.iters)
    out = {"config": args.config, "streams": args.streams, "full_frame_ms": round(full, 4), "runs": []}
    for plan in args.plans.split(","):
        for side in [int(x) for x in args.sides.split(",")]:
            for world in [int(x) for x in args.worlds.split(",")]:
                if plan == "rr":
                    shards = S.ShardPlan(W, H, world, side).tiles
                else:
                    costs = S.tile_costs(eng, cam, W, H, side, SEED)
                    shards = S.ShardPlan.balanced(costs, W, H, world, side).tiles
                ms = [timed(eng, cam, t, fr, stream, args.iters) for t in shards]
                out["runs"].append({"plan": plan, "side": side, "world": world,
                                    "rank_ms": [round(x, 4) for x in ms], "max": round(max(ms), 4),
                                    "mean": round(float(np.mean(ms)), 4), "ideal": round(full / world, 4),
                                    "balance": round(float(np.mean(ms)) / max(ms), 4),
                                    "speedup_pred": round(full / max(ms), 3)})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
