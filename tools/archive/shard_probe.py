"""One rank's shard of an N-way cost-balanced plan on one GPU: kernel time alone, ms per frame
with S frames in flight, and the wave lifetimes of that shard's launch (why small shards do
not scale: the slowest waves, not the work, set the launch time).

python tools/shard_probe.py [--world 8] [--side 64] [--variants cl,ps] [--streams 1,2,3,4]
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

VARS = {"cl": E.ATR_KERNEL_CLUSTER, "ps": E.ATR_KERNEL_PERSIST, "auto": E.ATR_KERNEL_AUTO}


def per_frame(eng, cam, tiles, frames, streams, iters, variant, fpl=1, stride=0):
    def go(fr, s):
        if fpl > 1:
            eng.render_start_frames(cam, tiles, fr, fpl, stride, SEED, stream=s.cuda_stream, variant=variant)
        else:
            eng.render_start(cam, tiles, fr, SEED, stream=s.cuda_stream, variant=variant)
    for q, s in enumerate(streams):
        go(frames[q], s)
    torch.cuda.synchronize()
    t0 = torch.cuda.Event(enable_timing=True)
    t0.record(streams[0])
    for s in streams[1:]:
        s.wait_stream(streams[0])
    n = iters * len(streams)
    for k in range(n):
        q = k % len(streams)
        go(frames[q], streams[q])
    ends = []
    for s in streams:
        e = torch.cuda.Event(enable_timing=True)
        e.record(s)
        ends.append(e)
    torch.cuda.synchronize()
    return max(t0.elapsed_time(e) for e in ends) / (n * fpl)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--side", type=int, default=64)
    ap.add_argument("--variants", default="cl,ps")
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--fpl", default="1", help="frames per launch values (atr_render_start_frames)")
    args = ap.parse_args()
    asset, W, H, spp, bounces, use_tree = CONFIGS[args.config]
    mesh = E.Mesh.load_obj(asset_path(asset))
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = E.Octree.build(mesh, 300) if use_tree else None
    eng = E.Engine(0)
    eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)],
               [(mesh, tree, box, 1)])
    cam = E.camera(W, H, spp, bounces)
    costs = S.tile_costs(eng, cam, W, H, args.side, SEED)
    plan = S.ShardPlan.balanced(costs, W, H, args.world, args.side) if args.world > 1 else S.ShardPlan(W, H, 1, args.side)
    rank = int(np.argmax([costs[plan.owner == r].sum() for r in range(args.world)])) if args.world > 1 else 0
    tiles = E.tiles_array(plan.tiles[rank])
    smax = max(int(x) for x in args.streams.split(","))
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(smax - 1)]
    n = max(1, plan.sizes[rank])
    fmax = max(int(x) for x in args.fpl.split(","))
    bufs = [torch.zeros(n * fmax, dtype=torch.int32, device="cuda") for _ in range(smax)]
    frames = [E.atr_frame(E.ATR_LAYOUT_PACKED, b.data_ptr(), None, None, None, None, None) for b in bufs]
    out = {"config": args.config, "world": args.world, "side": args.side, "rank": rank,
           "shard_pixels": int(plan.sizes[rank]), "frame_pixels": W * H, "variants": {}}
    for v in args.variants.split(","):
        res = {}
        for fpl in [int(x) for x in args.fpl.split(",")]:
            for sn in [int(x) for x in args.streams.split(",")]:
                key = f"s{sn}_ms_per_frame" + (f"_f{fpl}" if fpl > 1 else "")
                res[key] = round(per_frame(eng, cam, tiles, frames, streams[:sn], args.iters, VARS[v], fpl, n), 4)
        if v == "ps":  # persistent waves: no per-cell trace
            out["variants"][v] = res
            continue
        tr = eng.wave_trace(cam, tiles, SEED, VARS[v]).astype(np.int64)
        life = (tr[:, 1] - tr[:, 0]) / 100.0
        span = (tr[:, 1].max() - tr[:, 0].min()) / 100.0
        res["trace_span_us"] = round(float(span), 1)
        res["wave_life_us_pctl"] = {str(q): round(float(np.percentile(life, q)), 1) for q in (50, 90, 99, 100)}
        res["waves"] = int(len(tr))
        out["variants"][v] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
