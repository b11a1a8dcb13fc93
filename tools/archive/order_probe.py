"""Does the order of the 8x8 work blocks bound the render kernel (tail effect)? Kernel time of
the same frame with blocks in row-major order, heaviest-first and lightest-first (per-block
cost measured by one calibration render), under the current XCD mapping (ATR_XCD_CHUNK).

python tools/order_probe.py [--config c3]
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
from bench import CONFIGS, SEED  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variant", type=int, default=0)
    args = ap.parse_args()
    asset, W, H, spp, bounces, use_tree = CONFIGS[args.config]
    mesh = E.Mesh.load_obj(asset_path(asset))
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = E.Octree.build(mesh, 300) if use_tree else None
    eng = E.Engine(0)
    eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)],
               [(mesh, tree, box, 1)])
    cam = E.camera(W, H, spp, bounces)
    cells = E.shard_grid(W, H, 8)
    cost = eng.tile_costs(cam, cells, SEED)
    buf = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, buf.data_ptr(), None, None, None, None, None)
    stream = torch.cuda.current_stream().cuda_stream
    orders = {"full_tile": np.array([[0, 0, W - 1, H - 1]], np.int32), "cells_rowmajor": cells,
              "heavy_first": cells[np.argsort(-cost, kind="stable")],
              "light_first": cells[np.argsort(cost, kind="stable")]}
    out = {"chunk": os.environ.get("ATR_XCD_CHUNK", "0")}
    for name, tl in orders.items():
        t = E.tiles_array(tl)
        for _ in range(2):
            eng.render_start(cam, t, fr, SEED, stream=stream, variant=args.variant)
        torch.cuda.synchronize()
        ms = []
        for _ in range(args.iters):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            eng.render_start(cam, t, fr, SEED, stream=stream, variant=args.variant)
            b.record()
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
        out[name] = round(float(np.median(ms)), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
