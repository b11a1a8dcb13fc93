"""Per-8x8-block GPU cost (shader clocks, default kernel) of a config's frame, saved as an
(H/8, W/8) array for offline analysis (which blocks bound the per-wave latency).

python tools/block_costs.py [--config c3] [--out gpurun_out/block_costs_c3.npy]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from bench import CONFIGS, SEED  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "block_costs_c3.npy"))
    ap.add_argument("--reps", type=int, default=3)
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
    reps = np.stack([eng.tile_costs(cam, cells, SEED) for _ in range(args.reps)])
    c = np.median(reps, 0).reshape((H + 7) // 8, (W + 7) // 8)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    np.save(args.out, c)
    nz = c[c > 0]
    print(json.dumps({"blocks": int(c.size), "max": float(c.max()), "mean": float(c.mean()),
                      "p50": float(np.percentile(nz, 50)), "p90": float(np.percentile(nz, 90)),
                      "p99": float(np.percentile(nz, 99)), "sum": float(c.sum()),
                      "rep_spread": float(np.max(np.abs(reps - np.median(reps, 0))) / max(1.0, c.max()))}))


if __name__ == "__main__":
    main()
