"""Occupancy timeline of one render launch from the per-wave trace (atr_render_wave_trace):
how many waves each SIMD holds over time, per XCD work and end times, wave lifetimes.

python tools/wave_trace.py [--config c3] [--variant 0] [--out gpurun_out/wave_trace_c3.npy]
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
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--side", type=int, default=0, help="tile side (0 = one full-frame tile)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "wave_trace_c3.npy"))
    args = ap.parse_args()
    asset, W, H, spp, bounces, use_tree = CONFIGS[args.config]
    mesh = E.Mesh.load_obj(asset_path(asset))
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = E.Octree.build(mesh, 300) if use_tree else None
    eng = E.Engine(0)
    eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)],
               [(mesh, tree, box, 1)])
    cam = E.camera(W, H, spp, bounces)
    tiles = E.shard_grid(W, H, args.side) if args.side else np.array([[0, 0, W - 1, H - 1]], np.int32)
    eng.wave_trace(cam, tiles, SEED, args.variant)  # warm
    tr = eng.wave_trace(cam, tiles, SEED, args.variant).astype(np.int64)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    np.save(args.out, tr)
    t0, t1, hw = tr[:, 0], tr[:, 1], tr[:, 2]
    hwid, xcc = hw & 0xFFFFFFFF, hw >> 32
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 15
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 7
    slot = ((xcc * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
    T0 = t0.min()
    span = (t1.max() - T0) / 100.0  # us (100 MHz)
    life = (t1 - t0) / 100.0
    nslots = len(np.unique(slot))
    # resident waves per SIMD slot, sampled every 1 us
    grid = np.arange(0, span + 1.0, 1.0)
    s_ = (t0 - T0) / 100.0
    e_ = (t1 - T0) / 100.0
    res = np.zeros(len(grid))
    order = np.argsort(s_)
    for i in range(len(grid)):
        res[i] = np.count_nonzero((s_ <= grid[i]) & (e_ > grid[i]))
    per_xcd = {int(x): {"waves": int((xcc == x).sum()), "busy_us": round(float(life[xcc == x].sum()), 1),
                        "end_us": round(float(e_[xcc == x].max()), 1)} for x in np.unique(xcc)}
    heavy = life > 20.0
    out = {"blocks": int(len(tr)), "span_us": round(float(span), 1), "simd_slots_seen": int(nslots),
           "mean_resident_per_simd": round(float(life.sum() / span / 1024), 3),
           "resident_timeline_per_simd_every_50us": [round(float(res[i] / 1024), 2) for i in range(0, len(grid), 50)],
           "life_us_pctl": {str(q): round(float(np.percentile(life, q)), 2) for q in (50, 75, 90, 99, 100)},
           "heavy_waves(>20us)": int(heavy.sum()), "heavy_start_us_pctl": {
               str(q): round(float(np.percentile(s_[heavy], q)), 1) for q in (0, 50, 90, 100)} if heavy.any() else {},
           "per_xcd": per_xcd}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
