"""Where the FLAT/HYBRID waves spend their time: wave clocks in DFS passes, lane-private leaf
scans and dealt rounds (atr_render_phase_clocks, instrumented build) on Dragon 1920x1080, for the
primary-ray frame (HYBRID) and a multi-bounce frame (FLAT).

python tools/phase_probe.py [--spp 4]   (library built with make EXTRA=-DATR_PHASE_CLOCKS)

Measured (c3 one frame, HYBRID): DFS passes 6%, lane-private scans 41%, dealt rounds 10%, step
preparation 10%, whole tree query 69% of the wave clocks; FLAT at 4 spp x 5 bounces: passes 34%,
dealt rounds 49%, lane-private 9%, tree queries 95%.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from bench import MATERIALS, SEED  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=4)
    args = ap.parse_args()
    mesh = E.Mesh.load_obj(asset_path("Dragon"))
    box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
    tree = E.Octree.build(mesh, 300)
    eng = E.Engine(0)
    eng.upload(MATERIALS, [(mesh, tree, box, 1)])
    W, H = 1920, 1080
    tiles = [[0, 0, W - 1, H - 1]]
    out = {}
    for name, cam, var in (("c3_hybrid", E.camera(W, H), E.ATR_KERNEL_HYBRID),
                           ("c3_flat", E.camera(W, H), E.ATR_KERNEL_FLAT),
                           (f"spp{args.spp}_b5_flat", E.camera(W, H, args.spp, 5), E.ATR_KERNEL_FLAT)):
        eng.phase_clocks(cam, tiles, SEED, var)  # warm
        p = eng.phase_clocks(cam, tiles, SEED, var)
        w = max(1, p["wave"])
        out[name] = {**p, **{k + "_frac": round(p[k] / w, 3) for k in ("pass", "lane_private", "dealt", "step_prep", "scan")}}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
