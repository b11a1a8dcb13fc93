"""Kernel A/B timing + work counters on the GPU (interleaved variants in one process).

python tools/kprof.py [--config c3] [--rounds 5] [--iters 10] [--variants lane,wave]
Prints per-variant kernel ms (median/min over rounds, HIP events on the launch stream), Mrays/s,
the reference-equivalent work counters and the wave-schedule convergence
(lane triangle tests / (64 x wave-level triangle iterations)).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--variants", default="lane,wave")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--bounces", type=int, default=None)
    args = ap.parse_args()
    import numpy as np
    import torch

    import atray_amd.engine as E
    from atray_amd.assets import CENTERS, asset_path
    from bench import CONFIGS, SEED
    asset, W, H, spp, bounces, use_tree = CONFIGS[args.config]
    spp = args.spp or spp
    bounces = args.bounces or bounces
    mesh = E.Mesh.load_obj(asset_path(asset))
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = E.Octree.build(mesh, 300) if use_tree else None
    eng = E.Engine(0)
    eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)],
               [(mesh, tree, box, 1)])
    cam = E.camera(W, H, spp, bounces)
    tiles = [[0, 0, W - 1, H - 1]]
    fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, None, None)
    stream = torch.cuda.current_stream().cuda_stream
    names = {"lane": E.ATR_KERNEL_LANE, "wave": E.ATR_KERNEL_WAVE, "tile": E.ATR_KERNEL_TILE,
             "tile8": E.ATR_KERNEL_TILE8, "wf": E.ATR_KERNEL_WAVEFRONT, "cl": E.ATR_KERNEL_CLUSTER,
             "ps": E.ATR_KERNEL_PERSIST, "occ4": 20, "occ5": 21,
             "occ6": 22, "occ8": 24, "cl4": 36, "cl5": 37, "cl6": 38, "cl8": 40,
             "k4o4": 52, "k4o5": 53, "k4o6": 54, "k4o8": 56, "flat": E.ATR_KERNEL_FLAT,
             "hyb": E.ATR_KERNEL_HYBRID, "fl4": 68, "fl5": 69, "hyb4": 84, "hyb5": 85, "hyb6": 86}
    vs = args.variants.split(",")
    res = {v: [] for v in vs}
    def ctr_variant(code):
        if code < 16: return code
        if code >= 80: return E.ATR_KERNEL_HYBRID
        if code >= 64: return E.ATR_KERNEL_FLAT
        return E.ATR_KERNEL_CLUSTER if code >= 32 else E.ATR_KERNEL_LANE
    ctrs = {v: eng.counters(cam, tiles, SEED, ctr_variant(names[v])) for v in vs}
    for v in vs:  # warm
        eng.render_start(cam, tiles, fr, SEED, stream=stream, variant=names[v])
    torch.cuda.synchronize()
    for _ in range(args.rounds):
        for v in vs:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(args.iters):
                eng.render_start(cam, tiles, fr, SEED, stream=stream, variant=names[v])
            b.record()
            torch.cuda.synchronize()
            res[v].append(a.elapsed_time(b) / args.iters)
    out = {"config": args.config, "W": W, "H": H, "spp": spp, "bounces": bounces,
           "hyb": [os.environ.get("ATR_HYB_A"), os.environ.get("ATR_HYB_B")]}
    for v in vs:
        c = ctrs[v]
        ms = float(np.median(res[v]))
        d = {"ms_median": round(ms, 4), "ms_min": round(float(np.min(res[v])), 4),
             "mrays_s": round(c["n_rays"] / ms / 1e3, 2), "counters": c}
        if c["wave_tri_iters"]:
            d["wave_convergence"] = round(c["n_tri"] / (64.0 * c["wave_tri_iters"]), 4)
        out[v] = d
    print(json.dumps(out, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
