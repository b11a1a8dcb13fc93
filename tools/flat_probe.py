"""Multi-bounce (FLAT) diagnostics on the c4 geometry (Dragon 1920x1080, app camera): per-ray work
counters, bounce-loop lane use (atr_render_path_counters) and kernel time for a few bounce limits.
Usage: python tools/flat_probe.py [spp] [variant-code ...]   (prints one JSON object)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402

SEED = 0x853C49E6748FEA9B
spp = int(sys.argv[1]) if len(sys.argv) > 1 else 4
variants = [int(v) for v in sys.argv[2:]] or [E.ATR_KERNEL_FLAT]
W, H = 1920, 1080
mesh = E.Mesh.load_obj(asset_path("Dragon"))
box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
tree = E.Octree.build(mesh, 300)
eng = E.Engine(0)
eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)], [(mesh, tree, box, 1)])
tiles = [[0, 0, W - 1, H - 1]]
fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
casts = torch.zeros(W * H, dtype=torch.int32, device="cuda")
tr = torch.zeros(1, dtype=torch.int64, device="cuda")
fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, casts.data_ptr(), tr.data_ptr())
s = torch.cuda.current_stream()
out = {"spp": spp, "runs": []}


def timed(cam, v, n=3):
    evs = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.render_start(cam, tiles, fr, SEED, stream=s.cuda_stream, variant=v)
        b.record(s)
        evs.append((a, b))
    torch.cuda.synchronize()
    return min(a.elapsed_time(b) for a, b in evs)


for v in variants:
    for bounces in (2, 3, 5):
        cam = E.camera(W, H, spp, bounces)
        tr.zero_()
        eng.render_start(cam, tiles, fr, SEED, stream=s.cuda_stream, variant=v)
        torch.cuda.synchronize()
        rays = int(tr.item())
        ms = timed(cam, v)
        row = {"variant": v, "bounces": bounces, "ms": round(ms, 3), "rays": rays,
               "mrays_s": round(rays / ms / 1e3, 1), "casts": int(casts.sum().item())}
        if bounces == 5:
            ctr = eng.counters(cam, tiles, SEED, v)
            n = max(1, ctr["n_rays"])
            row["per_ray"] = {k: round(val / n, 3) for k, val in ctr.items()}
            row["path"] = eng.path_counters(cam, tiles, SEED, v)
            row["simd"] = eng.simd_counters(cam, tiles, SEED, v)
        out["runs"].append(row)
        print(json.dumps(row), flush=True)
c3 = E.camera(W, H)
out["c3_hybrid_ms"] = round(timed(c3, E.ATR_KERNEL_HYBRID), 3)
out["c3_hybrid_simd"] = eng.simd_counters(c3, tiles, SEED, E.ATR_KERNEL_HYBRID)
if os.environ.get("PHASES"):  # library built with -DATR_PHASE_CLOCKS (ATRAY_LIB)
    for name, cam, v in (("c3_hybrid", c3, E.ATR_KERNEL_HYBRID), ("c4_flat", E.camera(W, H, spp, 5), variants[0])):
        eng.phase_clocks(cam, tiles, SEED, v)
        p = eng.phase_clocks(cam, tiles, SEED, v)
        out["phases_" + name] = {**p, **{k + "_frac": round(p[k] / max(1, p["wave"]), 3)
                                         for k in ("pass", "lane_private", "dealt", "step_prep", "scan")}}
print(json.dumps(out), flush=True)
