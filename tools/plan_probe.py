"""The GPU-built single-frame plan (tuning frame_plan) on c3 (Dragon 1920x1080, HYBRID): one-frame
launch time with the plan on and off (interleaved), and how well the planned order follows the
measured cost (atr_render_plan_info). Prints JSON lines."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402

W, H = 1920, 1080
SEED = 0x853C49E6748FEA9B
VARIANT = int(sys.argv[1]) if len(sys.argv) > 1 else E.ATR_KERNEL_AUTO
mesh = E.Mesh.load_obj(asset_path("Dragon"))
box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
tree = E.Octree.build(mesh, 300)
eng = E.Engine(0)
eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)], [(mesh, tree, box, 1)])
full = [[0, 0, W - 1, H - 1]]
s = torch.cuda.current_stream()
fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, None, None)


def orbit(k):
    a = 2 * np.pi * k / 256
    return E.camera(W, H, eye=(0.1 + 0.5 * np.sin(a), 2.0, 0.5 * (1 - np.cos(a))))


def frames_ms(k0, n):
    """n consecutive single-frame launches along the orbit; per launch: (render + plan kernels) ms
    between events around the start call, and the render alone (atr_last_kernel_ms)."""
    out, ren = [], []
    for k in range(k0, k0 + n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.render_start(orbit(k), full, fr, SEED, stream=s.cuda_stream, variant=VARIANT)
        b.record(s)
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
        ren.append(eng.last_kernel_ms())
    return out, ren


for rep in range(3):
    for fp in (1, 0):
        eng.set_tuning(frame_plan=fp)
        ms, ren = frames_ms(rep * 40, 20)
        print(json.dumps({"frame_plan": fp, "rep": rep, "ms_median": round(float(np.median(ms[2:])), 4),
                          "render_ms_median": round(float(np.median(ren[2:])), 4),
                          "ms_first3": [round(x, 4) for x in ms[:3]]}), flush=True)
eng.set_tuning(frame_plan=1)
frames_ms(200, 3)
info = eng.plan_info(full, W, H)
if info is not None:
    base, masks, cost = info
    nb = int((W + 7) // 8 * ((H + 7) // 8))
    cost = cost[:nb].astype(np.int64)
    used = (masks[:, 0] | masks[:, 1]) != 0
    rank = np.empty(nb, np.int64)
    rank[np.argsort(-cost, kind="stable")] = np.arange(nb)  # 0 = heaviest
    pos = {}
    for i, b in enumerate(base):
        if used[i] and int(b) not in pos:
            pos[int(b)] = i
    heavy = np.argsort(-cost, kind="stable")[: nb // 20]
    print(json.dumps({"planned": int(len(base)), "used": int(used.sum()), "splits": int(used.sum() - nb),
                      "top5pct_mean_pos_frac": round(float(np.mean([pos[int(h)] for h in heavy])) / len(base), 4),
                      "first_200_mean_rank_frac": round(float(np.mean([rank[int(b)] for b in base[:200]])) / nb, 4),
                      "cost_top": [int(x) for x in np.sort(cost)[::-1][:5]], "cost_median": int(np.median(cost))}),
          flush=True)
