"""One-frame latency of the primary-ray kernel (c3: Dragon 1920x1080, app camera, HYBRID): the
launch time, its per-cell wave trace (which cells end the launch, when they started), the slowest
cells rendered alone, and the launch time under cell plans that split the measured heaviest cells
over 2/4/8 waves (atr_set_cell_plan). Prints JSON lines.

python tools/latency_probe.py [variant]"""
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
VARIANT = int(sys.argv[1]) if len(sys.argv) > 1 else E.ATR_KERNEL_HYBRID
mesh = E.Mesh.load_obj(asset_path("Dragon"))
box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
tree = E.Octree.build(mesh, 300)
eng = E.Engine(0)
eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)], [(mesh, tree, box, 1)])
cam = E.camera(W, H)
full = [[0, 0, W - 1, H - 1]]
s = torch.cuda.current_stream()
fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, None, None)


def launch_ms(tiles=full, frame=fr, n=10):
    ms = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.render_start(cam, tiles, frame, SEED, stream=s.cuda_stream, variant=VARIANT)
        b.record(s)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    return float(np.median(ms[1:]))


base = launch_ms()
print(json.dumps({"one_frame_ms": round(base, 4), "variant": VARIANT}), flush=True)
tr = eng.wave_trace(cam, full, SEED, VARIANT).astype(np.int64)
t0 = tr[:, 0].min()
start = (tr[:, 0] - t0) / 100.0  # us (100 MHz clock)
end = (tr[:, 1] - t0) / 100.0
dur = end - start
order = np.argsort(-dur)
print(json.dumps({"trace_span_us": round(float(end.max()), 1),
                  "wave_us_p50_p90_p99_max": [round(float(np.percentile(dur, q)), 1) for q in (50, 90, 99, 100)],
                  "slowest": [{"block": int(i), "start_us": round(float(start[i]), 1), "dur_us": round(float(dur[i]), 1)}
                              for i in order[:8]],
                  "last_ending": [{"block": int(i), "start_us": round(float(start[i]), 1), "dur_us": round(float(dur[i]), 1)}
                                  for i in np.argsort(-end)[:8]]}), flush=True)
pm = E.packed_pixel_map(full, W, H)
for bi in order[:4]:
    px = int(pm[64 * bi])
    x0, y0 = px % W, px // W
    tile = [[x0, y0, x0 + 7, y0 + 7]]
    big = torch.zeros(64, dtype=torch.int32, device="cuda")
    frp = E.atr_frame(E.ATR_LAYOUT_PACKED, big.data_ptr(), None, None, None, None, None)
    row = {"cell": [x0, y0], "in_frame_us": round(float(dur[bi]), 1),
           "alone_us": round(launch_ms(tile, frp, 6) * 1e3, 1)}
    c = eng.counters(cam, tile, SEED, VARIANT)
    row["per_ray"] = {k: round(c[k] / 64, 1) for k in ("box_all", "n_leaf", "cluster_boxes", "screened", "n_tri", "passes")}
    row["wave"] = eng.simd_counters(cam, tile, SEED, VARIANT)
    for parts in (2, 4, 8):  # the cell alone, split over `parts` waves
        plan = np.zeros(((W + 7) // 8) * ((H + 7) // 8), np.uint8)
        plan[(y0 // 8) * ((W + 7) // 8) + x0 // 8] = parts
        eng.set_cell_plan(W, H, plan)
        row[f"alone_split{parts}_us"] = round(launch_ms(tile, frp, 6) * 1e3, 1)
        eng.set_cell_plan(W, H, None)
    print(json.dumps(row), flush=True)
cc = eng.cell_costs(cam, SEED, VARIANT).ravel()
# the previous frame of a camera orbit (bench.py's: eye moved ~0.3 px at the dragon) as the cost source
prev = E.camera(W, H, eye=(0.1 + 0.5 * np.sin(-2 * np.pi / 256), 2.0, 0.5 * (1 - np.cos(-2 * np.pi / 256))))
cc_prev = eng.cell_costs(prev, SEED, VARIANT).ravel()


def graded(costs, edges, parts=None):
    """class 7 for the top edges[0] fraction of cells by cost, 6 for the next up to edges[1], ..."""
    plan = np.zeros(costs.size, np.uint8)
    order = np.argsort(-costs, kind="stable")
    lo = 0
    for k, e in enumerate(edges):
        hi = int(round(e * costs.size))
        plan[order[lo:hi]] = E.plan_class(7 - k)
        lo = hi
    if parts:
        p, frac = parts
        plan[order[:int(round(frac * costs.size))]] |= p
    return plan


specs = {"top10": ([0.10], None), "top20": ([0.20], None), "top30": ([0.30], None),
         "grade7": ([0.02, 0.05, 0.10, 0.20, 0.30, 0.50, 0.75], None),
         "grade4": ([0.05, 0.15, 0.30, 0.50], None),
         "grade7_split2": ([0.02, 0.05, 0.10, 0.20, 0.30, 0.50, 0.75], (2, 0.01)),
         "top20_split2": ([0.20], (2, 0.01))}
for name, (edges, parts) in specs.items():
    for src, costs in (("same", cc), ("prev", cc_prev)):
        eng.set_cell_plan(W, H, graded(costs, edges, parts))
        print(json.dumps({"plan": name, "costs": src, "one_frame_ms": round(launch_ms(), 4)}), flush=True)
        eng.set_cell_plan(W, H, None)
print(json.dumps({"no_plan_ms": round(launch_ms(), 4)}), flush=True)
