"""GPU diagnostic: latency of the heaviest 8x8 cells rendered alone (one wave on an idle GPU),
and with n copies in flight (frames of one launch), CLUSTER variant. Prints JSON lines."""
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
VARIANT = int(os.environ.get("VARIANT", str(E.ATR_KERNEL_CLUSTER)))
mesh = E.Mesh.load_obj(asset_path("Dragon"))
box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
tree = E.Octree.build(mesh, 300)
eng = E.Engine(0)
eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)], [(mesh, tree, box, 1)])
cam = E.camera(W, H)
full = [[0, 0, W - 1, H - 1]]
tr = eng.wave_trace(cam, full, SEED, E.ATR_KERNEL_CLUSTER).astype(np.int64)
dur = (tr[:, 1] - tr[:, 0]) / 100.0
# block order of the full-frame tile (Z order within the tile): recover each block's origin by
# rendering with the packed map
pm = E.packed_pixel_map(full, W, H)  # pixel of every packed slot, block by block (64 per full block)
order = np.argsort(-dur)[:8]
s = torch.cuda.current_stream()
for bi in order[:4]:
    px = int(pm[64 * bi])  # full-frame blocks own all 64 pixels: slot 64*bi is the cell's first pixel
    x0, y0 = px % W, px // W
    tile = [[x0, y0, x0 + 7, y0 + 7]]
    res = {"block": int(bi), "x0": x0, "y0": y0, "wave_us_in_frame": round(float(dur[bi]), 1)}
    assert E.packed_size(tile) == 64
    for n in (1, 8, 64):
        # PACKED layout: the 64 pixels of the cell, n frames 64 apart (an IMAGE layout would
        # address the whole W x H frame)
        big = torch.zeros(n * 64, dtype=torch.int32, device="cuda")
        frp = E.atr_frame(E.ATR_LAYOUT_PACKED, big.data_ptr(), None, None, None, None, None)
        ms = []
        for _ in range(5):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            eng.render_start_frames(cam, tile, frp, n, 64, SEED, stream=s.cuda_stream, variant=VARIANT)
            b.record(s)
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
        res[f"alone_x{n}_us"] = round(float(np.median(ms[1:])) * 1e3, 1)
    c = eng.counters(cam, tile, SEED, VARIANT)
    res["per_ray"] = {k: round(c[k] / 64, 1) for k in ("n_box", "box_all", "n_leaf", "cluster_boxes", "screened", "n_tri", "passes")}
    print(json.dumps(res), flush=True)
