"""GPU diagnostic: how many cell waves are resident at once (wave trace start/end stamps) and the
single-frame kernel time, for the CLUSTER cell kernel at 4/5/6 waves per SIMD (sched 32 + n),
unplanned order. Prints one JSON line per variant."""
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
mesh = E.Mesh.load_obj(asset_path("Dragon"))
box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
tree = E.Octree.build(mesh, 300)
eng = E.Engine(0)
eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)], [(mesh, tree, box, 1)])

cam = E.camera(W, H)
tiles = [[0, 0, W - 1, H - 1]]
fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, None, None)
s = torch.cuda.current_stream()
for v in [int(x) for x in os.environ.get("VARIANTS", "36 37 38").split()]:
    ms = []
    for _ in range(12):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        eng.render_start(cam, tiles, fr, SEED, stream=s.cuda_stream, variant=v)
        b.record(s)
        torch.cuda.synchronize()
        ms.append(a.elapsed_time(b))
    tr = eng.wave_trace(cam, tiles, SEED, v).astype(np.int64)
    st, en = tr[:, 0], tr[:, 1]
    t0 = st.min()
    ev = np.concatenate([np.stack([st - t0, np.ones_like(st)], 1), np.stack([en - t0, -np.ones_like(en)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    conc = np.cumsum(ev[:, 1])
    dur = (en - st) / 100.0  # us
    span = (en.max() - t0) / 100.0
    # time-weighted mean concurrency
    dt = np.diff(ev[:, 0], append=ev[-1, 0])
    print(json.dumps({"variant": v, "kernel_ms_med": round(float(np.median(ms[2:])), 4),
                      "trace_span_us": round(float(span), 1), "max_resident_waves": int(conc.max()),
                      "mean_resident_waves": round(float((conc * dt).sum() / max(1, dt.sum())), 1),
                      "wave_us_pct_50_90_99_max": np.percentile(dur, [50, 90, 99, 100]).round(1).tolist(),
                      "sum_wave_ms": round(float(dur.sum()) / 1e3, 1),
                      "resident_at_half_span": int(((st - t0 <= span * 50) & (en - t0 > span * 50)).sum())}),
          flush=True)
