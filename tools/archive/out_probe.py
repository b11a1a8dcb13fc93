import json, os, sys
import numpy as np, torch
sys.path.insert(0, "/root/repo") if os.path.exists("/root/repo") else None
import atray_amd.engine as E
from atray_amd.assets import CENTERS, asset_path
W, H = 1920, 1080
mesh = E.Mesh.load_obj(asset_path("Dragon")); box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
tree = E.Octree.build(mesh, 300)
eng = E.Engine(0)
eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)], [(mesh, tree, box, 1)])
cam = E.camera(W, H); tiles = [[0, 0, W - 1, H - 1]]
fb = torch.zeros(2 * W * H, dtype=torch.int32, device="cuda"); tr = torch.zeros(1, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
for name, fr in [("fb", E.atr_frame(0, fb.data_ptr(), None, None, None, None, None)),
                 ("fb+traced", E.atr_frame(0, fb.data_ptr(), None, None, None, None, tr.data_ptr())),
                 ("fb+casts+traced", E.atr_frame(0, fb.data_ptr(), None, None, None, fb.data_ptr() + 4 * W * H, tr.data_ptr()))]:
    ms = []
    for sync in (True, False):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
        for a, b in ev:
            a.record(s); eng.render_start(cam, tiles, fr, 1, stream=s.cuda_stream); b.record(s)
            if sync: torch.cuda.synchronize()
        torch.cuda.synchronize()
        ms.append(round(float(np.median([a.elapsed_time(b) for a, b in ev[2:]])), 4))
    print(json.dumps({"outputs": name, "ms_sync_async": ms, "chunk": os.environ.get("ATR_XCD_CHUNK", "16")}), flush=True)
