"""One-frame renders of a config through the C-ABI (no bench machinery), for rocprofv3 kernel traces
of the path engine: python tools/path_probe.py [c4|c5|c3] [variant] [frames] [tuning k=v,...]."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from bench import CONFIGS, MATERIALS, SEED  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
variant = int(sys.argv[2]) if len(sys.argv) > 2 else E.ATR_KERNEL_AUTO
frames = int(sys.argv[3]) if len(sys.argv) > 3 else 3
asset, W, H, spp, bounces, use_tree = CONFIGS[cfg]
m = E.Mesh.load_obj(asset_path(asset))
box = m.translate_to(m.aabb(), CENTERS[asset])
t = E.Octree.build(m, 300) if use_tree else None
eng = E.Engine(0)
if len(sys.argv) > 4 and sys.argv[4]:
    eng.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in sys.argv[4].split(","))})
eng.upload(MATERIALS, [(m, t, box, 1)])
fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
tr = torch.zeros(1, dtype=torch.int64, device="cuda")
fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, None, tr.data_ptr())
cam = E.camera(W, H, spp, bounces)
for i in range(frames):
    eng.render_start(cam, [[0, 0, W - 1, H - 1]], fr, SEED, stream=torch.cuda.current_stream().cuda_stream,
                     variant=variant)
    assert eng.wait()[0] == 0
    torch.cuda.synchronize()
    print(f"frame {i}: {eng.last_kernel_ms():.3f} ms, {int(tr.item())} traced rays", flush=True)
    tr.zero_()
eng.close()
