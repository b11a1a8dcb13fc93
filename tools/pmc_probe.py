"""Driver for rocprofv3 --pmc passes (tools/gpu_pmc2.sh): three one-frame renders (c3 geometry;
PMC_SPP / PMC_BOUNCES select e.g. the c4 shape) with the given variant, then three atr_unpack launches over the full frame (4-B stores per lane, exactly
W*H*4 bytes written and read: the calibration kernel for WRITE_SIZE / FETCH_SIZE)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402

variant = int(os.environ.get("PMC_VARIANT", str(E.ATR_KERNEL_AUTO)))
W, H = 1920, 1080
mesh = E.Mesh.load_obj(asset_path("Dragon"))
box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
tree = E.Octree.build(mesh, 300)
eng = E.Engine(0)
eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)], [(mesh, tree, box, 1)])
cam = E.camera(W, H, int(os.environ.get("PMC_SPP", "1")), int(os.environ.get("PMC_BOUNCES", "1")))
tiles = [[0, 0, W - 1, H - 1]]
fb = torch.zeros(W * H, dtype=torch.int32, device="cuda")
casts = torch.zeros(W * H, dtype=torch.int32, device="cuda")
tr = torch.zeros(1, dtype=torch.int64, device="cuda")
fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, fb.data_ptr(), None, None, None, casts.data_ptr(), tr.data_ptr())
s = torch.cuda.current_stream().cuda_stream
for _ in range(3):
    eng.render_start(cam, tiles, fr, 0x853C49E6748FEA9B, stream=s, variant=variant)
    torch.cuda.synchronize()
img = torch.zeros(W * H, dtype=torch.int32, device="cuda")
for _ in range(3):
    eng.unpack(tiles, W, fb.data_ptr(), img.data_ptr(), stream=s)
    torch.cuda.synchronize()
print("pmc probe done", int(tr.item()))
