"""Rank 0's frame assembly at N GPUs, timed on one MI355X: every rank's shard of the bench's N-way
c3 cost plan is rendered and encoded here (the masked stream, as that rank would send it), then
rank 0's per-launch assembly -- decode every other rank's stream into the images and copy its own
frames in -- is timed with HIP events on an otherwise idle GPU (median of repeats). Compares the
per-rank decode calls (atr_unpack_masked, one per rank, and an index copy of rank 0's own frames)
with the batched call (atr_unpack_masked_ranks: every rank's stream and rank 0's own frames); checks that both assemble
the same images as a one-launch full-frame render. Prints one JSON line per world size.

python tools/assembly_probe.py [worlds, e.g. 2,4,8] [frames]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import atray_amd.engine as E  # noqa: E402
from atray_amd import shard as S  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from bench import APP_FACING, MATERIALS, SEED, orbit_eye  # noqa: E402

worlds = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8").split(",")]
F = int(sys.argv[2]) if len(sys.argv) > 2 else 10
W, H, side = 1920, 1080, 32
mesh = E.Mesh.load_obj(asset_path("Dragon"))
box = mesh.translate_to(mesh.aabb(), CENTERS["Dragon"])
eng = E.Engine(0)
eng.upload(MATERIALS, [(mesh, E.Octree.build(mesh, 300), box, 1)])
cams = [E.camera(W, H, 1, 1, eye=orbit_eye(k), facing=APP_FACING) for k in range(5, 5 + F)]
costs = sum(S.tile_costs(eng, E.camera(W, H, 1, 1, eye=orbit_eye(k), facing=APP_FACING), W, H, side, SEED)
            for k in (2, 3, 4))
npx = W * H
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream()
want = torch.zeros(F * npx, dtype=torch.int32, device=dev)
eng.render_start_cameras(cams, [[0, 0, W - 1, H - 1]], E.atr_frame(E.ATR_LAYOUT_IMAGE, want.data_ptr(), None, None,
                                                                    None, None, None), npx, SEED)
torch.cuda.synchronize()
bg = S.background_value(want[:npx].cpu().numpy().view(np.uint32))


def probe(world):
    """One line: rank 0's assembly of one F-frame launch of the world-way plan."""
    plan = S.ShardPlan.balanced(costs, W, H, world, side, 0.1, True)
    tiles = [E.tiles_array([list(t) for t in plan.tiles[r]]) for r in range(world)]
    fbs, encs, sizes = [], [], []
    for r in range(world):
        own = plan.sizes[r]
        fb = torch.zeros(F * own, dtype=torch.int32, device=dev)
        eng.render_start_cameras(cams, tiles[r], E.atr_frame(E.ATR_LAYOUT_PACKED, fb.data_ptr(), None, None, None,
                                                             None, None), own, SEED)
        enc = torch.zeros(E.pack_bgr_masked_bound(F * own), dtype=torch.uint8, device=dev)
        nb = torch.zeros(1, dtype=torch.int64, device=dev)
        eng.pack_bgr_masked(fb.data_ptr(), F * own, bg, enc.data_ptr(), nb.data_ptr())
        torch.cuda.synchronize()
        fbs.append(fb)
        encs.append(enc)
        sizes.append(int(nb.item()))
    dst0 = torch.from_numpy(S.frames_assembly_index(plan, F)).to(dev)[:F * plan.sizes[0]]
    images = torch.zeros(F * npx, dtype=torch.int32, device=dev)

    def assemble_per_rank():
        for r in range(1, world):
            eng.unpack_masked(tiles[r], W, H, encs[r].data_ptr(), F, images.data_ptr(), npx, stream=s.cuda_stream)
        images.index_copy_(0, dst0, fbs[0])

    def assemble_batched():  # rank 0's own packed frames as a raw source of the same launch
        eng.unpack_masked_ranks([tiles[r] for r in range(1, world)] + [tiles[0]], W, H,
                                [encs[r].data_ptr() for r in range(1, world)] + [fbs[0].data_ptr()], F,
                                images.data_ptr(), npx, stream=s.cuda_stream, raw=[0] * (world - 1) + [1])

    def timed(fn, n=20):
        ms = []
        for _ in range(n):
            images.zero_()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn()
            b.record(s)
            torch.cuda.synchronize()
            ms.append(a.elapsed_time(b))
        return round(float(np.median(ms[2:])), 4), bool(torch.equal(images, want))

    out = {"world": world, "frames": F, "stream_bytes": sizes, "decoded_pixels": int(F * (npx - plan.sizes[0]))}
    out["per_rank_ms"], out["per_rank_exact"] = timed(assemble_per_rank)
    out["batched_ms"], out["batched_exact"] = timed(assemble_batched)
    return out


for world in worlds:
    print(json.dumps(probe(world)), flush=True)
eng.close()
