"""f3 timing: octree build on the host (atr_octree_build) vs on the GPU (atr_octree_build_device)
for the asset meshes; prints one JSON line per (asset, leaf size). Both trees are compared bit for
bit before a time is reported. Usage (GPU box): python tools/build_timing.py [reps]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from atray_amd import engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    for asset, leaf in [("Monkey", 300), ("Deer", 300), ("Dragon", 300), ("Dragon", 64)]:
        m = E.Mesh.load_obj(asset_path(asset))
        m.translate_to(m.aabb(), CENTERS[asset])
        E.Octree.build_device(m, leaf)  # warm-up: module load, allocator
        host, wall, dev = [], [], []
        for _ in range(reps):
            t0 = time.perf_counter()
            h = E.Octree.build(m, leaf)
            host.append((time.perf_counter() - t0) * 1e3)
            tm = {}
            g = E.Octree.build_device(m, leaf, timings=tm)
            wall.append(tm["wall_ms"])
            dev.append(tm["device_ms"])
        for x, y in zip(h.export(), g.export()):
            assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), asset
        st = g.stats()
        print(json.dumps({"asset": asset, "leaf": leaf, "faces": m.info()[2] if hasattr(m, "info") else None,
                          "nodes": st["nodes"], "leaf_prim_refs": st["leaf_prim_refs"],
                          "host_ms": round(float(np.median(host)), 3),
                          "device_wall_ms": round(float(np.median(wall)), 3),
                          "device_kernels_ms": round(float(np.median(dev)), 3), "bit_identical": True}),
              flush=True)


if __name__ == "__main__":
    main()
