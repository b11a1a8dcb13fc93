"""Per-ray work of the path engine by bounce depth (COUNT build; with the diagnostic build, ATRAY_LIB=
atray_amd/_lib/diag/libatray_hip.so, also the scan phases' wave clocks): c4's camera rays alone
(bounce_limit 1, spp 64), then bounce limits 2..5 -- each level's rays are the difference.
Environment SORT=b: the queue sort at b bits per axis (tuning path_sort_bits)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import atray_amd.engine as E  # noqa: E402
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from bench import MATERIALS, SEED  # noqa: E402

W, H = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1920x1080").split("x"))
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 64
m = E.Mesh.load_obj(asset_path("Dragon"))
box = m.translate_to(m.aabb(), CENTERS["Dragon"])
t = E.Octree.build(m, 300)
eng = E.Engine(0)
eng.upload(MATERIALS, [(m, t, box, 1)])
eng.set_tuning(path_sort_bits=int(os.environ.get("SORT", "0")))
tiles = [[0, 0, W - 1, H - 1]]
prev = None
rows = []
for bl in (1, 2, 3, 4, 5):
    cam = E.camera(W, H, spp, bl)
    c = eng.counters(cam, tiles, SEED, E.ATR_KERNEL_PATHS)
    raw = dict(c)
    if prev is not None:
        d = {k: c[k] - prev[k] for k in c}
    else:
        d = dict(c)
    n = max(1, d["n_rays"])
    row = {"bounce_limit": bl, "level_rays": d["n_rays"], **{f"{k}_per_ray": round(v / n, 2) for k, v in d.items() if k != "n_rays"}}
    if "atr_render_phase_clocks" in E.signatures():  # diagnostic build: cumulative over levels <= bl
        row["phase_clocks_cum"] = eng.phase_clocks(cam, tiles, SEED, E.ATR_KERNEL_PATHS)
        row["simd_cum"] = eng.simd_counters(cam, tiles, SEED, E.ATR_KERNEL_PATHS)
    rows.append(row)
    print(json.dumps(row), flush=True)
    prev = raw
eng.close()
