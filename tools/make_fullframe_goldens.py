"""Whole-frame oracle digests for the full-size configs.

The oracle (oracle/atr_oracle.c, the reference algorithm restated) renders, on every host thread
of this container:

  c4        Dragon 1920x1080, 64 spp, 5 bounces, app camera (app.cpp:81-88), SEED
  c5        Dragon 3840x2160, 256 spp, 5 bounces, app camera, SEED
  c3_orbitK Dragon 1920x1080, 1 spp, 1 bounce, bench.orbit_eye(K) for K = 5..24 -- the 20 frames
            the driver's `bench.py --steps 20 --warmup 5` times

and records per frame the digests of the framebuffer (BGRX u32), per-pixel ray_casts
(renderer.cpp:260), primary hit face and t bits (kd_tree.cpp:337-465) and the pre-clamp RGB bits
(renderer.cpp:358), plus hit / traced-ray / ray_casts totals and one CRC per row (to localise a
mismatch). tests/test_gpu_fullframe.py renders the same frames on the GPU and compares digests:
every pixel of these frames is then checked against the oracle, not only the row bands of
tests/test_gpu_configs.py. Digests cost bytes; the frames themselves (25-100 MB each) stay out
of the repository.

usage: python tools/make_fullframe_goldens.py [c4] [c5] [c3]   (default: all; c5 ~25 min on 8 cores)
"""
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import ctypes as C
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (orbit_eye, APP_* -- the bench's own camera path)
from atray_amd.assets import CENTERS, asset_path  # noqa: E402
from oracle import oracle as O  # noqa: E402
from tests.goldens import SEED, frame_digest, row_crcs  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "fullframe.json")
THREADS = os.cpu_count() or 8


def render_frame(scene, cam, seed, band=4):
    """Whole frame on THREADS host threads, `band` rows per work item (ctypes releases the GIL)."""
    W, H = cam.width, cam.height
    n = W * H
    rgb = np.empty((n, 3), np.float32)
    fb = np.empty(n, np.uint32)
    casts = np.empty(n, np.uint32)
    face = np.empty(n, np.uint32)
    t = np.empty(n, np.float32)
    L = O.lib()

    def work(y0):
        y1 = min(H, y0 + band)
        k = y0 * W
        c1, c2 = O.om_counters(), O.om_counters()
        L.om_render_rows(C.byref(scene.s), C.byref(cam.c), C.c_uint64(seed), y0, y1,
                         rgb[k:].ctypes.data_as(C.c_void_p), fb[k:].ctypes.data_as(C.c_void_p),
                         casts[k:].ctypes.data_as(C.c_void_p), C.byref(c1))
        L.om_primary_hits(C.byref(scene.s), C.byref(cam.c), y0, y1, face[k:].ctypes.data_as(C.c_void_p),
                          t[k:].ctypes.data_as(C.c_void_p), C.byref(c2))
        return c1.as_dict()

    with ThreadPoolExecutor(max_workers=THREADS) as ex:
        ctrs = list(ex.map(work, range(0, H, band)))
    tot = {k: sum(c[k] for c in ctrs) for k in ctrs[0]}
    return {"fb": fb.reshape(H, W), "casts": casts.reshape(H, W), "face": face.reshape(H, W),
            "t": t.reshape(H, W), "rgb": rgb.reshape(H, W, 3)}, tot


def record(frames, W, H, spp, bounces, eye):
    return {"W": W, "H": H, "spp": spp, "bounces": bounces, "eye": list(eye),
            "facing": list(bench.APP_FACING), "seed": SEED,
            "fb": frame_digest(frames["fb"]), "casts": frame_digest(frames["casts"]),
            "face": frame_digest(frames["face"]), "t": frame_digest(frames["t"]),
            "rgb": frame_digest(frames["rgb"]),
            "hits": int((frames["face"] != 0xFFFFFFFF).sum()),
            "casts_sum": int(frames["casts"].astype(np.uint64).sum()),
            "rows": row_crcs(frames)}


def main(which):
    gold = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            gold = json.load(f)
    gold["seed"] = SEED
    gold["generator"] = "tools/make_fullframe_goldens.py (oracle/atr_oracle.c, host threads)"
    scene = O.Scene(asset_path("Dragon"), center=CENTERS["Dragon"])

    def save():
        with open(OUT, "w") as f:
            json.dump(gold, f, indent=1, sort_keys=True)

    jobs = []
    if "c4" in which:
        jobs.append(("c4", 1920, 1080, 64, 5, bench.APP_EYE))
    if "c3" in which:
        jobs += [(f"c3_orbit{k}", 1920, 1080, 1, 1, bench.orbit_eye(k)) for k in range(5, 25)]
    if "c5" in which:
        jobs.append(("c5", 3840, 2160, 256, 5, bench.APP_EYE))
    for name, W, H, spp, b, eye in jobs:
        t0 = time.time()
        cam = O.Camera(W, H, spp=spp, bounces=b, eye=eye, facing=bench.APP_FACING)
        frames, ctr = render_frame(scene, cam, SEED, band=4 if W * spp < 100000 else 1)
        rec = record(frames, W, H, spp, b, eye)
        rec["traced"] = int(ctr["n_rays"])
        rec["ray_casts_ref"] = int(ctr["n_raycasts_ref"])
        rec["oracle_seconds"] = round(time.time() - t0, 1)
        gold[name] = rec
        save()
        print(name, rec["fb"], rec["hits"], rec["traced"], f"{rec['oracle_seconds']} s", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:] or ["c4", "c3", "c5"])
