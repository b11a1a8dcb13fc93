"""N = 8 projection from the per-rank shard timings (profiles/r03/sim8_shards.json, bench.py
--sim-world 8 --sim-rank r on one GPU, same timed shape as the full-frame line): render side =
full-frame ms per frame / slowest shard's; the exchange adds rank 0's receive of the other ranks'
3-byte pixels, (1 - share_0) x W x H x 3 B per frame, at an assumed xGMI rate into rank 0, either
fully exposed or exposed only for the last launch of each stream (the stream-priority overlap,
DESIGN.md §5), plus rank 0's scatter into BGRX images (HBM-bound: 3 B read + 4 B written per pixel
at 5 TB/s). Usage: PROFILE=profiles/r04 python tools/project8.py [xgmi GB/s ...] > profiles/r04/projection8.json"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sim = json.load(open(os.path.join(R, os.environ.get("PROFILE", "profiles/r04"), "sim8_shards.json")))
rates = [float(x) for x in sys.argv[1:]] or [200.0, 350.0, 500.0]
PIX = {"c3": 1920 * 1080, "c4": 1920 * 1080, "c5": 3840 * 2160}
out = {"assumptions": {"xgmi_gbs_into_rank0": rates, "scatter_tbs": 5.0, "bytes_per_pixel": 3}, "configs": {}}
for cfg, d in sim.items():
    n = PIX[cfg]
    full = d["full_frame"]["ms_per_frame"]
    mx = d["max_shard_ms_per_frame"]
    share0 = 1.0 / 8  # rank 0's pixels (the cost plan gives it a little less work, not fewer bytes)
    recv = (1 - share0) * n * 3
    scatter_ms = (n * 7) / 5e12 * 1e3
    launches = d["shape"]["launches"]
    last_frac = launches[-1] / sum(launches)  # the last launch's frames: their exchange is exposed
    row = {"full_ms_per_frame": full, "max_shard_ms_per_frame": mx, "render_side_speedup": round(full / mx, 2),
           "recv_bytes_per_frame": round(recv), "scatter_ms_per_frame": round(scatter_ms, 5), "by_rate": {}}
    for g in rates:
        x = recv / (g * 1e9) * 1e3
        exposed = mx + x + scatter_ms
        overlapped = mx + x * last_frac + scatter_ms
        row["by_rate"][str(g)] = {"exchange_ms_per_frame": round(x, 5),
                                  "speedup_exchange_exposed": round(full / exposed, 2),
                                  "speedup_exchange_overlapped": round(full / overlapped, 2)}
    out["configs"][cfg] = row
print(json.dumps(out, indent=1))
