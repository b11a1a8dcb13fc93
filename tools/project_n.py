"""N-GPU projection (N = 2, 4, 8) from per-rank shard timings measured on one MI355X
(bench.py --sim-world N --sim-rank r: each rank's shard of the N-way cost plan, alone, in the same
timed shape as the full-frame line; collected by tools/collect_r05.py into sim_shards.json).

  render side  = full-frame ms per frame / the slowest shard's ms per frame;
  exchange     = rank 0 receives the other ranks' pixels at 3 B each, (1 - 1/N) x W x H x 3 B per
                 frame, at an assumed xGMI rate into rank 0 (the 8-GPU node's rate is the driver's
                 to measure), plus rank 0's scatter into BGRX images (3 B read + 4 B written per
                 pixel at 5 TB/s);
  exposed      = every frame's exchange after the render;
  overlapped   = only the last launch's frames exchange after the render (the earlier launches'
                 exchanges overlap the later launches' rendering).
These are projections, not measurements. Usage:
  PROFILE=profiles/r05 python tools/project_n.py [xgmi GB/s ...] > profiles/r05/projection.json"""
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.environ.get("PROFILE", "profiles/r05")
sim = json.load(open(os.path.join(R, P, "sim_shards.json")))
rates = [float(x) for x in sys.argv[1:]] or [200.0, 350.0, 500.0]
PIX = {"c3": 1920 * 1080, "c4": 1920 * 1080, "c5": 3840 * 2160}
out = {"note": "projections from one-GPU shard timings, not multi-GPU measurements",
       "assumptions": {"xgmi_gbs_into_rank0": rates, "scatter_tbs": 5.0, "bytes_per_pixel": 3}, "configs": {}}
for cfg, per_world in sim.items():
    n = PIX[cfg]
    rows = {}
    for world, d in sorted(per_world.items(), key=lambda kv: int(kv[0])):
        N = int(world)
        full = d["full_frame"]["ms_per_frame"]
        mx = d["max_shard_ms_per_frame"]
        recv = (1 - 1.0 / N) * n * 3
        scatter_ms = (n * 7) / 5e12 * 1e3
        launches = d["shape"]["launches"]
        last_frac = d["shape"].get("exposed_frames", launches[-1]) / sum(launches)
        row = {"full_ms_per_frame": full, "max_shard_ms_per_frame": mx, "mean_shard_ms_per_frame":
               round(sum(r["ms_per_frame"] for r in d["ranks"]) / len(d["ranks"]), 5),
               "render_side_speedup": round(full / mx, 2), "per_gpu_efficiency": round(full / mx / N, 3),
               "recv_bytes_per_frame": round(recv), "scatter_ms_per_frame": round(scatter_ms, 5),
               "exposed_frame_fraction": round(last_frac, 3), "by_rate": {}}
        for g in rates:
            x = recv / (g * 1e9) * 1e3
            exposed = mx + x + scatter_ms
            overlapped = mx + (x + scatter_ms) * last_frac
            row["by_rate"][str(g)] = {"exchange_ms_per_frame": round(x, 5),
                                      "speedup_exchange_exposed": round(full / exposed, 2),
                                      "speedup_exchange_overlapped": round(full / overlapped, 2)}
        rows[str(N)] = row
    out["configs"][cfg] = rows
print(json.dumps(out, indent=1))
