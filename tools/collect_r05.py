"""Collect round-5 shard sets into profiles/r05/sim_shards.json: for each config the full-frame
line and every rank of the N-way plans (bench.py --sim-world N --sim-rank r) found in a gpurun_out
directory (files <cfg>_full.json, <cfg>_sim<N>_r<r>.json, as tools/gpu_r5_a.sh / gpu_r5_sim.sh
write them). Usage: python tools/collect_r05.py gpurun_out/r5a [more dirs ...]; then
tools/project_n.py turns the file into the 1/2/4/8 projection."""
import glob
import json
import os
import re
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(R, "profiles", "r05")
os.makedirs(P, exist_ok=True)


def last_json(path):
    lines = [ln for ln in open(path).read().strip().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


out_path = os.path.join(P, "sim_shards.json")
sim = json.load(open(out_path)) if os.path.exists(out_path) else {}
for d in sys.argv[1:]:
    for full_path in sorted(glob.glob(os.path.join(d, "*_full.json"))):
        cfg = os.path.basename(full_path).split("_")[0]
        full = last_json(full_path)
        worlds = sorted({int(m.group(1)) for f in glob.glob(os.path.join(d, f"{cfg}_sim*_r*.json"))
                         for m in [re.search(r"_sim(\d+)_r\d+\.json$", f)] if m})
        for N in worlds:
            ranks = []
            for r in range(N):
                f = os.path.join(d, f"{cfg}_sim{N}_r{r}.json")
                if not os.path.exists(f):
                    break
                x = last_json(f)
                ranks.append({"rank": r, "ms_per_frame": x["ms_per_step"], "mrays_s": x["value"],
                              "single_frame_latency_ms": x["single_frame"].get("latency_ms"),
                              "launches": x["config"].get("launches"),
                              "launch_render_done_ms": x["config"].get("launch_render_done_ms")})
            if len(ranks) != N:
                continue
            mx = max(x["ms_per_frame"] for x in ranks)
            sim.setdefault(cfg, {})[str(N)] = {
                "source": os.path.relpath(d, R), "workload": full["config"]["workload"],
                "shape": {"launches": ranks[0]["launches"] or full["config"]["launches"],
                          "streams": full["config"]["streams"]},
                "full_frame": {"ms_per_frame": full["ms_per_step"], "mrays_s": full["value"],
                               "single_frame_latency_ms": full["single_frame"].get("latency_ms")},
                "ranks": ranks, "max_shard_ms_per_frame": mx,
                "render_side_speedup": round(full["ms_per_step"] / mx, 3)}
            print(cfg, N, sim[cfg][str(N)]["render_side_speedup"], mx, full["ms_per_step"])
json.dump(sim, open(out_path, "w"), indent=1)
