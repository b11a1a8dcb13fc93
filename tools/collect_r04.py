"""Copy a round-4 measurement set (tools/gpu_r4_final.sh: gpurun_out/r4final, gpurun_out/bench_pmc,
gpurun_out/r4sim) into profiles/r04/, and check that each bench line's roofline is recomputable
from the committed PMC rows.

Every PMC file is named after what it holds: the config, the kernel and the grid (cell kernels:
the timed launches' grid) or the dispatch count (path engine: the timed frames' kernels).
verify_r04.json recomputes traffic per frame, VALU per frame and the L2 hit rate from those rows
and compares them with the bench lines (must agree within 1 %).

Usage: python tools/collect_r04.py [sim8 configs ...]"""
import collections
import glob
import json
import os
import re
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, P = os.path.join(R, "gpurun_out"), os.path.join(R, "profiles", "r04")
os.makedirs(P, exist_ok=True)


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def kernel_tag(name):
    """'void atr::render_kernel<7, false, true, 7>(...)' -> 'render_kernel_7_false_true_7'."""
    base = name.split("(")[0].replace("void ", "").replace("atr::", "")
    return re.sub(r"[^A-Za-z0-9]+", "_", base).strip("_")


verify = {}
for cfg in ("c3", "c4", "c5"):
    src = f"{G}/r4final/bench_{cfg}.json"
    if not os.path.exists(src):
        continue
    line = last_json(src)
    json.dump(line, open(f"{P}/bench_{cfg}.json", "w"), indent=1)
    rows_path = f"{G}/bench_pmc/rows_{cfg}.json"
    if not os.path.exists(rows_path):
        continue
    rows = json.load(open(rows_path))
    sel = rows["selection"]
    kernels = sorted({r[0] for r in rows["rows"]})
    if sel == "largest grid":
        grid = rows["rows"][0][1]
        name = f"pmc_{cfg}_{kernel_tag(kernels[0])}_grid{grid}.json"
    else:
        n = sum(sel["last dispatches"].values())
        name = f"pmc_{cfg}_path_kernels_{n}_timed_dispatches.json"
    json.dump(rows, open(f"{P}/{name}", "w"))
    # recompute the line's roofline from the rows
    tot = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for _, _, _, c, v in rows["rows"]:
        tot[c] += v
        cnt[c] += 1
    roof = line["roofline"]
    steps = line["steps"]
    if sel == "largest grid":
        fpl = max(roof["frames_per_launch"])
        mean = {c: tot[c] / cnt[c] for c in tot}
        traffic_frame = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0 / fpl
        valu_frame = mean.get("SQ_INSTS_VALU", 0.0) / fpl
    else:
        traffic_frame = (2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0 / steps
        valu_frame = tot.get("SQ_INSTS_VALU", 0.0) / steps
    hit = tot.get("TCC_HIT_sum", 0.0) / max(1.0, tot.get("TCC_HIT_sum", 0.0) + tot.get("TCC_MISS_sum", 0.0))
    got = {"traffic_per_frame": traffic_frame, "valu_wave_insts_per_frame": valu_frame, "l2_hit_rate": hit}
    want = {"traffic_per_frame": roof.get("traffic_per_frame"),
            "valu_wave_insts_per_frame": (roof.get("valu") or {}).get("wave_insts_per_frame"),
            "l2_hit_rate": roof.get("l2_hit_rate")}
    verify[cfg] = {"file": name, "recomputed": got, "bench_line": want,
                   "agree_1pct": all(w is None or abs(g - w) <= 0.01 * abs(w) for g, w in
                                     ((got[k], want[k]) for k in got))}
    print(cfg, name, verify[cfg]["agree_1pct"])
json.dump(verify, open(f"{P}/verify_r04.json", "w"), indent=1)

for f in ("pytest_gpu.log", "smoke.log"):
    if os.path.exists(f"{G}/r4final/{f}"):
        lines = open(f"{G}/r4final/{f}").read().strip().splitlines()
        open(f"{P}/{f.replace('.log', '_tail.txt')}", "w").write("\n".join(lines[-3:]) + "\n")
FPL = {"trace_c3_driver": 10, "trace_c4": 4}  # frames per timed launch of the traced command
for d in glob.glob(f"{G}/r4final/trace_*"):
    if os.path.isdir(d):
        tag = os.path.basename(d)
        for f in glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True):
            shutil.copy(f, f"{P}/{tag}_kernel_stats.csv")
        with open(f"{P}/{tag}_summary.json", "w") as fh:
            subprocess.run([sys.executable, f"{R}/tools/trace_summary.py", d, str(FPL.get(tag, 4)),
                            f"{P}/{tag}_kernel_stats.csv"], stdout=fh, check=True)

sim = json.load(open(f"{P}/sim8_shards.json")) if os.path.exists(f"{P}/sim8_shards.json") else {}
for cfg in sys.argv[1:]:
    full = last_json(f"{G}/r4sim/{cfg}_full.json")
    ranks = []
    for r in range(8):
        d = last_json(f"{G}/r4sim/{cfg}_sim8_r{r}.json")
        ranks.append({"rank": r, "ms_per_frame": d["ms_per_step"], "mrays_s": d["value"],
                      "single_frame_latency_ms": d["single_frame"].get("latency_ms"),
                      "launch_render_done_ms": d["config"]["launch_render_done_ms"]})
    mx = max(x["ms_per_frame"] for x in ranks)
    sim[cfg] = {"workload": full["config"]["workload"], "shape": {"launches": full["config"]["launches"],
                                                                   "streams": full["config"]["streams"]},
                "full_frame": {"ms_per_frame": full["ms_per_step"], "mrays_s": full["value"],
                               "single_frame_latency_ms": full["single_frame"].get("latency_ms")},
                "shard_pixels": full["config"].get("shard_pixels"), "ranks": ranks,
                "max_shard_ms_per_frame": mx, "render_side_speedup": round(full["ms_per_step"] / mx, 3)}
    print(cfg, sim[cfg]["render_side_speedup"], mx, full["ms_per_step"])
if sim:
    json.dump(sim, open(f"{P}/sim8_shards.json", "w"), indent=1)
