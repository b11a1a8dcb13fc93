"""Copy the judged summaries of a gpu_r3_check*.sh run (gpurun_out/r3c, gpurun_out/bench_pmc,
gpurun_out/r3sim) into profiles/r03/. Usage: python tools/collect_r03.py [c3|c4|c5 ...] (sim8 configs)."""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G, P = os.path.join(R, "gpurun_out"), os.path.join(R, "profiles", "r03")


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


shutil.copy(f"{G}/r3c/bench_driver.json", f"{P}/bench_c3_driver.json")
shutil.copy(f"{G}/r3c/bench_traced.json", f"{P}/bench_c3_traced.json")
shutil.copy(f"{G}/r3c/trace_driver/t_kernel_stats.csv", f"{P}/c3_driver_kernel_stats.csv")
with open(f"{P}/trace_c3_driver_summary.json", "w") as f:
    subprocess.run([sys.executable, f"{R}/tools/trace_summary.py", f"{G}/r3c/trace_driver"], stdout=f, check=True)
lines = open(f"{G}/r3c/pytest_gpu.log").read().strip().splitlines()
open(f"{P}/pytest_gpu_tail.txt", "w").write("\n".join(lines[-2:]) + "\n")
for src, dst in (("bench_c4_full.json", "bench_c4.json"), ("bench_c5_full.json", "bench_c5.json")):
    if os.path.exists(f"{G}/r3c/{src}"):
        shutil.copy(f"{G}/r3c/{src}", f"{P}/{dst}")
pmc = {}
for p in sorted(glob.glob(f"{G}/bench_pmc/pass*")):
    for r in csv.DictReader(open(p + "/pmc_counter_collection.csv")):
        if "render_kernel" not in r["Kernel_Name"]:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        pmc.setdefault(k, {}).setdefault(r["Counter_Name"], []).append([int(r["Grid_Size"]), float(r["Counter_Value"])])
json.dump(pmc, open(f"{P}/pmc_c3_driver_shape.json", "w"), indent=1)
sim = json.load(open(f"{P}/sim8_shards.json")) if os.path.exists(f"{P}/sim8_shards.json") else {}
for cfg in sys.argv[1:]:
    full = last_json(f"{G}/r3sim/{cfg}_full.json")
    ranks = []
    for r in range(8):
        d = last_json(f"{G}/r3sim/{cfg}_sim8_r{r}.json")
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
json.dump(sim, open(f"{P}/sim8_shards.json", "w"), indent=1)
