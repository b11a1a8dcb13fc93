"""Summarize tools/gpu_pmc2.sh output: per kernel (render / unpack), the mean of each counter over
its launches. Usage: python tools/pmc_summary2.py gpurun_out/pmc2 > profiles/.../pmc_summary.json"""
import collections
import csv
import glob
import json
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for f in sorted(glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
out = {}
for k, d in agg.items():
    out[k] = {c: sum(v) / len(v) for c, v in sorted(d.items())}
    if dur.get(k):
        out[k]["duration_ms_mean"] = sum(dur[k]) / len(dur[k])
print(json.dumps(out, indent=1))
