"""Aggregate rocprofv3 --pmc CSVs (one dir per counter group) per kernel name.

usage: python tools/pmc_summary.py DIR [DIR...]   (each DIR holds */p_counter_collection.csv)
Prints, per kernel: dispatches, mean duration and the summed counters, plus derived ratios
(VALU / LDS / VMEM active fractions of wave-cycles, wait fraction, VALU lane utilisation).
"""
import collections
import csv
import glob
import os
import sys


def load(dirs):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(dict)
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"].split("(")[0][:60]
                acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
                dur[k][(f, r["Dispatch_Id"])] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return acc, dur


def main():
    acc, dur = load(sys.argv[1:])
    for k, c in sorted(acc.items(), key=lambda kv: -sum(dur[kv[0]].values())):
        if k.startswith("__amd"):
            continue
        print(f"== {k}  dispatch-groups={len(dur[k])}  mean_us={sum(dur[k].values()) / max(1, len(dur[k])) / 1e3:.1f}")
        wc = c.get("SQ_WAVE_CYCLES", 0)
        for name in sorted(c):
            print(f"   {name:28s} {c[name]:16.0f}")
        if wc:
            for name in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                         "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
                if name in c:
                    print(f"   {name + '/WAVE_CYCLES':40s} {c[name] / wc:.3f}")
        if c.get("SQ_INSTS_VALU") and c.get("SQ_THREAD_CYCLES_VALU") and c.get("SQ_ACTIVE_INST_VALU"):
            print(f"   VALU lanes active ~ {c['SQ_THREAD_CYCLES_VALU'] / c['SQ_ACTIVE_INST_VALU']:.1f} / 64")


if __name__ == "__main__":
    main()
