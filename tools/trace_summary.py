"""Summarize a rocprofv3 kernel trace of a bench.py run: per (kernel, grid size) the launch count
and duration statistics, plus the GPU busy time (union of all kernel intervals) of the
multi-frame launches, so a reader can check bench.py's ms_per_step against the trace.

Usage: python tools/trace_summary.py <dir with *kernel_trace.csv or rocprofv3's *_results.db>
           [frames_per_launch] [stats.csv] > summary.json
(rocprofv3 of ROCm 7 writes an SQLite database by default; its `kernels` view holds the same
dispatch rows as the CSV, and `top_kernels` the --stats table, written to stats.csv if given.)
The bench's timed launches are the render_kernel dispatches whose grid is frames_per_launch x the
single-frame grid; their busy union / (launches x frames_per_launch) is the trace's ms per frame
(it includes the warmup launches of the same shape, which run the same orbit frames)."""
import collections
import csv
import glob
import json
import sqlite3
import sys


def short(name):
    return name.split("(")[0].replace("void ", "")


def union_ms(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        tot += ce - cs
    return tot / 1e6


def main():
    root = sys.argv[1]
    fpl = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows = []
    for f in sorted(glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)):
        rows += list(csv.DictReader(open(f)))
    for f in sorted(glob.glob(f"{root}/**/*_results.db", recursive=True)):
        db = sqlite3.connect(f)
        for r in db.execute("select name, start, end, grid_x, grid_y, grid_z, workgroup_x, workgroup_y, "
                            "workgroup_z, scratch_size from kernels"):
            rows.append(dict(zip(("Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Grid_Size_Y",
                                  "Grid_Size_Z", "Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z",
                                  "Scratch_Size"), r)))
        if len(sys.argv) > 3:
            cur = db.execute("select * from top_kernels")
            with open(sys.argv[3], "w", newline="") as fh:
                w = csv.writer(fh)
                w.writerow([d[0] for d in cur.description])
                w.writerows(cur)
    groups = collections.defaultdict(list)
    for r in rows:
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        wg = int(r["Workgroup_Size_X"]) * int(r["Workgroup_Size_Y"]) * int(r["Workgroup_Size_Z"])
        groups[(short(r["Kernel_Name"]), grid // max(wg, 1))].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Scratch_Size"])))
    out = {"launch_groups": []}
    for (k, wgs), v in sorted(groups.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
        d = [(e - s) / 1e6 for s, e, _ in v]
        out["launch_groups"].append({"kernel": k, "workgroups": wgs, "count": len(v),
                                     "mean_ms": round(sum(d) / len(d), 4), "min_ms": round(min(d), 4),
                                     "max_ms": round(max(d), 4), "total_ms": round(sum(d), 3),
                                     "scratch_bytes": v[0][2]})
    rk = [g for g in out["launch_groups"] if g["kernel"].startswith("atr::render_kernel")]
    if rk:
        single = min(rk, key=lambda g: g["workgroups"])["workgroups"]
        multi = [(k, w) for (k, w) in groups if k.startswith("atr::render_kernel") and w == fpl * single]
        if multi:
            iv = [(s, e) for key in multi for s, e, _ in groups[key]]
            n = len(iv)
            busy = union_ms(iv)
            out["multi_frame"] = {"frames_per_launch": fpl, "launches": n, "busy_union_ms": round(busy, 3),
                                  "ms_per_frame_busy": round(busy / (n * fpl), 4),
                                  "mean_launch_ms": round(sum((e - s) for s, e in iv) / n / 1e6, 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
