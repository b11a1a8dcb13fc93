"""Collect the round-6 measurement set into profiles/r06/ (shard sets: tools/project_r6.py).

  python tools/collect_r06.py final gpurun_out/r6final
      the bench lines (bench_<cfg>.json), their PMC rows (gpurun_out/bench_pmc/rows_<cfg>.json, named
      after the kernel and grid / dispatch count), verify_r06.json (traffic, VALU and L2 hit rate
      recomputed from the rows, must agree with the lines within 1 %), the GPU suite and smoke
      tails, and the rocprofv3 kernel traces' stats and summaries (tools/trace_summary.py)."""
import glob
import json
import os
import re
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(R, "profiles", "r06")
os.makedirs(P, exist_ok=True)


def last_json(path):
    lines = [ln for ln in open(path).read().strip().splitlines() if ln.startswith("{")]
    return json.loads(lines[-1])


def kernel_tag(name):
    """'void atr::render_kernel<7, false, true, 7>(...)' -> 'render_kernel_7_false_true_7'."""
    base = name.split("(")[0].replace("void ", "").replace("atr::", "")
    return re.sub(r"[^A-Za-z0-9]+", "_", base).strip("_")


def collect_final(d):
    import collections
    import shutil
    import subprocess
    G = os.path.join(R, "gpurun_out")
    vpath = f"{P}/verify_r06.json"
    verify = json.load(open(vpath)) if os.path.exists(vpath) else {}  # configs not in d keep theirs
    for cfg in ("c3", "c4", "c5"):
        src = os.path.join(d, f"bench_{cfg}.json")
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
            name = f"pmc_{cfg}_{kernel_tag(kernels[0])}_grid{rows['rows'][0][1]}.json"
        else:
            name = f"pmc_{cfg}_path_kernels_{sum(sel['last dispatches'].values())}_timed_dispatches.json"
        json.dump(rows, open(f"{P}/{name}", "w"))
        tot, cnt = collections.defaultdict(float), collections.defaultdict(int)
        for _, _, _, c, v in rows["rows"]:
            tot[c] += v
            cnt[c] += 1
        roof = line["roofline"]
        if sel == "largest grid":
            fpl = max(roof["frames_per_launch"])
            mean = {c: tot[c] / cnt[c] for c in tot}
            traffic_frame = (2.0 * mean["FETCH_SIZE"] + mean["WRITE_SIZE"]) * 1024.0 / fpl
            valu_frame = mean.get("SQ_INSTS_VALU", 0.0) / fpl
        else:
            traffic_frame = (2.0 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) * 1024.0 / line["steps"]
            valu_frame = tot.get("SQ_INSTS_VALU", 0.0) / line["steps"]
        hit = tot.get("TCC_HIT_sum", 0.0) / max(1.0, tot.get("TCC_HIT_sum", 0.0) + tot.get("TCC_MISS_sum", 0.0))
        got = {"traffic_per_frame": traffic_frame, "valu_wave_insts_per_frame": valu_frame, "l2_hit_rate": hit}
        want = {"traffic_per_frame": roof.get("traffic_per_frame"),
                "valu_wave_insts_per_frame": (roof.get("valu") or {}).get("wave_insts_per_frame"),
                "l2_hit_rate": roof.get("l2_hit_rate")}
        verify[cfg] = {"file": name, "recomputed": got, "bench_line": want,
                       "agree_1pct": all(w is None or abs(g - w) <= 0.01 * abs(w) for g, w in
                                         ((got[k], want[k]) for k in got))}
        print(cfg, name, verify[cfg]["agree_1pct"])
    if verify:
        json.dump(verify, open(f"{P}/verify_r06.json", "w"), indent=1)
    for f in ("pytest_gpu.log", "smoke.log"):
        if os.path.exists(f"{d}/{f}"):
            lines = open(f"{d}/{f}").read().strip().splitlines()
            open(f"{P}/{f.replace('.log', '_tail.txt')}", "w").write("\n".join(lines[-3:]) + "\n")
    fpl = {"trace_c3_driver": 20, "trace_c4": 8}  # frames per timed launch of the traced command
    for t in glob.glob(f"{d}/trace_*"):
        if os.path.isdir(t):
            tag = os.path.basename(t)
            for f in glob.glob(f"{t}/**/*kernel_stats.csv", recursive=True):
                shutil.copy(f, f"{P}/{tag}_kernel_stats.csv")
            with open(f"{P}/{tag}_summary.json", "w") as fh:
                subprocess.run([sys.executable, f"{R}/tools/trace_summary.py", t, str(fpl.get(tag, 4)),
                                f"{P}/{tag}_kernel_stats.csv"], stdout=fh, check=True)


if __name__ == "__main__":
    if sys.argv[1] == "final":
        collect_final(sys.argv[2])
    else:
        sys.exit(__doc__)
