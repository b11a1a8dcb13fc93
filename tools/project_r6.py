"""N-GPU projection (N = 2, 4, 8) from per-rank shard timings measured on one MI355X, with the
round-6 exchange (the masked stream: a bit per pixel plus 3 B per non-background pixel, its size
sent first) on a per-launch timeline. Reads the bench lines that tools/gpu_r6_sim.sh writes:
<cfg>_full_<i>.json (the one-GPU line) and <cfg>_sim<N>_r<r>_<i>.json (rank r's shard of the N-way
cost plan alone: bench.py --sim-world N --sim-rank r, which renders, counts and encodes exactly as
that rank does in the N-GPU run, and reports its stream bytes per frame).

Per repetition i and world N:
  ready_j   launch j's streams are ready on every sender: the max over ranks of the launch's encoding
            done (launch_encoded_ms; older lines: the render's completion, the last launch at the
            rank's whole timed span)
  x_j       rank 0 receives sum_r (stream bytes per frame of rank r) x frames_j at an assumed rate
            into rank 0 (200 / 350 / 500 GB/s: the 8-GPU node's rate is the driver's to measure),
            then decodes frames_j x W x H pixels (atr_unpack_masked: ~5.3 B of traffic per pixel at
            5 TB/s)
  end_j     max(ready_j, end_{j-1}) + x_j  (one exchange at a time into rank 0)
  T         max(end_last, every rank's whole span: render, encoding and per-tile counters)
  speedup   full-frame ms per frame x frames / T; render side = full / slowest rank alone
These are projections from one-GPU timings, not multi-GPU measurements.
With --assembly FILE (tools/assembly_probe.py's lines), rank 0's decode of a launch is the measured
batched assembly (atr_unpack_masked_ranks + its own frames' copy) per frame of that world size,
scaled by the frame's pixels against the probe's 1920x1080, instead of the byte model.
usage: python tools/project_r6.py DIR [--assembly FILE] [cfg ...] > profiles/r06/projection.json"""
import glob
import json
import os
import re
import sys
from collections import defaultdict

RATES = [200.0, 350.0, 500.0]
DECODE_BPP = 5.3  # atr_unpack_masked: 4 B written, 0.5 B of block records, ~0.8 B of stream and group offsets
HBM_TBS = 5.0


def line(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def main():
    args = sys.argv[1:]
    asm = {}  # world -> measured assembly ms per 1920x1080 frame
    if "--assembly" in args:
        k = args.index("--assembly")
        for ln in open(args[k + 1]):
            if ln.startswith("{"):
                a = json.loads(ln)
                asm[int(a["world"])] = a["batched_ms"] / a["frames"]
        del args[k:k + 2]
    d = args[0]
    cfgs = args[1:] or ["c3", "c4", "c5"]
    out = {"note": "projections from one-GPU shard timings with the masked exchange, not multi-GPU measurements",
           "assumptions": {"xgmi_gbs_into_rank0": RATES,
                           "decode": ({"measured_assembly_ms_per_1080p_frame": {str(w): round(v, 5) for w, v in asm.items()}}
                                      if asm else {"decode_bytes_per_pixel": DECODE_BPP, "decode_tbs": HBM_TBS})},
           "configs": {}}
    for cfg in cfgs:
        fulls = {}
        for p in glob.glob(os.path.join(d, f"{cfg}_full_*.json")):
            fulls[re.search(r"_(\d+)\.json$", p).group(1)] = line(p)
        sims = defaultdict(lambda: defaultdict(dict))  # world -> rep -> rank -> line
        for p in glob.glob(os.path.join(d, f"{cfg}_sim*_r*_*.json")):
            m = re.search(rf"{cfg}_sim(\d+)_r(\d+)_(\d+)\.json$", p)
            sims[int(m.group(1))][m.group(3)][int(m.group(2))] = line(p)
        if not fulls:
            continue
        rows = {}
        for N in sorted(sims):
            reps = []
            for rep, ranks in sorted(sims[N].items()):
                if len(ranks) != N or rep not in fulls:
                    continue
                full = fulls[rep]
                K = full["steps"]
                W, H = (int(x) for x in re.search(r"(\d+)x(\d+)", full["config"]["workload"]).groups())
                full_ms = full["ms_per_step"]
                span = {r: ln["ms_per_step"] * ln["steps"] for r, ln in ranks.items()}
                launches = ranks[0]["config"]["launches"]
                done = {r: ln["config"]["launch_render_done_ms"] for r, ln in ranks.items()}
                # a launch's streams are ready once encoded (lines that record it); the per-tile
                # counters that follow only feed the small reduction, so the job ends no earlier
                # than every rank's whole span either
                enc = {r: ln["config"].get("launch_encoded_ms") for r, ln in ranks.items()}
                bpf = {r: (ln.get("sim") or {}).get("stream_bytes_per_frame") or 0 for r, ln in ranks.items()}
                rep_row = {"full_ms_per_frame": full_ms,
                           "max_shard_ms_per_frame": round(max(span.values()) / K, 5),
                           "mean_shard_ms_per_frame": round(sum(span.values()) / N / K, 5),
                           "render_side_speedup": round(full_ms * K / max(span.values()), 3),
                           "recv_bytes_per_frame": int(sum(bpf[r] for r in range(1, N))),
                           "by_rate": {}}
                for g in RATES:
                    end = 0.0
                    for j, nf in enumerate(launches):
                        last = j == len(launches) - 1
                        ready = max(enc[r][j] if enc[r] else (span[r] if last else done[r][j]) for r in range(1, N))
                        dec = nf * asm[N] * W * H / (1920 * 1080) if N in asm else \
                            nf * W * H * DECODE_BPP / (HBM_TBS * 1e12) * 1e3
                        x = sum(bpf[r] for r in range(1, N)) * nf / (g * 1e9) * 1e3 + dec
                        end = max(ready, end) + x
                    T = max(end, max(span.values()))
                    rep_row["by_rate"][str(g)] = {"job_ms": round(T, 4), "speedup": round(full_ms * K / T, 3)}
                reps.append(rep_row)
            if not reps:
                continue
            rows[str(N)] = {"reps": reps,
                            "render_side_speedup": [r["render_side_speedup"] for r in reps],
                            "speedup_at_350": [r["by_rate"]["350.0"]["speedup"] for r in reps]}
        out["configs"][cfg] = rows
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
