"""Benchmark: Mrays/s of the render path on Dragon 1920x1080 (BASELINE.json metric, config c3).

python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c4|c5|...] [--variant auto|cl|ps|lane|...]

One step = one frame rendered by all ranks. Frames follow a small camera orbit around the app's
eye (app.cpp:88): frame k's eye moves along a 0.5-unit circle, so no two frames of a run trace
the same rays. Frames are rendered F per launch (atr_render_start_cameras: one grid, one camera
per frame) on S streams; each rank traces its shard tiles into a packed buffer (framebuffer and
the reference's per-pixel ray_casts); for N > 1 the packed buffers are gathered to rank 0 over
RCCL (torch.distributed "nccl") and scattered into the frame there, and rank 0 sums
total_ray_casts (renderer.cpp:465-468). The scene (OBJ load, octree build, upload) and the shard
plan are prepared before timing; inputs are resident in HBM when the timed region starts.

value = traced rays of all ranks in the K timed frames (counted by the kernels: every
get_intersection_data-equivalent call) / max-over-ranks wall time. The K frames are split into
launches of as equal size as possible (at most F each), so the pipeline's fill and drain are
the same share of the run whatever K is.

--gpus N > 1 without WORLD_SIZE in the environment: this process starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child before touching
the GPU and exits with its code. --selftest: no GPU; a synthetic fill (pixel index) stands in
for the render kernel so the launch, shard plan, gather and frame assembly run on CPU (gloo).
ATR_DIST_BACKEND=gloo rehearses N ranks on one GPU (host-staged gather).

Extra JSON fields: single_frame (one frame per launch, app camera: kernel time from HIP events
on the launch stream and its Mrays/s), roofline (that kernel: algorithmic bytes per launch /
its average duration, against 8 TB/s; traffic = HBM bytes per launch from rocprofv3 --pmc
FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, separate passes of a child run), cpu_baseline
(the C oracle, i.e. the reference algorithm restated, on the host's cores and on one thread),
prep (OBJ load, host and device octree build, upload; untimed for Mrays/s).
"""
import argparse
import csv
import glob
import json
import math
import os
import re
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mrays/sec on Dragon.obj 1920x1080 @ 1/2/4/8 GPU; % HBM roofline"
SEED = 0x853C49E6748FEA9B
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md, chip-level parameters)
APP_EYE = (0.1, 2.0, 0.0)        # app.cpp:88
APP_FACING = (-0.1, -0.5, -1.0)
ORBIT_RADIUS = 0.5
ORBIT_PERIOD = 256
# config -> (asset, W, H, spp, bounces, use_tree)  (BASELINE.json configs)
CONFIGS = {
    "c1": ("Cube", 256, 256, 1, 1, True),
    "c2": ("Monkey", 1280, 720, 1, 1, False),
    "c3": ("Dragon", 1920, 1080, 1, 1, True),
    "c4": ("Dragon", 1920, 1080, 64, 5, True),
    "c5": ("Dragon", 3840, 2160, 256, 5, True),
}
GOLDEN_COUNTERS = {"c3": "dragon_1920x1080_tree", "c2": "monkey_1280x720_bf", "c1": "cube_256_tree"}
MATERIALS = [((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)]  # app.cpp:91-105


MAX_FRAME_CAMS = 24  # cameras per atr_render_start_cameras launch (the library's kMaxFrameCams)


def default_streams(config, steps=0, world=1):
    """Launches in flight by default: one for the path-engine configs (two concurrent launches
    share the caches the sorted bounce queues rely on); for the 1-spp configs on one
    GPU, one when a single launch holds every timed frame (its cells graded heaviest first across
    all the frames: the driver's 20 c3 frames +2.5-3.6% over 10 + 10 on two streams, round 6), else
    two (one launch's tail hides behind the other's work); with N > 1 shards two (stream 0 at high
    priority: its launch and exchange finish while the other renders; the 8-way c3 projection
    4.98-5.12x against 4.45-4.58x for one launch)."""
    spp, bounces = CONFIGS[config][3:5]
    return 1 if (spp > 1 or bounces > 1 or (world <= 1 and steps <= MAX_FRAME_CAMS)) else 2


def orbit_eye(k):
    a = 2.0 * math.pi * (k % ORBIT_PERIOD) / ORBIT_PERIOD
    return (APP_EYE[0] + ORBIT_RADIUS * math.sin(a), APP_EYE[1], APP_EYE[2] + ORBIT_RADIUS * (1.0 - math.cos(a)))


def algorithmic_bytes_per_ray(ctr):
    """B = 24 (ray) + 12 (hit out) + 28 N_box + 40 N_tri + 8 N_leaf per ray,
    N_* = the reference's own per-ray work on this input."""
    n = ctr["n_rays"]
    return (36.0 + 28.0 * ctr["n_box"] / n + 40.0 * ctr["n_tri"] / n + 8.0 * ctr["n_leaf"] / n)


def cluster_bytes_per_ray(ctr):
    """The clustered kernels' own algorithmic bytes per ray, in their own data layout (DESIGN.md
    §6): ray in + hit out (36); one 48-B inner-node record per visit, shared by the 8 child boxes
    it tests (6 per box test, re-walks included); 8 per leaf range; 32 per cluster record; the
    screen's 6 (three f16) per screened primitive; a, ab, ac (36) per full triangle test. N_*
    counted live by the instrumented build of the same kernel on the same frame."""
    n = ctr["n_rays"]
    return (36.0 + 6.0 * ctr["box_all"] / n + 8.0 * ctr["n_leaf"] / n + 32.0 * ctr["cluster_boxes"] / n
            + 6.0 * ctr["screened"] / n + 36.0 * ctr["n_tri"] / n)


def cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup CPU quota if any."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(float(q) / float(p))))
    except (OSError, ValueError):
        pass
    return max(1, n)


# PMC passes of the child run, one counter group per rocprofv3 run (gfx950 block limits: FETCH_SIZE
# takes 3 of the 4 TCC counters, WRITE_SIZE 2, so each gets its own pass).
PMC_PASSES = [["FETCH_SIZE"], ["WRITE_SIZE"],
              ["SQ_INSTS_VALU", "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"],
              ["TCC_HIT_sum", "TCC_MISS_sum"]]
VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2.0  # wave-instructions/s: 1,024 SIMD-32s, one wave64 VALU op per 2 clocks
                                          # (MI355X_MICROARCH.md "Wave scheduling"), 2.4 GHz


def pmc_counters(args, kernel_name, path_tail=None):
    """Counters of the timed launches of THIS command's shape: a child run of bench.py with the same
    --config/--steps/--warmup/--streams/--frames-per-launch/--variant/--tuning (--pmc-child: no PMC,
    no CPU baseline, and nothing rendered after the timed region), profiled by separate rocprofv3
    --pmc passes (--kernel-trace only).
      cell kernels (kernel_name "render_kernel"): the dispatches of the largest render grid (the
        timed launches; warmup and priming launches are smaller) -- per counter the mean per launch;
      path engine (path_tail = {kernel: n}): the last n dispatches of each path kernel (the timed
        region is the child's last work) -- per counter the sum over them.
    The selected rows are written to gpurun_out/bench_pmc/rows_<config>.json (kernel, grid,
    dispatch, counter, value) so the line can be recomputed from them (tools/collect_r04.py copies
    them into profiles/). Returns ({counter: value}, {"grid" | "dispatches": ...}, note)."""
    exe = "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, None, "rocprofv3 missing"
    out = {}
    info = {}
    kept = []
    base = os.path.join(ROOT, "gpurun_out", "bench_pmc")
    for i, group in enumerate(PMC_PASSES):
        d = os.path.join(base, f"{args.config}_pass{i}")
        os.makedirs(d, exist_ok=True)
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            os.remove(f)  # a previous run's rows never mix into this one
        cmd = [exe, "--pmc", *group, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(args.steps), "--warmup",
               str(args.warmup), "--frames-per-launch", str(args.frames_per_launch), "--streams", str(args.streams),
               "--config", args.config, "--variant", args.variant, "--no-cpu-baseline", "--no-pmc", "--no-prep",
               "--no-steady", "--pmc-child"] + (["--tuning", args.tuning] if args.tuning else [])
        env = dict(os.environ)
        for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
            env.pop(k, None)
        try:
            subprocess.run(cmd, check=True, timeout=300, env=env, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
        except Exception as e:  # noqa: BLE001
            return None, None, f"rocprofv3 {group} failed: {e}"
        rows = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    # product launches only (not the instrumented COUNT builds: <.., true, ..>)
                    if kernel_name in name and not re.search(r"<(\d+, )?true", name):
                        rows.append((name, int(row.get("Grid_Size") or 0), int(row.get("Dispatch_Id") or 0),
                                     row["Counter_Name"], float(row["Counter_Value"])))
        if not rows:
            return None, None, f"no rows for {group}"
        if path_tail is None:
            big = max(r[1] for r in rows)
            info["grid"] = big
            sel = [r for r in rows if r[1] == big]
            for c in group:
                vals = [r[4] for r in sel if r[3] == c]
                if vals:
                    out[c] = sum(vals) / len(vals)
        else:
            sel = []
            for kn, n in path_tail.items():
                ids = sorted({r[2] for r in rows if kn in r[0]})[-n:] if n else []
                if len(ids) < n:
                    return None, None, f"{kn}: {len(ids)} dispatches, want {n}"
                idset = set(ids)
                sel += [r for r in rows if kn in r[0] and r[2] in idset]
                info.setdefault("dispatches", {})[kn] = n
            for c in group:
                out[c] = sum(r[4] for r in sel if r[3] == c)
                for kn in path_tail:
                    info.setdefault("per_kernel", {}).setdefault(kn, {})[c] = sum(
                        r[4] for r in sel if r[3] == c and kn in r[0])
        kept += sel
    with open(os.path.join(base, f"rows_{args.config}.json"), "w") as fh:
        json.dump({"config": args.config, "steps": args.steps, "warmup": args.warmup, "tuning": args.tuning,
                   "selection": "largest grid" if path_tail is None else {"last dispatches": path_tail},
                   "columns": ["kernel", "grid", "dispatch", "counter", "value"], "rows": kept}, fh)
    return out, info, "ok"


def path_dispatches(args, tiles, W, H, spp, bounces, batch_log2, sort_bits=0):
    """Kernel dispatches of the path engine in the timed region (capi.cpp launch_paths): per
    launch of nf frames, its nf x blocks cells in batches of 2^batch_log2 / (64 spp) cells; per
    batch one camera, bounces - 1 bounce and one resolve launch, and with the queue sort
    (path_sort_bits) bounces - 1 sorts of four kernels each."""
    cells = set()
    for x0, y0, x1, y1 in tiles:
        for cy in range(max(0, y0) // 8, min(H - 1, y1) // 8 + 1):
            for cx in range(max(0, x0) // 8, min(W - 1, x1) // 8 + 1):
                cells.add((cx, cy))
    per_batch = max(1, (1 << batch_log2) // (64 * max(1, spp)))
    nb = sum(-(-nf * len(cells) // per_batch) for nf in launch_sizes(args.steps, args.frames_per_launch,
                                                                      max(1, args.streams)))
    out = {"path_camera_kernel": nb, "path_bounce_kernel": nb * max(0, bounces - 1), "path_resolve_kernel": nb}
    if sort_bits and bounces >= 2:
        for k in ("path_sort_sums", "path_sort_part_scan", "path_sort_scan", "path_sort_rank"):
            out[k] = nb * (bounces - 1)
    return out


def cpu_baseline(asset, W, H, spp, bounces, use_tree, seconds):
    """The reference algorithm (C oracle restatement) on this host, render time only: (a) on the
    host's CPU share with the reference tile scheduler (renderer.cpp:403-455) over whole frames
    when one frame fits the budget, else a strided row sample claimed row by row; (b) on one
    thread, a strided row sample. Traced rays count every get_intersection_data call (the
    threaded whole-frame run traces the reference's 1-px tile overlaps twice, as its threads do);
    ray_casts is the reference's non-sky count (renderer.cpp:260)."""
    from atray_amd.assets import CENTERS, asset_path
    from oracle import oracle as O
    s = O.Scene(asset_path(asset), center=CENTERS[asset], use_tree=use_tree)
    cam = O.Camera(W, H, spp=spp, bounces=bounces)
    share = cpu_share()

    def rows_sample(threads, budget):
        # passes over rows r0, r0 + step, ... (2 x threads rows spread over the frame), r0 = 0, 1,
        # ... until the budget is spent: every row at most once
        step = max(1, H // max(4, 2 * threads))
        secs = traced = casts = done = 0
        while (secs < budget or done == 0) and done < step:
            dt, tr, ca = s.render_rows_threaded(cam, SEED, threads, done, step, (H - 1 - done) // step + 1)
            secs, traced, casts, done = secs + dt, traced + tr, casts + ca, done + 1
        return secs, traced, casts, f"rows r + {step} k for r < {done}, rows claimed by {threads} threads"

    def frames(threads, budget):
        secs = traced = casts = nf = 0
        while secs < budget or nf == 0:
            dt, _, tot, tr = s.render_threaded(cam, SEED, threads)
            secs, traced, casts, nf = secs + dt, traced + tr, casts + tot, nf + 1
        return secs, traced, casts, f"{nf} whole frames, reference tile scheduler ({W // threads}px tiles)"

    rows = []
    for threads, budget in ((share, 0.6 * seconds), (1, 0.4 * seconds)):
        per_frame_est = W * H * spp * (1.3 if bounces > 1 else 1.0) / (1.0e6 * threads)  # ~1 Mray/s/thread
        fn = frames if per_frame_est < budget / 2 else rows_sample
        secs, traced, casts, how = fn(threads, budget)
        rows.append({"value": traced / secs / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
                     "sample": f"{asset} {W}x{H} spp={spp} bounces={bounces}: {how}, {traced} traced rays, "
                               f"{secs:.1f}s of render time", "ray_casts": casts,
                     "ray_casts_per_s": casts / secs})
    out = dict(rows[0])
    out["nproc"] = os.cpu_count()
    out["cpu_share"] = share
    out["single_thread"] = rows[1]
    return out


def spawn_ranks(n):
    """--gpus n without a launcher: run this script under torch.distributed.run as a child (no
    GPU call in this process), return its exit code."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ)).returncode


def launch_sizes(k, f, s=1):
    """k frames in launches of at most f, sizes as equal as possible, the launch count a multiple
    of the s streams they are dealt to round-robin (so every stream ends with the same work and
    none runs its last launch alone: 20 frames at f=4, s=2 -> 4,4,3,3,3,3, not 4,4,4,4,4)."""
    if k <= 0:
        return []
    n = (k + f - 1) // f
    n = min(k, (n + s - 1) // s * s)
    return [k // n + (1 if i < k % n else 0) for i in range(n)]


VARIANT_NAMES = {}


def calib_frames(args):
    """Orbit positions the cost plan is calibrated on: the last calib_frames positions before the
    timed window (warmup - c, ..., warmup - 1, taken modulo the orbit), never a timed frame."""
    c = max(1, args.calib_frames)
    return sorted({(args.warmup - c + i) % ORBIT_PERIOD for i in range(c)})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--variant", default="auto", choices=["auto", "lane", "flat", "hyb", "paths"])
    ap.add_argument("--variant-code", type=int, default=-1,
                    help="diagnostic: raw kernel code passed to the engine (overrides --variant's kernel)")
    ap.add_argument("--tuning", default="",
                    help="diagnostic: k=v,... scheduling knobs for atr_set_tuning (xcd_chunk, frame_rotate, hybrid_a, "
                         "hybrid_b, path_batch_log2, cluster_size, path_camera_occ, path_bounce_occ, primary_occ, path_sort_bits); outputs never change")
    ap.add_argument("--side", type=int, default=32,
                    help="shard tile side (pixels); 32 balances the 8-way c3 plan ~4%% better than 64 (DESIGN.md §5)")
    ap.add_argument("--cpu-seconds", type=float, default=16.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-prep", action="store_true", help="skip the device octree build timing")
    ap.add_argument("--no-steady", action="store_true",
                    help="skip the steady-state figure (64 further frames in 16-frame launches, after the timed region)")
    ap.add_argument("--no-orbit", action="store_true", help="every frame from the app camera")
    ap.add_argument("--streams", type=int, default=0,
                    help="launches in flight (one HIP stream each); 0 = 2 for the 1-spp configs (c1-c3: one "
                         "launch's tail hides behind the other's work) and 1 for the path-engine configs (c4, c5: "
                         "two concurrent launches share the caches that the sorted bounce queues rely on, "
                         "DESIGN.md §4h)")
    ap.add_argument("--frames-per-launch", type=int, default=0,
                    help="frames per launch (atr_render_start_cameras, at most MAX_FRAME_CAMS = 24); 1 = one frame per launch; "
                         "0 = the K steps in as few launches per stream as the cap allows, at least 4 x ranks "
                         "(a launch boundary inside a stream and the last launch's tail are the overheads)")
    ap.add_argument("--plan", default="cost", choices=["cost", "curve", "rr"],
                    help="N>1 tile deal: measured-cost longest-first (default), equal-cost runs of the "
                         "near-rectangles (compact shards), or round-robin")
    ap.add_argument("--calib-frames", type=int, default=3,
                    help="cost plan: per-tile costs summed over this many of the run's frames (one calibration render each)")
    ap.add_argument("--cell-split", default="",
                    help="P:FRAC -- the FRAC most expensive 8x8 cells (measured on the calibration frames) are "
                         "traced by P waves each (atr_set_cell_plan; scheduling only, same outputs)")
    ap.add_argument("--cell-order", default="graded", choices=["list", "graded"],
                    help="graded (default): cells dispatched by the calibration frames' measured cost, heaviest "
                         "class first (atr_set_cell_plan classes); list: tile list order (Morton within a tile)")
    ap.add_argument("--cell-prio", type=float, default=0.0,
                    help="with --cell-order graded: the heaviest FRAC of the cells issue at raised wave priority")
    ap.add_argument("--stream-priority", type=int, default=-1,
                    help="1: stream 0 at the device's highest priority (its launch completes first, so at N > 1 "
                         "its exchange overlaps the other launches' rendering); -1 (default) = on for N > 1")
    ap.add_argument("--tile-order", default="cost", choices=["cost", "grid"],
                    help="N>1 (and --single-tiles cost): each rank's tiles heaviest first (default) or in grid order")
    ap.add_argument("--single-tiles", default="frame", choices=["frame", "cost"],
                    help="N=1 tile list: one full-frame tile (default) or the shard grid, heaviest tiles first")
    ap.add_argument("--rank0-extra", type=float, default=-1.0,
                    help="rank 0's frame-assembly share, as a fraction of the mean per-rank load; "
                         "-1 (default): estimated from the calibration renders (S.assembly_share)")
    ap.add_argument("--exchange", default="masked", choices=["masked", "bgr", "bgrx"],
                    help="N>1 frame exchange: masked (default, round 6): a bit per pixel plus 3 bytes for each "
                         "pixel that differs from the background value (atr_pack_bgr_masked / "
                         "atr_scatter_bgr_masked; c3 ~0.54 B/px; sizes first, then the exact streams); bgr: 3 bytes "
                         "per pixel (the framebuffer's X byte is always 0; atr_pack_bgr / atr_scatter_bgr); bgrx: "
                         "the u32 framebuffer. gloo rehearsals stage the bytes through the host")
    ap.add_argument("--check", action="store_true",
                    help="rank 0: compare every assembled frame with a one-launch full-frame render")
    ap.add_argument("--sim-world", type=int, default=0,
                    help="diagnostic, one process: render only rank --sim-rank's shard of a --sim-world plan "
                         "(packed outputs, per-tile ray_casts sums; no exchange): the per-rank render side of an N-GPU run")
    ap.add_argument("--sim-rank", type=int, default=0)
    ap.add_argument("--pmc-child", action="store_true",
                    help="internal (the PMC passes' child run): stop right after the timed region")
    ap.add_argument("--selftest", action="store_true",
                    help="CPU only: synthetic fill instead of the render kernel (launch/plan/gather test)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if args.streams <= 0:
        args.streams = default_streams(args.config, args.steps, max(world, args.sim_world))
    if args.frames_per_launch <= 0:  # the library's cap: MAX_FRAME_CAMS cameras per launch
        args.frames_per_launch = min(MAX_FRAME_CAMS, max(4 * max(world, args.sim_world),
                                                         -(-args.steps // max(1, args.streams))))
    args.frames_per_launch = max(1, min(32, args.frames_per_launch))  # explicit: experiment builds may allow more
    if args.selftest:
        return selftest(args)
    return run(args)


def selftest(args):
    """Launch + shard plan + exact gather + assembly + per-tile ray_casts reduction on CPU (gloo)
    with a synthetic fill in place of the render kernel: rank r writes pixel index + 7 k into its
    packed framebuffer slots of frame k and (pixel % 5) into ray_casts. Rank 0 checks every
    assembled frame and every shard tile's ray_casts sum."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from atray_amd import shard as S
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        dist.init_process_group("gloo")
    asset, W, H = CONFIGS[args.config][:3]
    W, H = min(W, 480), min(H, 272)  # keep the CPU run small
    side = min(args.side, 32)
    n = len(S.E.shard_grid(W, H, side))
    costs = (np.arange(n) * 7919) % 97 + 1  # deterministic stand-in for the calibration render
    plan = S.ShardPlan.balanced(costs, W, H, world, side, max(0.0, args.rank0_extra)) if args.plan == "cost" \
        else S.ShardPlan.curve(costs, W, H, world, side, max(0.0, args.rank0_extra)) if args.plan == "curve" \
        else S.ShardPlan(W, H, world, side)
    F = args.frames_per_launch
    pix = torch.from_numpy(plan.pixel_map(rank).astype(np.int64)) if plan.sizes[rank] else torch.zeros(0, dtype=torch.int64)
    own = plan.sizes[rank]
    off = S.frame_offsets(plan, F)
    dst = torch.from_numpy(S.frames_assembly_index(plan, F))
    stile = torch.from_numpy(S.slot_tiles(plan, rank))
    ngrid = S.grid_tile_count(plan)
    want_tiles = torch.zeros(ngrid, dtype=torch.int64).index_add_(
        0, torch.from_numpy(S.pixel_tiles(W, H, side)), torch.arange(W * H) % 5)
    mism, casts_ok, frames = 0, True, 0
    t0 = time.perf_counter()
    k = 0
    for nf in launch_sizes(args.steps, F):
        big = torch.zeros(F * W * H, dtype=torch.int64)
        fb = big[off[0]:off[0] + F * own] if rank == 0 else torch.zeros(F * own, dtype=torch.int64)
        casts = torch.zeros(F, own, dtype=torch.int64)
        for f in range(nf):
            fb[f * own:(f + 1) * own] = pix + 7 * (k + f)
            casts[f] = pix % 5
        tsum = torch.zeros(F, ngrid, dtype=torch.int64).index_add_(1, stile, casts)
        bgr = args.exchange == "bgr"
        if args.exchange == "masked":  # the masked exchange through its host references
            bgv = 7 * k  # frame k's most common value (pixel index 0 + 7 k): any value is exact
            st = S.pack_bgr_masked_host(fb[:nf * own].numpy().astype(np.uint32), bgv) if own else np.zeros(0, np.uint8)
            nb = torch.tensor([st.size], dtype=torch.int64)
            img = torch.zeros(F * W * H, dtype=torch.int64)
            if world > 1:
                sizes = torch.zeros(world, dtype=torch.int64)
                for w_ in S.gather_sizes(nb, sizes if rank == 0 else None, plan, rank, dist):
                    w_.wait()
                bounds = [int(S.E.pack_bgr_masked_bound(nf * plan.sizes[r])) if plan.sizes[r] else 0
                          for r in range(world)] if rank == 0 else None
                roff = [0] + list(np.cumsum(bounds)) if rank == 0 else None
                recv = torch.zeros(max(1, int(roff[-1])), dtype=torch.uint8) if rank == 0 else None
                for w_ in S.gather_streams(torch.from_numpy(st), recv, roff, sizes.tolist() if rank == 0 else None,
                                           plan, rank, dist):
                    w_.wait()
                for w_ in [dist.reduce(tsum, dst=0, async_op=True)]:
                    w_.wait()
            if rank == 0:
                im = np.zeros(F * W * H, np.uint32)
                if own:
                    im[dst[off[0]:off[0] + nf * own].numpy()] = fb[:nf * own].numpy().astype(np.uint32)
                for r in range(1, world):
                    if plan.sizes[r]:
                        S.scatter_bgr_masked_host(recv[int(roff[r]):].numpy(), nf * plan.sizes[r],
                                                  dst[off[r]:off[r] + nf * plan.sizes[r]].numpy(), im)
                img = torch.from_numpy(im.astype(np.int64))
                want = torch.arange(W * H, dtype=torch.int64)
                for f in range(nf):
                    got = img[f * W * H:(f + 1) * W * H]
                    mism += int((got != want + 7 * (k + f)).sum())
                    casts_ok &= bool(torch.equal(tsum[f], want_tiles))
                    frames += 1
            k += nf
            continue
        if bgr:  # the 3-byte exchange through the host references of atr_pack_bgr / atr_scatter_bgr
            big3 = torch.zeros(3 * F * W * H, dtype=torch.uint8)
            mine = torch.from_numpy(S.pack_bgr_host(fb[:F * own].numpy().astype(np.uint32)))
            if rank == 0:
                big3[3 * off[0]:3 * off[0] + 3 * F * own] = mine
        if world > 1:
            if bgr:
                works = S.gather_frames(mine, big3, plan, rank, nf, dist, unit=3)
            else:
                works = S.gather_frames(fb, big, plan, rank, nf, dist)
            works.append(dist.reduce(tsum, dst=0, async_op=True))
            for w_ in works:
                w_.wait()
        if rank == 0:
            img = torch.zeros(F * W * H, dtype=torch.int64)
            if bgr:
                im = np.zeros(F * W * H, np.uint32)
                S.scatter_bgr_host(big3.numpy(), dst.numpy(), im)
                img = torch.from_numpy(im.astype(np.int64))
            else:
                img.index_copy_(0, dst, big)
            want = torch.arange(W * H, dtype=torch.int64)
            for f in range(nf):
                got = img[f * W * H:(f + 1) * W * H]
                mism += int((got != want + 7 * (k + f)).sum())
                casts_ok &= bool(torch.equal(tsum[f], want_tiles))
                frames += 1
        k += nf
    elapsed = time.perf_counter() - t0
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 4),
                          "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
                          "data": "selftest: synthetic fill, no GPU", "selftest": True,
                          "config": {"workload": f"{args.config} plan/gather selftest {W}x{H}",
                                     "exchange": args.exchange,
                                     "parallelism": f"tiles{world}", "shard_pixels": [int(x) for x in plan.sizes]},
                          "frames_checked": frames, "check_mismatched_pixels": mism,
                          "total_ray_casts_ok": bool(casts_ok)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    import atray_amd.engine as E
    from atray_amd import shard as S
    from atray_amd.assets import CENTERS, asset_path

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(local % ndev)  # ranks > devices only for gloo rehearsals on one GPU
    dev = torch.device("cuda", local % ndev)
    backend = os.environ.get("ATR_DIST_BACKEND", "nccl")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    asset, W, H, spp, bounces, use_tree = CONFIGS[args.config]
    variant = {"auto": E.ATR_KERNEL_AUTO, "lane": E.ATR_KERNEL_LANE, "flat": E.ATR_KERNEL_FLAT,
               "hyb": E.ATR_KERNEL_HYBRID, "paths": E.ATR_KERNEL_PATHS}[args.variant]
    VARIANT_NAMES.update({E.ATR_KERNEL_AUTO: "auto", E.ATR_KERNEL_FLAT: "flat", E.ATR_KERNEL_HYBRID: "hybrid",
                          E.ATR_KERNEL_LANE: "lane", E.ATR_KERNEL_PATHS: "paths"})
    if args.variant_code >= 0:
        variant = args.variant_code
    # ---- scene prep (untimed for Mrays/s; reported under "prep")
    prep = {}
    path = asset_path(asset)
    t = time.perf_counter()
    mesh = E.Mesh.load_obj(path)  # load_model_data, parallel chunks (OBJ_loader.cpp:298-340)
    prep["obj_load_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = None
    if use_tree:
        t = time.perf_counter()
        tree = E.Octree.build(mesh, 300)
        prep["octree_host_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    eng = E.Engine(local % ndev)
    if args.tuning:
        eng.set_tuning(**{k: int(v) for k, v in (kv.split("=") for kv in args.tuning.split(","))})
    if use_tree and not args.no_prep and rank == 0:
        tm = {}
        E.Octree.build_device(mesh, 300, local % ndev, timings=tm)  # f3: same tree on the GPU
        prep["octree_device_ms"] = round(tm["wall_ms"], 2)
        prep["octree_device_kernel_ms"] = round(tm["device_ms"], 3)
    t = time.perf_counter()
    eng.upload(MATERIALS, [(mesh, tree, box, 1)])
    torch.cuda.synchronize()
    prep["upload_ms"] = round((time.perf_counter() - t) * 1e3, 2)
    prep["scene_device_bytes"] = eng.scene_info()["device_bytes"]
    app_cam = E.camera(W, H, spp, bounces)
    n_orbit = 1 if args.no_orbit else ORBIT_PERIOD
    cams = [app_cam if args.no_orbit else E.camera(W, H, spp, bounces, eye=orbit_eye(k), facing=APP_FACING)
            for k in range(n_orbit)]

    # ---- shard plan (untimed): one calibration render measures every grid tile's cost on rank 0,
    # broadcast so all ranks derive the same longest-first deal
    sim = world == 1 and args.sim_world > 1
    pw, pr = (args.sim_world, args.sim_rank) if sim else (world, rank)  # the plan's world and rank
    heavy_first = args.tile_order == "cost"
    if (pw > 1 and args.plan in ("cost", "curve")) or (pw == 1 and args.single_tiles == "cost"):
        # measured on frames BEFORE the timed window (the warmup's orbit positions, or the positions
        # just before them): a live renderer only has its previous frames
        ks = calib_frames(args)
        costs = np.zeros(len(E.shard_grid(W, H, args.side)), np.int64)
        calib_ms = []
        if rank == 0:
            for k in ks:
                torch.cuda.synchronize()
                t_ = time.perf_counter()
                costs += S.tile_costs(eng, cams[k % n_orbit], W, H, args.side, SEED)
                calib_ms.append((time.perf_counter() - t_) * 1e3)
        if args.rank0_extra < 0:  # rank 0's assembly against a rank's render, from the calibration
            args.rank0_extra = S.assembly_share(W * H, float(np.median(calib_ms)) if calib_ms else 0.0, pw)
            if world > 1:
                args.rank0_extra = float(S.shared_costs(np.array([int(args.rank0_extra * 1e6)]), rank, dist,
                                                        dev if backend == "nccl" else "cpu")[0]) / 1e6
        if world > 1:
            costs = S.shared_costs(costs, rank, dist, dev if backend == "nccl" else "cpu")
        mk = S.ShardPlan.curve if (pw > 1 and args.plan == "curve") else S.ShardPlan.balanced
        plan = mk(costs, W, H, pw, args.side, args.rank0_extra, heavy_first)
    else:
        plan = S.ShardPlan(W, H, pw, args.side)
    sizes = plan.sizes
    cell_split = None
    if args.cell_split or args.cell_order != "list":
        # the run's calibration frames' per-cell costs: the heaviest cells split over P waves
        # (--cell-split P:FRAC) and/or every cell graded into dispatch classes by cost, heaviest
        # first (--cell-order graded: the single-frame plan's class fractions, plan.hip), so a
        # launch's slowest cells start first instead of forming its tail
        ks = calib_frames(args)
        cc = sum(eng.cell_costs(cams[k % n_orbit], SEED, variant) for k in ks).ravel()
        cplan = np.zeros(cc.size, np.uint8)
        corder = np.argsort(-cc, kind="stable")
        cell_split = {"of": int(cc.size)}
        if args.cell_split:
            parts, frac = args.cell_split.split(":")
            nsplit = int(round(float(frac) * cc.size))
            cplan[corder[:nsplit]] = int(parts)
            cell_split.update(parts=int(parts), cells=nsplit)
        if args.cell_order != "list":  # class 7 for the top 2 %, ..., 0 for the rest; --cell-prio:
            cplan |= S.graded_cell_plan(cc, args.cell_prio)  # the heaviest cells' waves issue first
            cell_split["order"] = args.cell_order
            cell_split["prio_frac"] = args.cell_prio
        eng.set_cell_plan(W, H, cplan)
    if pw > 1 or args.single_tiles == "cost":
        tiles_list = [list(t) for t in plan.tiles[pr]]
    else:
        tiles_list = [[0, 0, W - 1, H - 1]]
    tiles = E.tiles_array(tiles_list)
    S_, F_ = max(1, args.streams), args.frames_per_launch
    # --stream-priority: stream 0 at the device's highest priority, so its launch's workgroups are
    # dispatched first and it completes early; the other streams' work fills its tail, and at
    # N > 1 its exchange overlaps their rendering
    if args.stream_priority < 0:
        args.stream_priority = int(pw > 1)
    hi_prio = torch.cuda.Stream.priority_range()[1] if args.stream_priority else 0
    streams = [torch.cuda.Stream(dev, priority=hi_prio if q == 0 else 0) for q in range(S_)]
    launch_ev = []  # per timed launch: (frames, event before its render, event after), launch order
    launch_xev = []  # N > 1: per timed launch, an event after its exchange encoding (before the counters)
    own = W * H if pw == 1 else sizes[pr]  # output elements per frame (stride between frames)
    npx = W * H
    on_host = world > 1 and backend != "nccl"
    # 3-byte exchange (atr_pack_bgr / atr_scatter_bgr on the device; a gloo rehearsal stages the
    # packed bytes through the host)
    bgr = pw > 1 and args.exchange == "bgr"
    masked = pw > 1 and args.exchange == "masked"
    traced = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(S_)]
    # per stream slot: F framebuffers and F ray_casts images (u32), frames back to back
    casts = [torch.zeros(F_ * max(1, own), dtype=torch.int32, device=dev) for _ in range(S_)]
    if pw == 1:
        fbs = [torch.zeros(F_ * npx, dtype=torch.int32, device=dev) for _ in range(S_)]
    else:
        # N > 1: rank r's packed frames go to rank 0 by exact-size send/recv into one buffer per
        # slot holding every rank's F frames back to back (shard.frame_offsets); rank 0 renders
        # its own block in place. The per-pixel ray_casts stay on their rank: each rank reduces
        # them to per-tile sums (the reference's per-tile counters) and those are summed on rank 0.
        off = S.frame_offsets(plan, F_)
        ngrid = S.grid_tile_count(plan)
        tids = torch.from_numpy(S.tile_ids(plan, pr)).to(dev)
        tcasts = [torch.zeros(F_, max(1, len(tids)), dtype=torch.int64, device=dev) for _ in range(S_)]
        tsum = [torch.zeros(F_, ngrid, dtype=torch.int64, device="cpu" if on_host else dev) for _ in range(S_)]
        if masked:
            # masked exchange: every rank encodes its F frames into one stream (atr_pack_bgr_masked);
            # the streams' sizes go to rank 0 first, then the exact streams; rank 0 decodes each into
            # the images through the assembly index and copies its own frames in directly
            fbs = [torch.zeros(F_ * max(1, own), dtype=torch.int32, device=dev) for _ in range(S_)]
            enc = [torch.zeros(E.pack_bgr_masked_bound(F_ * max(1, own)), dtype=torch.uint8, device=dev)
                   for _ in range(S_)]
            nbytes = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(S_)]
            if rank == 0 and not sim:
                bounds = [E.pack_bgr_masked_bound(F_ * sizes[r]) if sizes[r] else 0 for r in range(world)]
                roff = [0] + list(np.cumsum(bounds))
                recv = [torch.zeros(max(1, int(roff[-1])), dtype=torch.uint8, device="cpu" if on_host else dev)
                        for _ in range(S_)]
                recv_dev = [torch.zeros(max(1, int(roff[-1])), dtype=torch.uint8, device=dev) for _ in range(S_)] \
                    if on_host else recv
                nsz = [torch.zeros(world, dtype=torch.int64, device="cpu" if on_host else dev) for _ in range(S_)]
                dst_idx = torch.from_numpy(S.frames_assembly_index(plan, F_)).to(dev)
                images = [torch.zeros(F_ * npx, dtype=torch.int32, device=dev) for _ in range(S_)]
                rtiles = [E.tiles_array([list(t) for t in plan.tiles[r]]) if sizes[r] else None for r in range(world)]
        elif bgr:
            # 3-byte exchange: every rank packs its F frames into bytes (rank 0 straight into its
            # block of the byte gather buffer), rank 0 scatters the gathered bytes into the images
            fbs = [torch.zeros(F_ * max(1, own), dtype=torch.int32, device=dev) for _ in range(S_)]
            if rank == 0 and not sim:
                big = [torch.zeros(3 * F_ * npx, dtype=torch.uint8, device=dev) for _ in range(S_)]
                if on_host:  # gloo: the gather lands in host memory, then goes to the device
                    bigh = [torch.zeros(3 * F_ * npx, dtype=torch.uint8) for _ in range(S_)]
                dst_idx = torch.from_numpy(S.frames_assembly_index(plan, F_)).to(dev)
                images = [torch.zeros(F_ * npx, dtype=torch.int32, device=dev) for _ in range(S_)]
                send3 = [b_[3 * off[0]:3 * off[0] + 3 * F_ * own] for b_ in big]
            else:
                send3 = [torch.zeros(3 * F_ * max(1, own), dtype=torch.uint8, device=dev) for _ in range(S_)]
        elif rank == 0 and not sim:
            big = [torch.zeros(F_ * npx, dtype=torch.int32, device="cpu" if on_host else dev) for _ in range(S_)]
            dst_idx = torch.from_numpy(S.frames_assembly_index(plan, F_)).to(dev)
            images = [torch.zeros(F_ * npx, dtype=torch.int32, device=dev) for _ in range(S_)]
            staging = torch.zeros(F_ * npx, dtype=torch.int32, device=dev) if on_host else None
            fbs = [b_[off[0]:off[0] + F_ * own] if not on_host else torch.zeros(F_ * max(1, own), dtype=torch.int32, device=dev)
                   for b_ in big]
        else:
            fbs = [torch.zeros(F_ * max(1, own), dtype=torch.int32, device=dev) for _ in range(S_)]
    layout = E.ATR_LAYOUT_IMAGE if pw == 1 else E.ATR_LAYOUT_PACKED

    def frame_of(q):
        return E.atr_frame(layout, fbs[q].data_ptr(), None, None, None, casts[q].data_ptr(), traced[q].data_ptr())

    pending = {}
    launch_nf = {}
    timing = [False]
    bgv = [0]  # the masked exchange's background value (this rank's most common pixel, set below)

    def image_views(q, f):
        """(framebuffer, ray_casts or None) of frame f of stream slot q: (H*W,) views; at N > 1
        the ray_casts are the reduced per-tile sums (ngrid,)."""
        if pw == 1:
            return fbs[q][f * npx:(f + 1) * npx], casts[q][f * npx:(f + 1) * npx]
        if sim:
            return None, tsum[q][f]
        return images[q][f * npx:(f + 1) * npx], tsum[q][f]

    def assemble(j):
        """Launch j's exchange done (its stream waits on it); rank 0 scatters every rank's packed
        frames into that slot's images, on the launch's stream."""
        q, works = pending.pop(j)
        if world == 1:
            return
        with torch.cuda.stream(streams[q]):
            for w_ in works:
                w_.wait()
            if masked:  # the sizes are in: the exact streams, then rank 0 decodes them
                nf = launch_nf[j]
                if rank == 0:
                    sz = nsz[q].cpu().tolist()
                    works2 = S.gather_streams(None, recv[q], roff, sz, plan, rank, dist)
                else:
                    mine = int(nbytes[q].item()) if own else 0
                    src = enc[q][:mine].cpu() if on_host else enc[q][:mine]
                    works2 = S.gather_streams(src, None, None, None, plan, rank, dist)
                for w_ in works2:
                    w_.wait()
                if rank == 0:
                    if on_host:
                        recv_dev[q].copy_(recv[q])
                    # every other rank's stream and rank 0's own packed frames in one call,
                    # positions from each source's tile blocks (atr_unpack_masked_ranks: one
                    # launch pair instead of two launches per rank and an index copy)
                    src = [r for r in range(1, world) if sizes[r]]
                    tl = [rtiles[r] for r in src] + ([rtiles[0]] if own else [])
                    ptrs = [recv_dev[q][int(roff[r]):].data_ptr() for r in src] + ([fbs[q].data_ptr()] if own else [])
                    if tl:
                        eng.unpack_masked_ranks(tl, W, H, ptrs, nf, images[q].data_ptr(), npx,
                                                stream=streams[q].cuda_stream, raw=[0] * len(src) + [1] * (1 if own else 0))
                return
            if rank == 0 and bgr:
                if on_host:
                    big[q].copy_(bigh[q])
                eng.scatter_bgr(big[q].data_ptr(), big[q].numel() // 3, dst_idx.data_ptr(), images[q].data_ptr(),
                                stream=streams[q].cuda_stream)
            elif rank == 0:
                src = big[q]
                if on_host:
                    staging.copy_(src, non_blocking=False)
                    src = staging
                images[q].index_copy_(0, dst_idx, src)

    def launch(j, k0, nf, q):
        if j - S_ in pending:
            assemble(j - S_)  # before this slot's buffers are reused
        fr = [cams[(k0 + f) % n_orbit] for f in range(nf)]
        if timing[0]:
            ev_a = torch.cuda.Event(enable_timing=True)
            ev_a.record(streams[q])
        eng.render_start_cameras(fr, tiles, frame_of(q), own, SEED, stream=streams[q].cuda_stream, variant=variant)
        if timing[0]:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(streams[q])
            launch_ev.append((nf, ev_a, ev))
        if pw > 1:
            with torch.cuda.stream(streams[q]):
                # the exchange's encoding first (it heads the critical path: encode, sizes, streams,
                # rank 0's decode), then the per-tile counters, which only the reduction needs
                if bgr and own:  # the rank's frames in 3 bytes per pixel (part of its per-rank work)
                    eng.pack_bgr(fbs[q].data_ptr(), nf * own, send3[q].data_ptr(), stream=streams[q].cuda_stream)
                if masked and own and pr != 0:  # the rank's frames as one masked stream (rank 0 keeps its own)
                    eng.pack_bgr_masked(fbs[q].data_ptr(), nf * own, bgv[0], enc[q].data_ptr(), nbytes[q].data_ptr(),
                                        stream=streams[q].cuda_stream)
                if timing[0] and sim:  # the launch's streams are ready to send from here (projection)
                    ev_x = torch.cuda.Event(enable_timing=True)
                    ev_x.record(streams[q])
                    launch_xev.append(ev_x)
                ts = tsum[q]
                if rank == 0 and not sim:  # the reduction lands in rank 0's buffer: clear it; other
                    ts.zero_()             # ranks' stay zero outside their own tile columns
                if own:  # the reference's per-tile counters of this rank's tiles, scattered into the grid
                    eng.packed_tile_ray_casts(tiles, W, H, casts[q].data_ptr(), nf, own, tcasts[q].data_ptr(),
                                              stream=streams[q].cuda_stream)
                    part = tcasts[q][:, :len(tids)]
                    if on_host:
                        ts.index_copy_(1, tids.cpu(), part.cpu())
                    else:
                        ts.index_copy_(1, tids, part)
                launch_nf[j] = nf
                if sim:
                    pending[j] = (q, [])
                    return
                if masked:  # phase 1: every stream's byte count to rank 0 (phase 2 in assemble)
                    if on_host:
                        torch.cuda.synchronize()
                        works = S.gather_sizes(nbytes[q].cpu(), nsz[q] if rank == 0 else None, plan, rank, dist)
                    else:
                        works = S.gather_sizes(nbytes[q], nsz[q] if rank == 0 else None, plan, rank, dist)
                    works.append(dist.reduce(ts, dst=0, async_op=True))
                    pending[j] = (q, works)
                    return
                if bgr:
                    if on_host:
                        torch.cuda.synchronize()
                        send = send3[q][:3 * nf * own].cpu()
                        if rank == 0:
                            bigh[q][3 * off[0]:3 * off[0] + 3 * nf * own] = send
                        works = S.gather_frames(send, bigh[q] if rank == 0 else None, plan, rank, nf, dist, unit=3)
                    else:
                        works = S.gather_frames(send3[q], big[q] if rank == 0 else None, plan, rank, nf, dist, unit=3)
                    works.append(dist.reduce(ts, dst=0, async_op=True))
                    pending[j] = (q, works)
                    return
                send = fbs[q]
                if on_host:
                    torch.cuda.synchronize()
                    send = send.cpu()
                    if rank == 0:
                        big[q][off[0]:off[0] + nf * own] = send[:nf * own]
                works = S.gather_frames(send, big[q] if rank == 0 else None, plan, rank, nf, dist)
                works.append(dist.reduce(ts, dst=0, async_op=True))
                pending[j] = (q, works)
        else:
            pending[j] = (q, [])

    def run_frames(k0, k, on_launch=None):
        j0 = 0
        for nf in launch_sizes(k, F_, S_):
            q = j0 % S_
            launch(j0, k0, nf, q)
            if on_launch:
                on_launch(j0, k0, nf, q)
            k0 += nf
            j0 += 1
        for j in sorted(pending):
            assemble(j)

    # setup, not warmup: one small launch on every stream (a stream's first launch pays its
    # hardware-queue setup, ~ms) so the timed region does not depend on W reaching every stream
    for q in range(S_):
        eng.render_start_cameras([cams[0]], tiles, frame_of(q), own, SEED, stream=streams[q].cuda_stream,
                                 variant=variant)
    torch.cuda.synchronize()
    if masked and own:  # untimed: the background value from this rank's first frame (any value is exact)
        bgv[0] = S.background_value(fbs[0][:own].cpu().numpy().view(np.uint32))
    if world > 1:
        dist.barrier()
    run_frames(0, args.warmup)
    torch.cuda.synchronize()
    for t_ in traced:
        t_.zero_()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev0.record(streams[0])
    timing[0] = True
    t0 = time.perf_counter()
    run_frames(args.warmup, args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    timing[0] = False
    if args.pmc_child:  # the profiler's view: the timed region is this process's last GPU work
        eng.close()
        if world > 1:
            dist.destroy_process_group()
        return
    launch_done = [round(ev0.elapsed_time(e), 3) for _, _, e in launch_ev]  # ms after the timed region's start
    launch_ms = [a.elapsed_time(e) for _, a, e in launch_ev]  # each timed launch's render, on its stream
    launch_frames = [nf for nf, _, _ in launch_ev]
    launch_encoded = [round(ev0.elapsed_time(e), 3) for e in launch_xev]
    stream_bpf = None  # this rank's masked stream bytes per frame (the last launch of each stream)
    if masked and own and pr != 0:
        js = sorted(launch_nf)[-S_:]
        stream_bpf = round(sum(int(nbytes[j % S_].item()) for j in js) / max(1, sum(launch_nf[j] for j in js)))
    rays = torch.stack(traced).sum().reshape(1)
    local_rays_per_frame = float(rays.item()) / max(1, args.steps)  # this rank's traced rays per frame
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
        rays = rays if backend == "nccl" else rays.cpu()
        dist.all_reduce(rays)
    rays_total = int(rays.item())

    # ---- check (rank 0): the last S x F frames in the slots against one-launch full-frame renders
    # (framebuffer per pixel; ray_casts per pixel at N = 1, per shard tile at N > 1)
    check = None
    casts_total = None
    if rank == 0:
        ref = torch.zeros(W * H, dtype=torch.int32, device=dev)
        refc = torch.zeros(W * H, dtype=torch.int32, device=dev)
        if pw > 1 and not sim:
            full_tiles = torch.from_numpy(S.pixel_tiles(W, H, args.side)).to(dev)
        sizes_l = launch_sizes(args.steps, F_, S_)
        k0 = args.warmup
        last = {}
        for j, nf in enumerate(sizes_l):
            last[j % S_] = (k0, nf)
            k0 += nf
        casts_total = 0
        mism = 0
        for q, (kk, nf) in sorted(last.items()):
            for f in range(nf):
                fb, cs = image_views(q, f)
                casts_total += int(cs.to(torch.int64).sum().item())
                if args.check and not sim:
                    fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, ref.data_ptr(), None, None, None, refc.data_ptr(), None)
                    eng.render_start(cams[(kk + f) % n_orbit], [[0, 0, W - 1, H - 1]], fr, SEED,
                                     stream=torch.cuda.current_stream(dev).cuda_stream)
                    torch.cuda.synchronize()
                    mism += int((ref != fb).sum().item())
                    if world == 1:
                        mism += int((refc != cs).sum().item())
                    else:  # every shard tile's ray_casts sum (a mismatching tile counts as one)
                        want = torch.zeros(ngrid, dtype=torch.int64, device=dev).index_add_(0, full_tiles, refc.to(torch.int64))
                        mism += int((want.cpu() != cs.cpu()).sum().item())
        check = mism if args.check else None
        casts_frames = sum(nf for _, nf in last.values())

    # ---- the roofline kernel: the timed launches' schedule, one app-camera frame per launch,
    # serialized (AUTO: HYBRID for primary-only frames, the path engine otherwise; capi.cpp auto_sched)
    roof_variant = variant
    if variant == E.ATR_KERNEL_AUTO:
        roof_variant = E.ATR_KERNEL_HYBRID if bounces == 1 and spp == 1 else E.ATR_KERNEL_PATHS
    s0 = streams[0]

    def time_one(v, n=10):
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for a, b in evs:
            a.record(s0)
            eng.render_start(app_cam, tiles, frame_of(0), SEED, stream=s0.cuda_stream, variant=v)
            b.record(s0)
        torch.cuda.synchronize()
        rc, _ = eng.wait()
        assert rc == 0
        return float(np.mean([a.elapsed_time(b) for a, b in evs]))
    kern_ms = time_one(roof_variant)

    def latency_one(v, n=10):
        # the live view's case: one frame on an idle GPU, render start -> framebuffer complete
        # (atr_last_kernel_ms: the library's events around the render alone; the plan kernels that
        # prepare the NEXT frame's dispatch run after that point and are in time_one's period)
        lat = []
        for _ in range(n):
            eng.render_start(app_cam, tiles, frame_of(0), SEED, stream=s0.cuda_stream, variant=v)
            torch.cuda.synchronize()
            lat.append(eng.last_kernel_ms())
        rc, _ = eng.wait()
        assert rc == 0
        return float(np.median(lat))
    lat_ms = latency_one(roof_variant)
    # steady state (informational, not `value`): 64 further orbit frames in 16-frame launches on the
    # same streams, after the timed region -- the rate without a short run's pipeline fill and drain
    steady = None
    if not args.no_steady and pw == 1 and world == 1:
        F0 = F_
        nst = 64
        torch.cuda.synchronize()
        for t_ in traced:
            t_.zero_()
        fst = min(16, F0)
        t1 = time.perf_counter()
        k0 = args.warmup + args.steps
        for j, nf in enumerate(launch_sizes(nst, fst, S_)):
            q = j % S_
            fr = [cams[(k0 + f) % n_orbit] for f in range(nf)]
            eng.render_start_cameras(fr, tiles, frame_of(q), own, SEED, stream=streams[q].cuda_stream, variant=variant)
            k0 += nf
        torch.cuda.synchronize()
        dt = time.perf_counter() - t1
        st_rays = int(torch.stack(traced).sum().item())
        steady = {"frames": nst, "frames_per_launch": fst, "ms_per_frame": round(dt / nst * 1e3, 4),
                  "mrays_s": round(st_rays / dt / 1e6, 1)}
    live_ctr = eng.counters(app_cam, tiles, SEED, roof_variant) if rank == 0 else None

    if rank == 0:
        value = rays_total / elapsed / 1e6
        out = {"metric": METRIC, "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic: the survey's Dragon surrogate (Dragon.obj absent), app materials, "
                       + ("app camera every frame" if args.no_orbit else
                          f"camera orbit r={ORBIT_RADIUS} around the app eye, {ORBIT_PERIOD} distinct frames"),
               "config": {"workload": f"{args.config}: {asset} {W}x{H} spp={spp} bounces={bounces} "
                                      f"{'octree' if use_tree else 'brute-force'}",
                          "rays_per_step": round(rays_total / args.steps), "shard_tile": args.side,
                          "parallelism": f"tiles{world}", "kernel": args.variant,
                          **({"tuning": eng.tuning()} if args.tuning else {}),
                          "plan": (f"{args.plan}/{args.tile_order}" if pw > 1 else
                                   "single" if args.single_tiles == "frame" else f"single/{args.tile_order}"),
                          "streams": args.streams, "frames_per_launch": F_,
                          **({"exchange": "masked (mask bit + 3 B per non-background px)" if masked else
                              "bgr (3 B/px)" if bgr else "bgrx (4 B/px)"} if pw > 1 else {}),
                          "launches": launch_sizes(args.steps, F_, S_),
                          **({"rank0_extra": round(args.rank0_extra, 4)} if pw > 1 else {}),
                          "launch_render_done_ms": launch_done,
                          **({"launch_encoded_ms": launch_encoded} if launch_encoded else {}),
                          "stream_priority": bool(args.stream_priority),
                          "cell_plan": cell_split,
                          "shard_pixels": [int(x) for x in sizes]},
               **({"sim": {"world": pw, "rank": pr, "note": "one rank's shard rendered alone, no exchange",
                           "stream_bytes_per_frame": stream_bpf}} if sim else {}),
               "total_ray_casts_per_frame": round(casts_total / max(1, casts_frames))}
        if steady:
            out["steady_state"] = steady
        if (pw > 1 and args.plan in ("cost", "curve")) or args.cell_split or args.cell_order != "list" or \
            (pw == 1 and args.single_tiles == "cost"):
            out["config"]["calibration_frames"] = calib_frames(args)  # orbit positions, all before the timed ones
        if check is not None:
            out["check_mismatched_pixels"] = check
        n1 = live_ctr["n_rays"]
        out["single_frame"] = {"kernel_ms": round(kern_ms, 4), "mrays_s": round(n1 / kern_ms / 1e3, 1),
                               "latency_ms": round(lat_ms, 4),
                               "camera": "app", "rays": n1, "variant": VARIANT_NAMES.get(roof_variant, roof_variant)}
        # roofline. HBM: the bytes HBM actually moved (PMC, per timed launch of this
        # command's shape, per frame) over the measured time per frame -- the kernel's real HBM
        # fraction. Algorithmic models beside it: the compulsory bytes (outputs + one read of the
        # scene per launch) and the clustered scan's own-work bytes per ray at chip level (cache-level
        # traffic: above the HBM peak, which is why it cannot be the HBM fraction). VALU: the binding
        # resource, wave-instructions issued per second against the chip's issue peak.
        clustered = args.variant in ("auto", "flat", "hyb", "paths")
        bpr = cluster_bytes_per_ray(live_ctr) if clustered else algorithmic_bytes_per_ray(live_ctr)
        step_s = elapsed / args.steps
        fpl = max(launch_frames)
        out_bytes = (4 + 4) * (own if pw > 1 else W * H)  # framebuffer + ray_casts, u32 each, per frame
        scene_bytes = prep["scene_device_bytes"]
        compulsory = out_bytes + scene_bytes / fpl
        roof = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s", "kernel": None, "variant": None,
                "ms_per_frame": round(step_s * 1e3, 4), "frames_per_launch": launch_frames,
                "launch_ms": [round(x, 3) for x in launch_ms], "concurrent_launches": S_,
                "compulsory": {"bytes_per_frame": round(compulsory), "achieved": round(compulsory / step_s / 1e9, 1),
                               "frac": round(compulsory / step_s / 1e9 / HBM_PEAK_GBS, 5),
                               "model": "outputs (framebuffer + ray_casts, 8 B/px) + the scene read once per launch"},
                "own_work": {"bytes_per_ray": round(bpr, 1), "achieved_chip": round(bpr * rays_total / args.steps / world
                                                                                      / step_s / 1e9, 1),
                             "model": ("clustered scan, own work (DESIGN.md §6): L1/LDS/L2-level bytes"
                                       if clustered else "reference work (SURVEY.md 8(d))")},
                "single_frame_launch": {"kernel_ms": round(kern_ms, 4), "rays": n1}}
        gname = GOLDEN_COUNTERS.get(args.config)
        if gname:  # the reference algorithm's bytes per ray for the same rays
            with open(os.path.join(ROOT, "tests", "golden", "goldens.json")) as f:
                ctr = json.load(f)["hits"][gname]["counters"]
            roof["own_work"]["ref_bytes_per_ray"] = round(algorithmic_bytes_per_ray(ctr), 1)
        kname = "path_" if roof_variant == E.ATR_KERNEL_PATHS else "render_kernel"
        roof["kernel"] = kname
        roof["variant"] = VARIANT_NAMES.get(roof_variant, roof_variant)
        # default: the compulsory model (no counters); replaced by the PMC-measured bytes below
        roof["achieved"] = roof["compulsory"]["achieved"]
        roof["frac"] = roof["compulsory"]["frac"]
        roof["traffic"] = None
        roof["source"] = "compulsory bytes (no PMC)"
        paths = roof_variant == E.ATR_KERNEL_PATHS
        if world == 1 and not args.no_pmc and paths:
            # the path engine: every kernel of the timed frames (camera, bounces, resolve), per frame
            tune = eng.tuning()
            tail = path_dispatches(args, tiles_list, W, H, spp, bounces, tune["path_batch_log2"], tune["path_sort_bits"])
            pmc, info, why = pmc_counters(args, "path_", tail)
            roof["pmc_note"] = why
            roof["kernel"] = ("path engine: path_camera_kernel + path_bounce_kernel x (bounces - 1) + path_resolve_kernel"
                              + (" + queue sort (path_sort_*) x (bounces - 1)" if len(tail) > 3 else ""))
            if pmc and "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
                K = args.steps
                per_frame = (2.0 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0 / K
                roof["traffic"] = round(per_frame)
                roof["traffic_per_frame"] = round(per_frame)
                roof["traffic_per_traced_ray"] = round(per_frame / (rays_total / K), 1)
                roof["pmc_frames"] = {"frames": K, "dispatches": info["dispatches"],
                                      "fetch_bytes_per_frame": round(2.0 * pmc["FETCH_SIZE"] * 1024.0 / K),
                                      "write_bytes_per_frame": round(pmc["WRITE_SIZE"] * 1024.0 / K),
                                      "per_kernel_bytes_per_frame": {
                                          kn: round((2.0 * v.get("FETCH_SIZE", 0.0) + v.get("WRITE_SIZE", 0.0)) * 1024.0 / K)
                                          for kn, v in info["per_kernel"].items()}}
                roof["achieved"] = round(per_frame / step_s / 1e9, 2)
                roof["frac"] = round(per_frame / step_s / 1e9 / HBM_PEAK_GBS, 5)
                roof["source"] = "PMC bytes of the timed frames' path kernels / frames / measured time per frame"
            if pmc and "SQ_INSTS_VALU" in pmc:
                valu_frame = pmc["SQ_INSTS_VALU"] / args.steps
                roof["valu"] = {"bound": "valu-issue", "wave_insts_per_frame": round(valu_frame),
                                "achieved": round(valu_frame / step_s / 1e9, 1), "peak": round(VALU_ISSUE_PEAK / 1e9, 1),
                                "unit": "G wave-instr/s", "frac": round(valu_frame / step_s / VALU_ISSUE_PEAK, 4),
                                "wait_frac": round(pmc.get("SQ_WAIT_ANY", 0.0) / max(1.0, pmc.get("SQ_WAVE_CYCLES", 1.0)), 4),
                                "waves_per_frame": round(pmc.get("SQ_WAVES", 0.0) / args.steps),
                                "per_kernel_insts_per_frame": {kn: round(v.get("SQ_INSTS_VALU", 0.0) / args.steps)
                                                               for kn, v in info["per_kernel"].items()}}
            if pmc and "TCC_HIT_sum" in pmc:
                h, m = pmc["TCC_HIT_sum"], pmc.get("TCC_MISS_sum", 0.0)
                roof["l2_hit_rate"] = round(h / max(1.0, h + m), 4)
        elif world == 1 and not args.no_pmc:
            pmc, info, why = pmc_counters(args, kname)
            grid = info["grid"] if info else None
            roof["pmc_note"] = why
            if pmc and "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
                # FETCH_SIZE doubled (MI355X_MICROARCH.md, HBM: gfx950 reports half the bytes of wide
                # reads), both in KB; L2 <-> fabric bytes, Infinity-Cache hits included
                traffic = 2.0 * pmc["FETCH_SIZE"] * 1024.0 + pmc["WRITE_SIZE"] * 1024.0
                per_frame = traffic / fpl
                roof["traffic"] = round(traffic)
                roof["traffic_per_frame"] = round(per_frame)
                roof["pmc_launch"] = {"frames": fpl, "grid_size": grid,
                                      "fetch_bytes": round(2.0 * pmc["FETCH_SIZE"] * 1024.0),
                                      "write_bytes": round(pmc["WRITE_SIZE"] * 1024.0)}
                roof["achieved"] = round(per_frame / step_s / 1e9, 2)
                roof["frac"] = round(per_frame / step_s / 1e9 / HBM_PEAK_GBS, 5)
                roof["source"] = "PMC bytes of one timed-shape launch / frames / measured time per frame"
            if pmc and "SQ_INSTS_VALU" in pmc:
                valu_frame = pmc["SQ_INSTS_VALU"] / fpl
                roof["valu"] = {"bound": "valu-issue", "wave_insts_per_frame": round(valu_frame),
                                "achieved": round(valu_frame / step_s / 1e9, 1), "peak": round(VALU_ISSUE_PEAK / 1e9, 1),
                                "unit": "G wave-instr/s", "frac": round(valu_frame / step_s / VALU_ISSUE_PEAK, 4),
                                "wait_frac": round(pmc.get("SQ_WAIT_ANY", 0.0) / max(1.0, pmc.get("SQ_WAVE_CYCLES", 1.0)), 4),
                                "waves_per_frame": round(pmc.get("SQ_WAVES", 0.0) / fpl)}
            if pmc and "TCC_HIT_sum" in pmc:
                h, m = pmc["TCC_HIT_sum"], pmc.get("TCC_MISS_sum", 0.0)
                roof["l2_hit_rate"] = round(h / max(1.0, h + m), 4)
        out["roofline"] = roof
        out["prep"] = prep
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(asset, W, H, spp, bounces, use_tree, args.cpu_seconds)
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 2)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
