"""Benchmark: Mrays/s of the render path on Dragon 1920x1080 (BASELINE.json metric, config 3).

python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3] [--variant auto|lane|wave]

One step = one frame of the config rendered by all ranks: each rank traces its 64x64 shard tiles
into a packed buffer; for N > 1 the packed buffers are gathered to rank 0 over RCCL
(torch.distributed "nccl", async, double-buffered: frame k's gather overlaps frame k+1's render)
and scattered into the frame there. Tiles are dealt longest-first by cost measured in one
calibration render on rank 0 (--plan cost, default; --plan rr = round-robin). The scene
(OBJ load, octree build, upload) and the plan are prepared before timing; inputs are resident
in HBM when the timed region starts. value = traced rays of all ranks / max-over-ranks wall
time. ATR_DIST_BACKEND=gloo rehearses N ranks on one GPU (host-staged gather).

Extra JSON fields: roofline (render kernel: algorithmic bytes per launch / average launch time
from HIP events on the launch stream, against 8 TB/s; traffic = HBM bytes per launch from a
rocprofv3 --pmc child run, FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE, separate passes),
cpu_baseline (the C oracle, i.e. the reference algorithm restated, on the host cores of the
same box, reference tile scheduler).
"""
import argparse
import csv
import glob
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


SEED = 0x853C49E6748FEA9B
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# config -> (asset, W, H, spp, bounces, use_tree)  (BASELINE.json configs)
CONFIGS = {
    "c1": ("Cube", 256, 256, 1, 1, True),
    "c2": ("Monkey", 1280, 720, 1, 1, False),
    "c3": ("Dragon", 1920, 1080, 1, 1, True),
    "c4": ("Dragon", 1920, 1080, 64, 5, True),
    "c5": ("Dragon", 3840, 2160, 256, 5, True),
}
GOLDEN_COUNTERS = {"c3": "dragon_1920x1080_tree", "c2": "monkey_1280x720_bf", "c1": "cube_256_tree"}


def algorithmic_bytes_per_ray(ctr):
    """B = 24 (ray) + 12 (hit out) + 28 N_box + 40 N_tri + 8 N_leaf per ray,
    N_* = the reference's own per-ray work on this input (golden counters, tools/make_goldens.py)."""
    n = ctr["n_rays"]
    return (36.0 + 28.0 * ctr["n_box"] / n + 40.0 * ctr["n_tri"] / n + 8.0 * ctr["n_leaf"] / n)


def cluster_bytes_per_ray(ctr):
    """The clustered kernel's own algorithmic bytes per ray, in its own data layout (DESIGN.md
    §6): ray in + hit out (36); one 48-B inner-node record per visit, shared by the 8 child boxes
    it tests (6 per box test, re-walks included); 8 per leaf range; 32 per cluster record; the
    screen's 6 (three f16) per screened primitive; a, ab, ac (36) per full triangle test. N_*
    counted live by the instrumented build of the same kernel on the same frame."""
    n = ctr["n_rays"]
    return (36.0 + 6.0 * ctr["box_all"] / n + 8.0 * ctr["n_leaf"] / n + 32.0 * ctr["cluster_boxes"] / n
            + 6.0 * ctr["screened"] / n + 36.0 * ctr["n_tri"] / n)


def pmc_traffic(args, kernel_name="render_kernel"):
    """HBM bytes per render launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) of a
    short child run of this benchmark. FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: gfx950
    reports half the bytes of wide reads); both counters are in KB."""
    exe = "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, "rocprofv3 missing"
    out = {}
    for ctr in ["FETCH_SIZE", "WRITE_SIZE"]:
        d = os.path.join(ROOT, "gpurun_out", f"pmc_{ctr.lower()}")
        os.makedirs(d, exist_ok=True)
        cmd = [exe, "--pmc", ctr, "--kernel-trace", "--output-format", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1",
               "--frames-per-launch", "1", "--streams", "1",
               "--config", args.config, "--variant", args.variant, "--no-cpu-baseline", "--no-pmc"]
        env = dict(os.environ)
        env.pop("RANK", None)
        env.pop("WORLD_SIZE", None)
        try:
            subprocess.run(cmd, check=True, timeout=300, env=env, stdout=subprocess.DEVNULL,
                           stderr=subprocess.DEVNULL)
        except Exception as e:  # noqa: BLE001
            return None, f"rocprofv3 {ctr} failed: {e}"
        vals = []
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    name = row.get("Kernel_Name", "")
                    # one-frame launches of the product kernel (not the instrumented COUNT build)
                    if kernel_name in name and not re.search(r"render_kernel<\d+, true", name) \
                            and row.get("Counter_Name") == ctr:
                        vals.append(float(row["Counter_Value"]))
        if not vals:
            return None, f"no {ctr} rows"
        out[ctr] = sum(vals) / len(vals)
    return 2.0 * out["FETCH_SIZE"] * 1024.0 + out["WRITE_SIZE"] * 1024.0, "ok"


def cpu_baseline(asset, W, H, spp, bounces, use_tree, seconds):
    """The reference algorithm (C oracle restatement) on this host: reference tile scheduler
    (renderer.cpp:403-455) on `threads` pthreads, whole frames until `seconds` elapse."""
    from atray_amd.assets import CENTERS, asset_path
    from oracle import oracle as O
    threads = max(1, min(16, os.cpu_count() or 1))
    s = O.Scene(asset_path(asset), center=CENTERS[asset], use_tree=use_tree)
    cam = O.Camera(W, H, spp=spp, bounces=bounces)
    frames, secs = 0, 0.0
    while secs < seconds or frames == 0:
        dt, _, _, _ = s.render_threaded(cam, SEED, threads)
        secs += dt
        frames += 1
    rays = frames * W * H * spp  # traced primary rays; 1 ray per pixel-sample at bounce_limit 1
    return {"value": rays / secs / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{frames} full {asset} {W}x{H} frames spp={spp} bounces={bounces}, "
                      f"reference tile scheduler ({W // threads}px tiles), {secs:.1f}s of render time"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=48)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--variant", default="auto", choices=["auto", "lane", "wave", "tile", "tile8", "wf", "cl", "ps"])
    ap.add_argument("--side", type=int, default=64, help="shard tile side (pixels)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--streams", type=int, default=2,
                    help="launches in flight (one HIP stream each)")
    ap.add_argument("--frames-per-launch", type=int, default=8,
                    help="frames rendered by one launch (atr_render_start_frames); 1 = one frame per launch")
    ap.add_argument("--plan", default="cost", choices=["cost", "rr"],
                    help="N>1 tile deal: measured-cost longest-first (default) or round-robin")
    ap.add_argument("--rank0-extra", type=float, default=0.05,
                    help="rank 0's frame-assembly share, as a fraction of the mean per-rank load")
    ap.add_argument("--check", action="store_true",
                    help="rank 0: compare the assembled frame with a one-launch full-frame render")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES floor for this process (0 = leave the environment alone)")
    args = ap.parse_args()
    # Frames in flight run on separate HIP streams; HIP maps a process's streams onto
    # GPU_MAX_HW_QUEUES hardware queues (default 4, shared with RCCL's streams), and streams on
    # one queue serialize. Read at HIP initialization, so set before torch loads.
    if args.hw_queues and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < args.hw_queues:
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)

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
    variant = {"auto": E.ATR_KERNEL_AUTO, "lane": E.ATR_KERNEL_LANE, "wave": E.ATR_KERNEL_WAVE,
               "tile": E.ATR_KERNEL_TILE, "tile8": E.ATR_KERNEL_TILE8,
               "wf": E.ATR_KERNEL_WAVEFRONT, "cl": E.ATR_KERNEL_CLUSTER,
               "ps": E.ATR_KERNEL_PERSIST}[args.variant]
    mesh = E.Mesh.load_obj(asset_path(asset))
    box = mesh.translate_to(mesh.aabb(), CENTERS[asset])
    tree = E.Octree.build(mesh, 300) if use_tree else None
    eng = E.Engine(local % ndev)
    eng.upload([((0.3, 0.4, 0.5), (0.2, 0.3, 0.4), 0.3), ((0.4, 0.2, 0.2), (0.92, 0.5, 0.0), 0.3)],
               [(mesh, tree, box, 1)])
    cam = E.camera(W, H, spp, bounces)
    stream = torch.cuda.current_stream(dev).cuda_stream

    # shard plan (scene prep, untimed): one calibration render measures every grid tile's cost
    # on rank 0, broadcast so all ranks derive the same longest-first deal
    if world > 1 and args.plan == "cost":
        costs = S.tile_costs(eng, cam, W, H, args.side, SEED) if rank == 0 else np.zeros(
            len(E.shard_grid(W, H, args.side)), np.int64)
        costs = S.shared_costs(costs, rank, dist, dev if backend == "nccl" else "cpu")
        plan = S.ShardPlan.balanced(costs, W, H, world, args.side, args.rank0_extra)
    else:
        plan = S.ShardPlan(W, H, world, args.side)
    sizes, maxn = plan.sizes, plan.max_size
    tiles = E.tiles_array(plan.tiles[rank])
    # Frames in flight: launch j renders frames jF .. jF+F-1 (F = --frames-per-launch, one grid:
    # a frame's slow cells overlap the other frames') on stream j % S (S = --streams, output
    # buffers per stream); for N > 1 the launch's F packed frames are gathered to rank 0 in ONE
    # gather on that stream and assembled there with ONE index_copy_ while later launches run.
    S_, F_ = max(1, args.streams), max(1, args.frames_per_launch)
    # frame slots on streams of their own (not the null stream, which HIP orders against the
    # process's blocking streams)
    streams = [torch.cuda.Stream(dev) for _ in range(S_)]
    npf = W * H if world == 1 else maxn  # output elements per frame (stride between frames)
    outbuf = [torch.zeros(F_ * npf, dtype=torch.int32, device=dev) for _ in range(S_)]
    on_host = world > 1 and backend != "nccl"
    images = None
    if world == 1:
        images = [outbuf[q][f * npf:(f + 1) * npf] for q in range(S_) for f in range(F_)]
    elif rank == 0:
        # per stream slot: every rank's F packed frames [world x F x maxn]; one index_copy_ through
        # the plan's assembly index (padding -> a trash pixel past each frame) writes F images
        big = [torch.zeros(world * F_ * maxn, dtype=torch.int32, device="cpu" if on_host else dev)
               for _ in range(S_)]
        gather = [[b_[r * F_ * maxn:(r + 1) * F_ * maxn] for r in range(world)] for b_ in big]
        one = S.assembly_index(plan).reshape(world, 1, maxn)
        dst_all = one + (np.arange(F_, dtype=np.int64) * (W * H + 1)).reshape(1, F_, 1)
        dst_idx = torch.from_numpy(np.ascontiguousarray(dst_all).ravel()).to(dev)
        images_ext = [torch.zeros(F_ * (W * H + 1), dtype=torch.int32, device=dev) for _ in range(S_)]
        images = [im[f * (W * H + 1):f * (W * H + 1) + W * H] for im in images_ext for f in range(F_)]
        staging = torch.zeros(world * F_ * maxn, dtype=torch.int32, device=dev) if on_host else None
    traced = torch.zeros(1, dtype=torch.int64, device=dev)
    layout = E.ATR_LAYOUT_IMAGE if world == 1 else E.ATR_LAYOUT_PACKED
    frames = [E.atr_frame(layout, outbuf[q].data_ptr(), None, None, None, None, None) for q in range(S_)]
    pending = {}

    def assemble(j):
        """Launch j's gather done (its stream waits on it); rank 0 scatters every rank's packed
        frames into that slot's images, on the launch's stream."""
        q = j % S_
        work = pending.pop(j)
        with torch.cuda.stream(streams[q]):
            if work is not None:
                work.wait()
            if rank == 0:
                src = big[q]
                if on_host:
                    staging.copy_(src, non_blocking=False)
                    src = staging
                images_ext[q].index_copy_(0, dst_idx, src)

    def launch(j, nf, fr=None):
        q = j % S_
        if j - S_ in pending:
            assemble(j - S_)  # before this slot's buffers are reused
        eng.render_start_frames(cam, tiles, fr or frames[q], nf, npf, SEED, stream=streams[q].cuda_stream,
                                variant=variant)
        if world == 1:
            return
        with torch.cuda.stream(streams[q]):
            buf = outbuf[q]
            if on_host:
                torch.cuda.synchronize()
                buf = buf.cpu()
            pending[j] = dist.gather(buf, gather[q] if rank == 0 else None, dst=0, async_op=True)

    def run_steps(n):
        for j in range((n + F_ - 1) // F_):
            launch(j, min(F_, n - j * F_))
        for j in sorted(pending):
            assemble(j)

    torch.cuda.synchronize()  # buffers were zero-filled on the current stream
    # rays per frame (all ranks): counted by the kernel (every get_intersection_data call)
    launch(0, 1, E.atr_frame(layout, outbuf[0].data_ptr(), None, None, None, None, traced.data_ptr()))
    for j in sorted(pending):
        assemble(j)
    torch.cuda.synchronize()
    rays_t = traced.clone() if backend == "nccl" or world == 1 else traced.cpu()
    if world > 1:
        dist.all_reduce(rays_t)
    rays_per_step = int(rays_t.item())

    run_steps(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run_steps(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    # roofline: the render kernel's own average duration, launches serialized on one stream
    # (HIP events on that stream; rocprofv3 of `bench.py --streams 1` reports the same kernel)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
    for a, b in evs:
        a.record(streams[0])
        eng.render_start(cam, tiles, frames[0], SEED, stream=streams[0].cuda_stream, variant=variant)
        b.record(streams[0])
    torch.cuda.synchronize()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    rc, _ = eng.wait()
    assert rc == 0
    # the dominant kernel's work on this rank's tiles, counted by the instrumented build of the
    # same variant (untimed; deterministic)
    live_ctr = eng.counters(cam, tiles, SEED, variant) if rank == 0 else None
    check = None
    if args.check and rank == 0:
        ref = torch.zeros(W * H, dtype=torch.int32, device=dev)
        fr = E.atr_frame(E.ATR_LAYOUT_IMAGE, ref.data_ptr(), None, None, None, None, None)
        eng.render_start(cam, [[0, 0, W - 1, H - 1]], fr, SEED, stream=stream)
        torch.cuda.synchronize()
        # images holding a frame: stream slot j % S, position f of launch j
        used = sorted({((k // F_) % S_) * F_ + k % F_ for k in range(max(args.steps, args.warmup))})
        check = sum(int((ref != images[q]).sum().item()) for q in used)

    if rank == 0:
        value = rays_per_step * args.steps / elapsed / 1e6
        out = {"metric": "Mrays/sec on Dragon.obj 1920x1080 @ 1/2/4/8 GPU; % HBM roofline",
               "value": round(value, 3), "unit": "Mrays/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
               "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic: the survey's Dragon surrogate (Dragon.obj absent), app camera/materials",
               "config": {"workload": f"{args.config}: {asset} {W}x{H} spp={spp} bounces={bounces} "
                                      f"{'octree' if use_tree else 'brute-force'}",
                          "rays_per_step": rays_per_step, "shard_tile": args.side,
                          "parallelism": f"tiles{world}", "kernel": args.variant,
                          "plan": args.plan if world > 1 else "single",
                          "frames_in_flight": args.streams * args.frames_per_launch,
                          "streams": args.streams, "frames_per_launch": args.frames_per_launch,
                          "shard_pixels": [int(x) for x in sizes]}}
        if check is not None:
            out["check_mismatched_pixels"] = check
        roof = {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None, "kernel_ms": round(kern_ms, 4)}
        clustered = args.variant in ("auto", "cl", "ps")
        if clustered:
            bpr = cluster_bytes_per_ray(live_ctr)
        else:
            bpr = algorithmic_bytes_per_ray(live_ctr)
        achieved = bpr * live_ctr["n_rays"] / (kern_ms * 1e-3) / 1e9
        roof.update({"achieved": round(achieved, 1), "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "bytes_per_ray": round(bpr, 1), "rays_per_launch": live_ctr["n_rays"],
                     "model": "clustered scan, own work (DESIGN.md 6)" if clustered
                     else "reference work (SURVEY.md 8(d))"})
        gname = GOLDEN_COUNTERS.get(args.config)
        if gname:  # the reference algorithm's bytes for the same rays, at this kernel's speed
            with open(os.path.join(ROOT, "tests", "golden", "goldens.json")) as f:
                ctr = json.load(f)["hits"][gname]["counters"]
            rbpr = algorithmic_bytes_per_ray(ctr)
            roof["ref_bytes_per_ray"] = round(rbpr, 1)
            roof["ref_equivalent_GBs"] = round(rbpr * live_ctr["n_rays"] / (kern_ms * 1e-3) / 1e9, 1)
        if world == 1 and not args.no_pmc:
            traffic, why = pmc_traffic(args)
            roof["traffic"] = traffic
            roof["traffic_note"] = why
        out["roofline"] = roof
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(asset, W, H, spp, bounces, use_tree, args.cpu_seconds)
            out["speedup_vs_cpu"] = round(value / out["cpu_baseline"]["value"], 2)
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
