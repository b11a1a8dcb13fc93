"""Distributed path on CPU: world_size-2 gloo run of the shard plan + gather to rank 0. Each
rank 'renders' its packed slots with the CPU oracle, rank 0 reassembles the frame and it must
equal the single-process frame (pixel ownership is exact, every pixel once)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    from atray_amd.assets import CENTERS, asset_path
    from atray_amd.shard import ShardPlan, gather_packed, scatter_host
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H = 200, 120
    plan = ShardPlan(W, H, world, side=32)
    s = O.Scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    face, _, _ = s.primary_hits(O.Camera(W, H))
    m = plan.pixel_map(rank)
    assert len(m) == plan.sizes[rank]
    packed = torch.zeros(plan.max_size, dtype=torch.int64)
    packed[:len(m)] = torch.from_numpy(face.ravel()[m].astype(np.int64))
    lst = gather_packed(packed, plan, rank, dist)
    if rank == 0:
        img = scatter_host([t.numpy() for t in lst], plan)
        np.save(out_path, img)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_reassembles_frame(tmp_path):
    out = str(tmp_path / "img.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    img = np.load(out)
    from atray_amd.assets import CENTERS, asset_path
    from oracle import oracle as O
    s = O.Scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    face, _, _ = s.primary_hits(O.Camera(200, 120))
    assert np.array_equal(img.astype(np.uint32), face)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_plan_covers_each_pixel_once(world):
    from atray_amd.shard import ShardPlan
    plan = ShardPlan(1920, 1080, world, side=64)
    seen = np.zeros(1920 * 1080, np.int32)
    for r in range(world):
        np.add.at(seen, plan.pixel_map(r), 1)
    assert (seen == 1).all()
    assert sum(plan.sizes) == 1920 * 1080
    assert max(plan.sizes) - min(plan.sizes) <= 64 * 64


@pytest.mark.parametrize("world", [1, 2, 5, 8])
def test_balanced_plan_covers_each_pixel_once_and_balances(world):
    """Cost-balanced deal (atr_balance_shard_tiles): every pixel owned once, deterministic, and
    the longest-first bound: max load <= mean load + the largest tile cost."""
    from atray_amd import engine as E
    from atray_amd.shard import ShardPlan
    W, H, side = 1920, 1080, 64
    n = len(E.shard_grid(W, H, side))
    costs = np.random.default_rng(world).integers(1, 10**6, n) * (np.arange(n) % 7 == 0) + 1
    plan = ShardPlan.balanced(costs, W, H, world, side)
    again = ShardPlan.balanced(costs, W, H, world, side)
    assert np.array_equal(plan.owner, again.owner)
    seen = np.zeros(W * H, np.int32)
    for r in range(world):
        np.add.at(seen, plan.pixel_map(r), 1)
    assert (seen == 1).all()
    loads = np.array([costs[plan.owner == r].sum() for r in range(world)])
    assert loads.max() <= costs.sum() / world + costs.max()
    extra = ShardPlan.balanced(costs, W, H, world, side, rank0_extra=0.5)
    if world > 1:
        l0 = costs[extra.owner == 0].sum()
        assert l0 <= np.array([costs[extra.owner == r].sum() for r in range(world)]).max()


def _bench_worker(rank, world, port, out_path):
    """The bench's frame-assembly pipeline (double-buffered async gather, lagged scatter) on
    CPU tensors with the host scatter, fed by oracle hits: the assembled frames must equal the
    single-process frame for every step."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist

    from atray_amd import engine as E
    from atray_amd.assets import CENTERS, asset_path
    from atray_amd.shard import ShardPlan, assembly_index
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    W, H, side = 160, 96, 32
    s = O.Scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    face, _, _ = s.primary_hits(O.Camera(W, H))
    costs = np.where(np.arange(len(E.shard_grid(W, H, side))) % 3 == 0, 50, 1)
    plan = ShardPlan.balanced(costs, W, H, world, side, rank0_extra=0.1)
    m = plan.pixel_map(rank)
    packed = [torch.zeros(plan.max_size, dtype=torch.int64) for _ in range(2)]
    # as bench.py: gather into views of one [world x max_size] tensor, assemble with one
    # index_copy_ through the plan's assembly index (padding -> trash pixel W * H)
    big = [torch.zeros(world * plan.max_size, dtype=torch.int64) for _ in range(2)]
    gather = [[b[r * plan.max_size:(r + 1) * plan.max_size] for r in range(world)] for b in big]
    dst = torch.from_numpy(assembly_index(plan))
    pending, frames = {}, []

    def assemble(q):
        img = torch.zeros(W * H + 1, dtype=torch.int64)
        img.index_copy_(0, dst, big[q])
        return img[:W * H].numpy().reshape(H, W)

    for k in range(5):
        packed[k % 2].zero_()
        packed[k % 2][:len(m)] = torch.from_numpy(face.ravel()[m].astype(np.int64) + k)
        pending[k] = dist.gather(packed[k % 2], gather[k % 2] if rank == 0 else None, dst=0, async_op=True)
        if k - 1 in pending:
            pending.pop(k - 1).wait()
            if rank == 0:
                frames.append(assemble((k - 1) % 2))
    pending.pop(4).wait()
    if rank == 0:
        frames.append(assemble(0))
        np.save(out_path, np.stack(frames))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_pipelined_gather_reassembles_every_frame(tmp_path):
    out = str(tmp_path / "frames.npy")
    mp.spawn(_bench_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    frames = np.load(out)
    from atray_amd.assets import CENTERS, asset_path
    from oracle import oracle as O
    s = O.Scene(asset_path("Monkey"), center=CENTERS["Monkey"])
    face, _, _ = s.primary_hits(O.Camera(160, 96))
    assert len(frames) == 5
    for k in range(5):
        assert np.array_equal(frames[k], face.astype(np.int64) + k)


def test_bgr_pack_scatter_host_roundtrip():
    """The 3-byte exchange's host references (atr_pack_bgr / atr_scatter_bgr): BGRX pixels survive
    pack -> scatter through an assembly permutation, and a nonzero X byte is refused."""
    from atray_amd.shard import pack_bgr_host, scatter_bgr_host
    rng = np.random.default_rng(1)
    fb = rng.integers(0, 1 << 24, size=1000, dtype=np.uint32)
    p = pack_bgr_host(fb)
    assert p.dtype == np.uint8 and p.size == 3000
    assert list(p[:3]) == [fb[0] & 255, (fb[0] >> 8) & 255, (fb[0] >> 16) & 255]
    perm = rng.permutation(1000)
    img = np.zeros(1000, np.uint32)
    scatter_bgr_host(p, perm, img)
    assert np.array_equal(img[perm], fb)
    with pytest.raises(AssertionError):
        pack_bgr_host(np.array([1 << 24], np.uint32))


def test_assembly_share():
    """rank 0's assembly against a rank's render (bench.py's default rank0_extra): HBM-bound pack +
    scatter of the frame vs frame_ms / world; 0 without a measurement or at one rank."""
    from atray_amd.shard import assembly_share
    n = 1920 * 1080
    c3 = assembly_share(n, 0.34, 8)        # a 0.34-ms calibration frame over 8 ranks
    c4 = assembly_share(n, 69.0, 8)
    assert 0.1 < c3 < 0.2 and 0.0 < c4 < 0.001
    assert assembly_share(n, 0.0, 8) == 0.0 and assembly_share(n, 0.34, 1) == 0.0
    assert assembly_share(n, 1e-6, 8) == 0.5  # capped


def test_masked_stream_group_offsets():
    """The stream's group offsets (layout "ATRN", exchange.hip): word k of chunk c is the payload
    pixel index of pixel 64 k of the chunk -- the count of non-background pixels before it in the
    whole stream -- so a decoder reads a 64-pixel group's payload without a scan."""
    from atray_amd.shard import MASK_CHUNK, MASK_MAGIC, pack_bgr_masked_host
    rng = np.random.default_rng(11)
    for n in (1, 64, 8191, 8192, 20000):
        bg = 0x00123456
        fb = np.where(rng.random(n) < 0.3, rng.integers(0, 1 << 24, n), bg).astype(np.uint32)
        st = pack_bgr_masked_host(fb, bg)
        hdr = st[:16].view("<u4")
        nc = int(hdr[2])
        assert int(hdr[0]) == MASK_MAGIC and nc == -(-n // MASK_CHUNK)
        g0 = 16 + 4 * nc + 4 * nc * (MASK_CHUNK // 32)
        goff = st[g0:g0 + 4 * nc * (MASK_CHUNK // 64)].view("<u4")
        nb = np.zeros(nc * MASK_CHUNK, bool)
        nb[:n] = fb != bg
        want = np.concatenate([[0], np.cumsum(nb)])[::64][:nc * (MASK_CHUNK // 64)]
        assert np.array_equal(goff, want)


def test_masked_exchange_host_roundtrip():
    """The masked exchange's host references (atr_pack_bgr_masked / atr_scatter_bgr_masked): any
    background value, ragged chunk counts and empty input round-trip exactly, and the stream length
    is header + chunk offsets + 1 KB of mask and 512 B of group offsets per 8192-pixel chunk + 3 B
    per non-background pixel."""
    from atray_amd.shard import pack_bgr_masked_host, scatter_bgr_masked_host, background_value
    rng = np.random.default_rng(7)
    for n in (0, 1, 63, 64, 65, 8191, 8192, 8193, 70001):
        bg = 0x007F664C
        fb = np.where(rng.random(n) < 0.15, rng.integers(0, 1 << 24, n), bg).astype(np.uint32)
        for b in (bg, background_value(fb), 0x01000000):
            st = pack_bgr_masked_host(fb, b)
            nc = -(-n // 8192)
            assert st.size == 16 + 4 * nc + 1024 * nc + 512 * nc + 3 * int((fb != b).sum())
            perm = rng.permutation(n)
            img = np.zeros(n, np.uint32)
            scatter_bgr_masked_host(st, n, perm, img)
            assert np.array_equal(img[perm], fb)
