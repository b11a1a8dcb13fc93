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
