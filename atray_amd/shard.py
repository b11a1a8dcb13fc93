"""Image sharding across ranks (one process per GPU) and the frame gather to rank 0.

Pixels are independent given the replicated read-only scene, so the frame is
split into square shard tiles dealt round-robin to ranks (interleaved: per-tile cost varies
~3.4x across the reference demo's tiles, centre >> edge). Each rank traces its tiles into a
packed buffer (every owned pixel once, tile order); the one exchange step is a gather of the
packed buffers to rank 0 (RCCL over xGMI for backend "nccl"; gloo in the CPU tests), where
they are scattered into the image. Each pixel's spp/bounce loop stays on one rank, so the
result is bit-identical to a single-GPU render.
"""
from __future__ import annotations

import numpy as np

from . import engine as E


class ShardPlan:
    """Which side x side tiles each rank traces. Default: round-robin deal of the row-major grid
    (atr_make_shard_tiles). With `owner` (one rank per grid tile, e.g. from `balanced`): that
    assignment, each rank's tiles kept in grid order."""

    def __init__(self, width: int, height: int, world: int, side: int = 64, owner=None):
        self.width, self.height, self.world, self.side = width, height, world, side
        if owner is None:
            self.tiles = [E.make_shard_tiles(width, height, side, r, world) for r in range(world)]
        else:
            grid = E.shard_grid(width, height, side)
            owner = np.asarray(owner, np.int32)
            assert len(owner) == len(grid) and owner.min() >= 0 and owner.max() < world
            self.tiles = [grid[owner == r] for r in range(world)]
        self.owner = owner
        self.sizes = [E.packed_size(t) if len(t) else 0 for t in self.tiles]
        self.max_size = max(1, max(self.sizes))

    @classmethod
    def balanced(cls, costs, width: int, height: int, world: int, side: int = 64, rank0_extra: float = 0.0):
        """Longest-first deal by measured per-tile cost (`tile_costs`); rank 0 starts with
        rank0_extra x the mean per-rank load (its frame assembly)."""
        costs = np.asarray(costs, np.int64)
        extra = int(rank0_extra * costs.sum() / max(1, world))
        return cls(width, height, world, side, E.balance_shard_tiles(width, height, side, world, costs, extra))

    def pixel_map(self, rank: int) -> np.ndarray:
        return E.packed_pixel_map(self.tiles[rank], self.width, self.height)


def assembly_index(plan: ShardPlan) -> np.ndarray:
    """Destination pixel of every slot of the gathered [world x max_size] buffer (rank r's packed
    pixels at r * max_size); padding slots point at a trash pixel width * height just past the
    image, so the whole frame assembles with one index_copy_ into a (W * H + 1) buffer."""
    n = plan.world * plan.max_size
    dst = np.full(n, plan.width * plan.height, np.int64)
    for r in range(plan.world):
        m = plan.pixel_map(r) if len(plan.tiles[r]) else np.zeros(0, np.int64)
        dst[r * plan.max_size:r * plan.max_size + len(m)] = m
    return dst


def tile_costs(eng, cam, width: int, height: int, side: int, seed: int) -> np.ndarray:
    """Measured cost (GPU shader clocks) of every grid tile: one calibration render."""
    return eng.tile_costs(cam, E.shard_grid(width, height, side), seed)


def shared_costs(costs, rank: int, dist, device):
    """Rank 0's measured costs on every rank (timings differ per GPU; the plan must not)."""
    import torch
    t = torch.as_tensor(np.asarray(costs, np.int64), device=device)
    dist.broadcast(t, src=0)
    return t.cpu().numpy()


def gather_packed(packed, plan: ShardPlan, rank: int, dist, group=None):
    """Gather every rank's packed buffer (padded to plan.max_size) to rank 0; returns the list
    of per-rank buffers on rank 0, None elsewhere. `packed` is a torch tensor."""
    import torch
    assert packed.numel() == plan.max_size, (packed.numel(), plan.max_size)
    lst = [torch.empty_like(packed) for _ in range(plan.world)] if rank == 0 else None
    dist.gather(packed, lst, dst=0, group=group)
    return lst


def scatter_host(bufs, plan: ShardPlan) -> np.ndarray:
    """Host-side reassembly of gathered packed buffers (the GPU path uses atr_unpack)."""
    img = np.zeros(plan.width * plan.height, dtype=np.asarray(bufs[0]).dtype)
    for r, b in enumerate(bufs):
        m = plan.pixel_map(r)
        img[m] = np.asarray(b)[:len(m)]
    return img.reshape(plan.height, plan.width)
