"""Image sharding across ranks (one process per GPU) and the frame gather to rank 0.

Pixels are independent given the replicated read-only scene, so the frame is
split into square shard tiles dealt to ranks (longest-first by measured cost, or round-robin:
per-tile cost varies ~3.4x across the reference demo's tiles, centre >> edge). Each rank traces
its tiles into a packed buffer (every owned pixel once, tile order); the one exchange step is
an exact-size gather of the packed framebuffers to rank 0 (`gather_frames`: RCCL send/recv over
xGMI for backend "nccl"; gloo in the CPU tests), where they are scattered into the image, plus
a reduction of the per-tile ray_casts sums (a few KB). Each pixel's spp/bounce loop stays on
one rank, so the result is bit-identical to a single-GPU render.
"""
from __future__ import annotations

import numpy as np

from . import engine as E


class ShardPlan:
    """Which side x side tiles each rank traces. Default: round-robin deal of the row-major grid
    (atr_make_shard_tiles). With `owner` (one rank per grid tile, e.g. from `balanced`): that
    assignment, each rank's tiles kept in grid order."""

    def __init__(self, width: int, height: int, world: int, side: int = 64, owner=None, costs=None):
        self.width, self.height, self.world, self.side = width, height, world, side
        if owner is None and costs is None:
            self.tiles = [E.make_shard_tiles(width, height, side, r, world) for r in range(world)]
        else:
            grid = E.shard_grid(width, height, side)
            if owner is None:
                owner = np.arange(len(grid)) % world
            owner = np.asarray(owner, np.int32)
            assert len(owner) == len(grid) and owner.min() >= 0 and owner.max() < world
            idx = np.arange(len(grid))
            if costs is not None:  # each rank's tiles heaviest first: a launch starts its slowest cells
                idx = np.argsort(-np.asarray(costs, np.int64), kind="stable")  # first, so they do not form its tail
            self.tiles = [grid[idx[owner[idx] == r]] for r in range(world)]
        self.owner = owner
        self.sizes = [E.packed_size(t) if len(t) else 0 for t in self.tiles]
        self.max_size = max(1, max(self.sizes))

    @classmethod
    def balanced(cls, costs, width: int, height: int, world: int, side: int = 64, rank0_extra: float = 0.0,
                 heavy_first: bool = True):
        """Longest-first deal by measured per-tile cost (`tile_costs`); rank 0 starts with
        rank0_extra x the mean per-rank load (its frame assembly). heavy_first: each rank's tiles
        in descending cost (else grid order)."""
        costs = np.asarray(costs, np.int64)
        extra = int(rank0_extra * costs.sum() / max(1, world))
        owner = E.balance_shard_tiles(width, height, side, world, costs, extra)
        return cls(width, height, world, side, owner, costs if heavy_first else None)

    @classmethod
    def curve(cls, costs, width: int, height: int, world: int, side: int = 64, rank0_extra: float = 0.0,
              heavy_first: bool = True):
        """Compact shards by recursive cost bisection: a group of ranks' tiles are cut across their
        bounding box's longer side (tiles in column-major order for a vertical cut, row-major for a
        horizontal one) where the first half of the ranks' share of the measured cost is reached,
        each half recursing on its ranks; rank 0's share is short by rank0_extra x the mean load.
        Each rank's tiles form a near-rectangle (one step at the cut), so its rays walk a compact
        part of the scene (its caches hold less of the tree than under the longest-first deal,
        whose tiles spread over the frame); the balance is within about one tile's cost per cut."""
        costs = np.asarray(costs, np.int64)
        grid = E.shard_grid(width, height, side)
        total = float(costs.sum())
        extra = rank0_extra * total / max(1, world)
        want = np.full(world, (total + extra) / max(1, world))
        want[0] -= extra
        owner = np.zeros(len(grid), np.int32)

        def cut(idx, r0, r1):
            if r1 - r0 == 1 or len(idx) == 0:
                owner[idx] = r0
                return
            m = (r0 + r1) // 2
            x, y = grid[idx, 0], grid[idx, 1]
            vertical = (x.max() - x.min()) >= (y.max() - y.min())
            o = idx[np.lexsort((y, x) if vertical else (x, y))]
            cum = np.cumsum(costs[o].astype(np.float64))
            frac = want[r0:m].sum() / max(1e-30, want[r0:r1].sum())
            k = int(np.searchsorted(cum, frac * cum[-1], side="left"))
            if k < len(cum) and (k == 0 or abs(cum[k] - frac * cum[-1]) < abs(cum[k - 1] - frac * cum[-1])):
                k += 1  # the nearer of the tile boundaries around the target
            cut(o[:k], r0, m)
            cut(o[k:], m, r1)

        cut(np.arange(len(grid)), 0, world)
        return cls(width, height, world, side, owner, costs if heavy_first else None)

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


def assembly_share(npixels: int, frame_ms: float, world: int, hbm_tbs: float = 5.0) -> float:
    """Rank 0's frame assembly as a fraction of one rank's render of a frame (the plan's
    rank0_extra): packing (4 B read, 3 written per pixel of its own shard) and the scatter of the
    whole frame (3 B read, 8 B of index, 4 B written per pixel), HBM-bound at `hbm_tbs`, against
    frame_ms / world of render (frame_ms: a calibration render of the whole frame). 0 without a
    measurement. c3 at 8 ranks: ~0.1; c4: ~0.0003."""
    if frame_ms <= 0.0 or world <= 1:
        return 0.0
    asm_ms = npixels * (7.0 / world + 15.0) / (hbm_tbs * 1e12) * 1e3
    return min(0.5, asm_ms / (frame_ms / world))


def tile_costs(eng, cam, width: int, height: int, side: int, seed: int) -> np.ndarray:
    """Measured cost (GPU shader clocks) of every grid tile: one calibration render."""
    return eng.tile_costs(cam, E.shard_grid(width, height, side), seed)


GRADE_BOUNDS = (0.02, 0.05, 0.10, 0.20, 0.30, 0.50, 0.75)  # cumulative fractions, heaviest first


def graded_cell_plan(cell_costs, prio_frac: float = 0.0) -> np.ndarray:
    """atr_set_cell_plan bytes that dispatch cells by measured cost, heaviest class first: class 7
    (bits 4-6) for the top 2 % of the cells that cost anything, 6 for the next to 5 %, ..., 0 for the
    rest (the single-frame plan's fractions, plan.hip); prio_frac: the heaviest cells' waves also
    issue at raised priority (ATR_PLAN_PRIO, 0x80). Scheduling only: outputs never change."""
    cc = np.asarray(cell_costs).ravel()
    order = np.argsort(-cc, kind="stable")
    live = int((cc > 0).sum())
    crank = np.empty(cc.size, np.int64)
    crank[order] = np.arange(cc.size)
    cls = np.zeros(cc.size, np.uint8)
    for k, f in enumerate(GRADE_BOUNDS):
        cls[crank >= int(round(f * live))] = 6 - k
    cls[crank < int(round(GRADE_BOUNDS[0] * live))] = 7
    plan = (cls << 4).astype(np.uint8)
    if prio_frac > 0:
        plan[crank < int(round(prio_frac * live))] |= 0x80
    return plan


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


def frame_offsets(plan: ShardPlan, nframes: int) -> list:
    """Start of rank r's block in the exact gather buffer: every rank's F packed frames back to
    back, rank after rank (F x size_r elements each, no padding)."""
    off = np.concatenate([[0], np.cumsum(np.asarray(plan.sizes, np.int64) * nframes)])
    return [int(x) for x in off]


def frames_assembly_index(plan: ShardPlan, nframes: int) -> np.ndarray:
    """Destination of every element of the exact gather buffer (frame_offsets) in nframes images
    of width x height: element i of rank r's frame f goes to f * W * H + pixel_map(r)[i]. The
    shard tiles partition the image, so the buffer is exactly nframes * W * H long and one
    index_copy_ assembles a whole launch."""
    npx = plan.width * plan.height
    parts = []
    for r in range(plan.world):
        if plan.sizes[r] == 0:
            continue
        m = plan.pixel_map(r).astype(np.int64)
        parts.append((np.arange(nframes, dtype=np.int64)[:, None] * npx + m[None, :]).ravel())
    out = np.concatenate(parts)
    assert out.size == nframes * npx
    return out


def slot_tiles(plan: ShardPlan, rank: int) -> np.ndarray:
    """Shard-grid tile (row-major index in shard_grid order) of every packed slot of `rank`: the
    per-tile ray_casts sums (the reference's per-tile counters, renderer.cpp:465-468) are
    index_add_ reductions over it."""
    if plan.sizes[rank] == 0:
        return np.zeros(0, np.int64)
    m = plan.pixel_map(rank).astype(np.int64)
    ntx = -(-plan.width // plan.side)
    return (m // plan.width // plan.side) * ntx + (m % plan.width) // plan.side


def tile_ids(plan: ShardPlan, rank: int) -> np.ndarray:
    """Shard-grid index of each of `rank`'s tiles, in its tile-list order."""
    t = np.asarray(plan.tiles[rank]).reshape(-1, 4).astype(np.int64)
    ntx = -(-plan.width // plan.side)
    return (t[:, 1] // plan.side) * ntx + t[:, 0] // plan.side


def pixel_tiles(width: int, height: int, side: int) -> np.ndarray:
    """Shard-grid tile of every pixel of an IMAGE-layout frame (y * width + x)."""
    ntx = -(-width // side)
    y, x = np.divmod(np.arange(width * height, dtype=np.int64), width)
    return (y // side) * ntx + x // side


def grid_tile_count(plan: ShardPlan) -> int:
    return (-(-plan.width // plan.side)) * (-(-plan.height // plan.side))


def gather_frames(send, recv, plan: ShardPlan, rank: int, nframes: int, dist, unit: int = 1):
    """Exact-size gather of nframes packed frames to rank 0 (the one exchange step: RCCL send/recv
    over xGMI for backend "nccl"). `send`: this rank's frames back to back (nframes x size_r
    pixels; rank 0's own block is written in place by its render). `recv` (rank 0): the exact
    gather buffer (frame_offsets with the launch's frame capacity F). `unit`: elements per pixel
    (1: u32 BGRX; 3: the 3-byte BGR exchange, u8 tensors). Returns the async works."""
    ops = []
    if rank == 0:
        off = frame_offsets(plan, recv.numel() // (unit * plan.width * plan.height))
        for r in range(1, plan.world):
            n = plan.sizes[r] * nframes * unit
            if n:
                ops.append(dist.P2POp(dist.irecv, recv[unit * off[r]:unit * off[r] + n], r))
    elif plan.sizes[rank]:
        ops.append(dist.P2POp(dist.isend, send[:plan.sizes[rank] * nframes * unit], 0))
    return dist.batch_isend_irecv(ops) if ops else []


def gather_sizes(nbytes, sizes, plan: ShardPlan, rank: int, dist):
    """Phase 1 of the masked exchange: every rank's stream length (a (1,) int64 tensor) into rank 0's
    `sizes` (world,) at index r. Ranks without pixels send nothing. Returns the async works."""
    ops = []
    if rank == 0:
        for r in range(1, plan.world):
            if plan.sizes[r]:
                ops.append(dist.P2POp(dist.irecv, sizes[r:r + 1], r))
    elif plan.sizes[rank]:
        ops.append(dist.P2POp(dist.isend, nbytes, 0))
    return dist.batch_isend_irecv(ops) if ops else []


def gather_streams(send, recv, roff, sizes, plan: ShardPlan, rank: int, dist):
    """Phase 2 of the masked exchange: the exact streams to rank 0 (rank r's into recv[roff[r]:],
    sizes[r] bytes, u8 tensors). `send` (other ranks): this rank's stream, exactly its length."""
    ops = []
    if rank == 0:
        for r in range(1, plan.world):
            if plan.sizes[r] and sizes[r]:
                ops.append(dist.P2POp(dist.irecv, recv[int(roff[r]):int(roff[r]) + int(sizes[r])], r))
    elif plan.sizes[rank] and send.numel():
        ops.append(dist.P2POp(dist.isend, send, 0))
    return dist.batch_isend_irecv(ops) if ops else []


def pack_bgr_host(fb) -> np.ndarray:
    """Host reference of atr_pack_bgr: BGRX u32 pixels -> 3 bytes each (B, G, R); the X byte must
    be 0 (texture.h:27-38), so nothing is lost."""
    b = np.ascontiguousarray(np.asarray(fb, np.uint32)).view(np.uint8).reshape(-1, 4)
    assert not b[:, 3].any(), "BGRX framebuffer with a nonzero X byte"
    return np.ascontiguousarray(b[:, :3]).reshape(-1)


def scatter_bgr_host(packed, dst_index, image) -> None:
    """Host reference of atr_scatter_bgr: image[dst_index[i]] = B | G << 8 | R << 16."""
    p = np.asarray(packed, np.uint8).reshape(-1, 3).astype(np.uint32)
    image[np.asarray(dst_index, np.int64)] = p[:, 0] | (p[:, 1] << 8) | (p[:, 2] << 16)


MASK_CHUNK = 8192  # pixels per chunk of the masked stream (exchange.hip)
MASK_MAGIC = 0x4E525441  # "ATRN": the masked stream layout with group offsets (exchange.hip)


def background_value(fb) -> int:
    """The most common BGRX value of a frame (the masked exchange's background: a c3 frame's sky).
    Any value gives a correct stream; the common one gives the shortest."""
    v, c = np.unique(np.asarray(fb, np.uint32), return_counts=True)
    return int(v[np.argmax(c)]) if v.size else 0


def pack_bgr_masked_host(fb, background: int) -> np.ndarray:
    """Host reference of atr_pack_bgr_masked: the same bytes as the device stream (header, chunk
    offsets, mask words, group offsets, B, G, R of every pixel != background)."""
    fb = np.ascontiguousarray(np.asarray(fb, np.uint32))
    n = fb.size
    nc = -(-n // MASK_CHUNK)
    nb = np.zeros(nc * MASK_CHUNK, bool)
    nb[:n] = fb != np.uint32(background)
    words = np.packbits(nb.reshape(-1, 32)[:, ::-1], axis=1).view(">u4").ravel().astype("<u4")
    counts = nb.reshape(nc, MASK_CHUNK).sum(1) if nc else np.zeros(0, np.int64)
    off = (np.cumsum(counts) - counts).astype("<u4")
    gcounts = nb.reshape(-1, 64).sum(1)  # every 64-pixel group's payload pixels
    goff = (np.cumsum(gcounts) - gcounts).astype("<u4")
    total = int(counts.sum())
    hdr = np.array([MASK_MAGIC, int(background) & 0xFFFFFFFF, nc, total], "<u4")
    pay = pack_bgr_host(fb[nb[:n]]) if total else np.zeros(0, np.uint8)
    return np.concatenate([hdr.view(np.uint8), off.view(np.uint8), words.view(np.uint8), goff.view(np.uint8), pay])


def scatter_bgr_masked_host(stream, npixels: int, dst_index, image) -> None:
    """Host reference of atr_scatter_bgr_masked: image[dst_index[i]] = pixel i of the stream."""
    b = np.asarray(stream, np.uint8)
    hdr = b[:16].view("<u4")
    assert int(hdr[0]) == MASK_MAGIC, "not a masked exchange stream"
    bg, nc, total = int(hdr[1]), int(hdr[2]), int(hdr[3])
    assert nc == -(-npixels // MASK_CHUNK)
    w0 = 16 + 4 * nc
    words = b[w0:w0 + 4 * nc * (MASK_CHUNK // 32)].view("<u4")
    bits = np.unpackbits(words.astype(">u4").view(np.uint8).reshape(-1, 4), axis=1)
    nb = bits.reshape(-1, 32)[:, ::-1].ravel()[:npixels].astype(bool)
    vals = np.full(npixels, bg, np.uint32)
    p0 = w0 + 4 * nc * (MASK_CHUNK // 32) + 4 * nc * (MASK_CHUNK // 64)  # past the masks and group offsets
    p = b[p0:][:3 * total].reshape(-1, 3).astype(np.uint32)
    vals[nb] = p[:, 0] | (p[:, 1] << 8) | (p[:, 2] << 16)
    image[np.asarray(dst_index, np.int64)] = vals


def scatter_host(bufs, plan: ShardPlan) -> np.ndarray:
    """Host-side reassembly of gathered packed buffers (the GPU path uses atr_unpack)."""
    img = np.zeros(plan.width * plan.height, dtype=np.asarray(bufs[0]).dtype)
    for r, b in enumerate(bufs):
        m = plan.pixel_map(r)
        img[m] = np.asarray(b)[:len(m)]
    return img.reshape(plan.height, plan.width)
