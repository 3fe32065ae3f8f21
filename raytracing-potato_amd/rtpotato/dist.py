"""Multi-GPU frames: one process per GPU, image tiles dealt across ranks (interleaved -- tile t goes to rank t %
world -- or by the balanced cost plan, RP_SHARD_BALANCED), one RCCL all-gather per frame over xGMI inside librp.so (rp_frame_gather / rp_render_gather), then
a device-side de-interleave into frame order.  The scene is replicated per GPU.

The reference's only parallelism is its thread tile queue (main.rs:36-98, `Arc<Mutex<Vec<Tile>>>`); this
replaces it across devices.  Per-pixel RNG seeding makes the gathered frame bitwise identical for any world
size (tests/test_dist.py, tests/test_gpu_configs.py).  torch.distributed (gloo) is only the bootstrap: it
carries rank 0's RCCL unique id to the other ranks and the benchmark's barrier and max-time reduction; the
frame itself never passes through torch.
"""
from __future__ import annotations

from dataclasses import replace

import numpy as np

from .scene import RenderParams, shard_slot_count


def shard_params(params: RenderParams, rank: int, world: int) -> RenderParams:
    return replace(params, shard=rank, num_shards=world)


def max_slots(params: RenderParams, world: int) -> int:
    """Shard 0 holds the most tiles: the per-rank buffer length (slots) of a gathered frame
    (rp_gather_stride)."""
    return shard_slot_count(replace(params, shard=0, num_shards=world))


def assemble_frame(gathered: np.ndarray, params: RenderParams, world: int, tile_map=None) -> np.ndarray:
    """NumPy restatement of the device frame assembly (rp_kernel.hip frame_assemble_kernel, rp_frame_assemble):
    gathered = (world * stride, C) slots, rank r's shard at r * stride; returns (H, W, C) in frame order.
    Pixel (i, j) is in tile t = (j / th) * tiles_x + i / tw at position pos of the deal order (pos = t for the
    interleave; tile_map = the deal order of a balanced frame, rp_workspace_tile_map), owned by rank pos % world as
    its shard tile k = pos / world, slot k * tw * th + (j % th) * tw + i % tw."""
    tw, th = params.tile_w, params.tile_h
    tiles_x = -(-params.width // tw)
    stride = max_slots(params, world)
    j, i = np.mgrid[0:params.height, 0:params.width]
    t = (j // th) * tiles_x + i // tw
    if tile_map is not None:
        inv = np.empty(len(tile_map), dtype=np.int64)
        inv[np.asarray(tile_map, dtype=np.int64)] = np.arange(len(tile_map))
        t = inv[t]
    r, k = t % world, t // world
    slot = r * stride + k * tw * th + (j % th) * tw + i % tw
    return gathered[slot]


def deal_tiles(cost, world: int, tiles_x: int = 0, block: int = 1) -> np.ndarray:
    """NumPy restatement of the balanced tile plan's deal (rp_kernel.hip tile_plan_kernel, RP_SHARD_BALANCED): the frame
    tiles (row-major, `tiles_x` a row) grouped into blocks of block x block tiles, the tiles sorted by their block's
    summed cost descending (ties by block index, then tile index), then dealt in units of block**2 sorted positions,
    rounds of `world` units alternating direction (round k to ranks 0..world-1 when k is even, world-1..0 when odd),
    the positions past the last whole round one at a time the same way (the last partial round forward).  block = 1:
    tile by tile.  Returns the deal order: shard s's k-th tile is order[s + k * world]."""
    cost = np.asarray(cost, dtype=np.int64)
    n = len(cost)
    t = np.arange(n)
    if block > 1:
        bx_n = -(-tiles_x // block)
        b = (t // tiles_x // block) * bx_n + (t % tiles_x) // block
    else:
        b = t
    bcost = np.zeros(n, dtype=np.int64)
    np.add.at(bcost, b, cost)
    bc = np.minimum(bcost[b], 0xFFFFFFFF)
    srt = np.lexsort((t, b, -bc))  # block cost descending, then block, then tile
    U = block * block
    R = n // (U * world)
    head = R * U * world
    tail_full = (n - head) // world
    p = np.arange(n)
    u = p // U
    k, i = u // world, u % world
    rank = np.where(k % 2 == 1, world - 1 - i, i)
    j = k * U + (p - u * U)
    q = p - head
    k2, i2 = q // world, q % world
    rank = np.where(p < head, rank, np.where((k2 < tail_full) & (k2 % 2 == 1), world - 1 - i2, i2))
    j = np.where(p < head, j, R * U + k2)
    order = np.empty(n, dtype=np.int64)
    order[j * world + rank] = srt
    return order


def share_unique_id(rank: int, world: int, group=None) -> bytes:
    """Rank 0's RCCL unique id (rp_comm_unique_id), broadcast to every rank over torch.distributed (any
    backend; gloo suffices)."""
    import torch.distributed as dist
    from .render import comm_unique_id
    box = [comm_unique_id() if rank == 0 else None]
    if world > 1:
        dist.broadcast_object_list(box, src=0, group=group)
    return box[0]


def bootstrap_comm(rank: int, world: int, device: int, group=None):
    """rp_comm for this rank on `device`: every rank joins rank 0's communicator (rp_comm_create)."""
    from .render import Comm
    return Comm(share_unique_id(rank, world, group), world, rank, device)
