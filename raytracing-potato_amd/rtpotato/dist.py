"""Multi-GPU frame assembly: one process per GPU, image tiles interleaved across ranks (tile t goes to
rank t % world), one collective per frame -- an all-gather of the per-rank shard buffers over RCCL
(xGMI) -- then a device-side scatter of slot order into frame order.  The scene is replicated per GPU.

The reference's only parallelism is its thread tile queue (main.rs:36-98, `Arc<Mutex<Vec<Tile>>>`);
this replaces it across devices.  Per-pixel RNG seeding makes the gathered frame bitwise identical for
any world size (tests/test_dist.py, tests/test_gpu_parity.py::test_shards_cover_frame_bitwise).
"""
from __future__ import annotations

from dataclasses import replace

import numpy as np

from .scene import RenderParams, shard_slot_count, shard_slot_pixels


def shard_params(params: RenderParams, rank: int, world: int) -> RenderParams:
    return replace(params, shard=rank, num_shards=world)


def max_slots(params: RenderParams, world: int) -> int:
    """Shard 0 holds the most tiles: the padded per-rank buffer length (in pixels) for the all-gather."""
    return shard_slot_count(replace(params, shard=0, num_shards=world))


class FrameAssembler:
    """Precomputed (slot -> pixel) scatter indices for every rank's shard, as torch tensors on `device`."""

    def __init__(self, params: RenderParams, world: int, device):
        import torch
        self.params = params
        self.world = world
        self.slots = max_slots(params, world)
        src, dst = [], []
        for r in range(world):
            pix = shard_slot_pixels(shard_params(params, r, world))
            ok = np.nonzero(pix >= 0)[0]
            src.append(r * self.slots + ok)
            dst.append(pix[ok])
        self.src = torch.as_tensor(np.concatenate(src), dtype=torch.int64, device=device)
        self.dst = torch.as_tensor(np.concatenate(dst), dtype=torch.int64, device=device)
        self.device = device

    def new_shard_buffer(self, dtype=None):
        import torch
        return torch.zeros(3 * self.slots, dtype=dtype or torch.float64, device=self.device)

    def gather(self, shard_buf, group=None, out=None):
        """All-gather every rank's shard buffer and scatter into an (h, w, 3) frame tensor (every rank)."""
        import torch
        import torch.distributed as dist
        p = self.params
        if self.world > 1:
            gathered = torch.empty(self.world * 3 * self.slots, dtype=shard_buf.dtype, device=shard_buf.device)
            if dist.get_backend(group) == "gloo":  # gloo has no all_gather_into_tensor
                dist.all_gather(list(gathered.view(self.world, -1).unbind(0)), shard_buf, group=group)
            else:
                dist.all_gather_into_tensor(gathered, shard_buf, group=group)
        else:
            gathered = shard_buf
        if out is None:
            out = torch.zeros(p.height * p.width, 3, dtype=shard_buf.dtype, device=shard_buf.device)
        out.view(-1, 3)[self.dst] = gathered.view(-1, 3)[self.src]
        return out.view(p.height, p.width, 3)

    def new_bgra_buffer(self):
        import torch
        return torch.zeros(4 * self.slots, dtype=torch.uint8, device=self.device)

    def gather_bgra(self, shard_bgra, group=None, out=None):
        """Like gather() for the output stage's bytes (DeviceScene.to_bgra8): 4 bytes per pixel instead of
        24, moved and scattered as one int32 each; returns the (h, w, 4) B, G, R, A frame -- the body of
        the reference's output.tga (rtpotato.render.tga_bytes)."""
        import torch
        import torch.distributed as dist
        p = self.params
        words = shard_bgra.view(torch.int32)
        if self.world > 1:
            gathered = torch.empty(self.world * self.slots, dtype=torch.int32, device=words.device)
            if dist.get_backend(group) == "gloo":
                dist.all_gather(list(gathered.view(self.world, -1).unbind(0)), words, group=group)
            else:
                dist.all_gather_into_tensor(gathered, words, group=group)
        else:
            gathered = words
        if out is None:
            out = torch.zeros(p.height * p.width * 4, dtype=torch.uint8, device=words.device)
        out.view(torch.int32)[self.dst] = gathered[self.src]
        return out.view(p.height, p.width, 4)
