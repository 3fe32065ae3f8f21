"""Multi-process frames on CPU with gloo, world size 2 and 3: each rank renders its interleaved tile shard
(here with the CPU oracle, whose per-pixel seeding the GPU shares) into a buffer padded to the gather
stride, the buffers are all-gathered, and the NumPy restatement of the device frame assembly
(rtpotato.dist.assemble_frame = rp_frame_assemble's index arithmetic) must rebuild the single-process frame
bit for bit.  The RCCL bootstrap (rank 0's unique id broadcast over gloo) runs for real."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_dir):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "raytracing-potato_amd")]
    import torch
    import torch.distributed as dist
    from parity import oracle_render
    from rtpotato import scenes
    from rtpotato.dist import assemble_frame, max_slots, shard_params, share_unique_id
    from rtpotato.scene import RenderParams, shard_slot_pixels
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    uid = share_unique_id(rank, world)
    ids = [None] * world
    dist.all_gather_object(ids, uid)
    scene = scenes.configure(scenes.bunny_full(), 75, 41)
    params = RenderParams(75, 41, 2, 8, 77, 16, 16)
    sp = shard_params(params, rank, world)
    frame, _, ctr = oracle_render(scene, sp, threads=2)
    stride = max_slots(params, world)
    buf = torch.zeros(stride, 3, dtype=torch.float64)
    pix = shard_slot_pixels(sp)
    ok = pix >= 0
    buf[:len(pix)][torch.as_tensor(ok)] = torch.as_tensor(frame.reshape(-1, 3)[pix[ok]])
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = assemble_frame(torch.cat(parts).numpy(), params, world)
    # the output-stage bytes (B, G, R, A per slot, as rp_shard_to_bgra8 writes them) assemble the same way
    from rtpotato import _ffi as F
    lin = np.ascontiguousarray(buf.numpy())
    rgba = np.zeros((stride, 4), dtype=np.uint8)
    F.host().rph_to_srgb_u8(lin.ctypes.data, stride, rgba.ctypes.data)
    words = torch.as_tensor(np.ascontiguousarray(rgba[:, [2, 1, 0, 3]]).view(np.int32).reshape(-1))
    wparts = [torch.zeros_like(words) for _ in range(world)]
    dist.all_gather(wparts, words)
    out8 = assemble_frame(torch.cat(wparts).numpy()[:, None], params, world).view(np.uint8)
    rays = torch.tensor([ctr["rays"]], dtype=torch.int64)
    dist.all_reduce(rays)
    if rank == 0:
        np.save(os.path.join(result_dir, "frame.npy"), out)
        np.save(os.path.join(result_dir, "frame8.npy"), out8)
        np.save(os.path.join(result_dir, "rays.npy"), rays.numpy())
        np.save(os.path.join(result_dir, "ids.npy"), np.array([np.frombuffer(i, dtype=np.uint8) for i in ids]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gather_rebuilds_frame(tmp_path, world):
    from parity import oracle_render
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    got = np.load(tmp_path / "frame.npy")
    scene = scenes.configure(scenes.bunny_full(), 75, 41)
    ref, _, ctr = oracle_render(scene, RenderParams(75, 41, 2, 8, 77, 16, 16), threads=4)
    assert np.array_equal(got, ref)
    assert int(np.load(tmp_path / "rays.npy")[0]) == ctr["rays"]
    from rtpotato import _ffi as F
    rgba = np.zeros((41 * 75, 4), dtype=np.uint8)
    F.host().rph_to_srgb_u8(np.ascontiguousarray(ref).ctypes.data, 41 * 75, rgba.ctypes.data)
    assert np.array_equal(np.load(tmp_path / "frame8.npy").reshape(-1, 4), rgba[:, [2, 1, 0, 3]])
    ids = np.load(tmp_path / "ids.npy")
    assert ids.shape == (world, F.RP_COMM_ID_BYTES) and (ids == ids[0]).all() and ids[0].any()


def test_max_slots_and_shard_partition():
    """Shard 0 is the largest; shards partition the frame exactly."""
    from rtpotato.dist import max_slots, shard_params
    from rtpotato.scene import RenderParams, shard_slot_count, shard_slot_pixels
    p = RenderParams(1920, 1080, 1, 8, 0)
    for world in (1, 2, 3, 4, 8):
        sizes = [shard_slot_count(shard_params(p, r, world)) for r in range(world)]
        assert max(sizes) == max_slots(p, world) == sizes[0]
        allpix = np.concatenate([shard_slot_pixels(shard_params(p, r, world)) for r in range(world)])
        allpix = np.sort(allpix[allpix >= 0])
        assert np.array_equal(allpix, np.arange(1920 * 1080))


def test_deal_tiles_balances_and_keeps_counts():
    """The balanced plan's deal (rtpotato.dist.deal_tiles, the restatement of tile_plan_kernel): a permutation of
    the frame's tiles, every rank holding exactly the interleave's tile count (so shard buffers and gather strides
    are unchanged), and per-rank cost totals within a few percent on a skewed cost field -- where the interleave,
    whose columns of tiles follow the frame's structure, is far off."""
    from rtpotato.dist import deal_tiles, shard_params
    from rtpotato.scene import RenderParams, shard_slot_count
    rng = np.random.default_rng(5)
    p = RenderParams(1920, 1080, 1, 8, 0)
    tx, ty = 60, 34
    n = tx * ty
    # a bright object in the middle third (costly), cheap sky elsewhere, noisy
    xs, ys = np.meshgrid(np.arange(tx), np.arange(ty))
    cost = (100 + 900 * ((abs(xs - 30) < 10) & (ys < 20)) * (1 + (xs % 8 == 3))) * rng.uniform(0.7, 1.3, (ty, tx))
    cost = cost.astype(np.int64).reshape(-1)
    for world in (1, 2, 3, 4, 8):
        order = deal_tiles(cost, world)
        assert np.array_equal(np.sort(order), np.arange(n))
        loads = np.zeros(world)
        for r in range(world):
            mine = order[r::world]
            assert len(mine) * 32 * 32 == shard_slot_count(shard_params(p, r, world))
            loads[r] = cost[mine].sum()
        assert loads.max() / loads.mean() < 1.01, (world, loads)
        inter = np.array([cost[r::world].sum() for r in range(world)])
        if world == 8:
            assert inter.max() / inter.mean() > 1.05  # the interleave is not balanced on this field


def test_block_deal_keeps_counts_and_compact_squares():
    """The block deal of large scenes (tile_plan_kernel with block = 4; rtpotato.dist.deal_tiles(..., block=4)): still a
    permutation with the interleave's tile count per rank (C5's 128 x 128 tiles; a ragged 1080p grid with a partial last
    round), a rank's tiles come in whole 4 x 4 squares of the frame (C5's grid divides evenly), and the per-rank cost
    totals stay balanced.  block = 1 is the per-tile deal."""
    from rtpotato.dist import deal_tiles, shard_params
    from rtpotato.scene import RenderParams, shard_slot_count
    rng = np.random.default_rng(7)
    for (W, H, tx, ty) in ((4096, 4096, 128, 128), (1920, 1080, 60, 34)):
        p = RenderParams(W, H, 1, 8, 0)
        n = tx * ty
        xs, ys = np.meshgrid(np.arange(tx), np.arange(ty))
        r2 = ((xs - tx / 2) ** 2 + (ys - ty / 2) ** 2) / (tx * tx / 4)
        cost = ((100 + 900 * (r2 < 0.5)) * rng.uniform(0.8, 1.2, (ty, tx))).astype(np.int64).reshape(-1)
        assert np.array_equal(deal_tiles(cost, 8, tx, 1), deal_tiles(cost, 8))
        for world in (2, 3, 8):
            # rp_api.cpp plan_block: 4 x 4 or 2 x 2 blocks while every rank gets >= 32 of them
            block = next((b for b in (4, 2) if n >= 32 * world * b * b), 1)
            order = deal_tiles(cost, world, tx, block)
            assert np.array_equal(np.sort(order), np.arange(n))
            loads = np.zeros(world)
            for r in range(world):
                mine = order[r::world]
                assert len(mine) * 32 * 32 == shard_slot_count(shard_params(p, r, world))
                loads[r] = cost[mine].sum()
                if block > 1 and tx % block == 0 and ty % block == 0 and n % (block * block * world) == 0:
                    blocks = (mine // tx // block) * (tx // block) + (mine % tx) // block
                    _, counts = np.unique(blocks, return_counts=True)
                    assert (counts == block * block).all()  # whole squares only
            assert loads.max() / loads.mean() < 1.03, (W, world, block, loads)
            assert (W, block) != (4096, 1)  # C5's grid always deals blocks


def _worker_balanced(rank, world, port, result_dir):
    """Ranks deal the tiles by the balanced plan (costs: the frame's per-tile ray counts, the same on every rank),
    render their shards (pixels of the oracle frame: per-pixel seeding), all-gather and assemble with the plan."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.dirname(here), os.path.join(os.path.dirname(here), "raytracing-potato_amd")]
    from dataclasses import replace
    import torch
    import torch.distributed as dist
    from parity import oracle_render
    from rtpotato import scenes
    from rtpotato.dist import assemble_frame, deal_tiles, max_slots, shard_params
    from rtpotato.scene import RenderParams, shard_slot_pixels
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    scene = scenes.configure(scenes.bunny_full(), 75, 41)
    params = RenderParams(75, 41, 2, 8, 77, 16, 16, shard_map=1)
    tiles_x, tiles_y = 5, 3
    cost = np.zeros(tiles_x * tiles_y, dtype=np.int64)
    for t in range(tiles_x * tiles_y):  # per-tile cost: the tile's rays (a shard of one tile)
        _, _, c = oracle_render(scene, replace(params, shard=t, num_shards=tiles_x * tiles_y, shard_map=0), threads=1)
        cost[t] = c["rays"]
    order = deal_tiles(cost, world)
    full, _, _ = oracle_render(scene, replace(params, shard_map=0), threads=2)
    sp = shard_params(params, rank, world)
    stride = max_slots(params, world)
    buf = torch.zeros(stride, 3, dtype=torch.float64)
    pix = shard_slot_pixels(sp, order)
    ok = pix >= 0
    buf[:len(pix)][torch.as_tensor(ok)] = torch.as_tensor(full.reshape(-1, 3)[pix[ok]])
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf)
    out = assemble_frame(torch.cat(parts).numpy(), params, world, order)
    orders = [None] * world
    dist.all_gather_object(orders, order.tolist())
    if rank == 0:
        np.save(os.path.join(result_dir, "frame.npy"), out)
        np.save(os.path.join(result_dir, "orders.npy"), np.array(orders))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_balanced_gather_rebuilds_frame(tmp_path, world):
    from dataclasses import replace
    from parity import oracle_render
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    mp.spawn(_worker_balanced, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    scene = scenes.configure(scenes.bunny_full(), 75, 41)
    ref, _, _ = oracle_render(scene, RenderParams(75, 41, 2, 8, 77, 16, 16), threads=4)
    assert np.array_equal(np.load(tmp_path / "frame.npy"), ref)
    orders = np.load(tmp_path / "orders.npy")
    assert (orders == orders[0]).all() and not np.array_equal(orders[0], np.arange(15))

def test_block_deal_ragged_grid():
    """on a grid whose tile counts are not multiples of the block, the edge blocks hold fewer than block^2
    tiles and the deal's units of block^2 consecutive sorted positions then straddle two blocks (rp_api.cpp plan_block's
    comment).  What still holds: a permutation, the interleave's count per rank, balanced loads, and most of a rank's
    tiles in whole squares; what does not: every square whole."""
    from rtpotato.dist import deal_tiles
    rng = np.random.default_rng(11)
    tx, ty, world, block = 65, 61, 2, 4
    n = tx * ty
    cost = rng.integers(50, 500, n)
    order = deal_tiles(cost, world, tx, block)
    assert np.array_equal(np.sort(order), np.arange(n))
    bx_n = -(-tx // block)
    split = 0
    for r in range(world):
        mine = order[r::world]
        assert len(mine) == len(range(r, n, world))
        blocks = (mine // tx // block) * bx_n + (mine % tx) // block
        size = np.bincount((np.arange(n) // tx // block) * bx_n + (np.arange(n) % tx) // block)
        b, counts = np.unique(blocks, return_counts=True)
        split += int((counts != size[b]).sum())
    loads = [cost[order[r::world]].sum() for r in range(world)]
    assert max(loads) / np.mean(loads) < 1.03
    assert 0 < split < 0.5 * len(size)  # some squares split (documented), most whole
