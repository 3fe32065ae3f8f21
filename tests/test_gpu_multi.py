"""GPU tests of the multi-GPU boundary added in ABI v5 (include/rp.h): the balanced tile plan (RP_SHARD_BALANCED)
and the frame gather's status reduction, plus the error path of a traversal-stack overflow made reachable by the
test-only option rp_scene_options.debug_stack_depth.

The reference splits a frame over its worker threads with one shared tile queue (main.rs:41,55-59), so no
worker idles while tiles remain; across GPUs the split is static, and the balanced plan deals the tiles by a
probed cost instead of tile t -> rank t % N.  Every plan is checked to rebuild the single-device frame bit for bit.
"""
import ctypes
import os
import subprocess
import sys
from dataclasses import replace

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


def _params(w, h, spp, **kw):
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    return RenderParams(w, h, spp, 8, scenes.DEFAULT_SEED, 16, 16, **kw)


@pytest.mark.parametrize("world", [3, 8])
def test_balanced_plan_rebuilds_frame(gpu, world):
    """Every rank's render (here: `world` workspaces on one GPU) makes the same plan -- a permutation of the
    frame's tiles with the interleave's tile count per rank, different from the interleave -- and the shards,
    laid out as the all-gather leaves them and assembled with rp_frame_assemble_ws, are the rp_render frame bit
    for bit; so is the NumPy restatement of the assembly with the plan (rtpotato.dist.assemble_frame)."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import assemble_frame, max_slots, shard_params
    from rtpotato.scene import shard_slot_count
    sc = scenes.configure(scenes.bunny_full(), 150, 90)
    p = _params(150, 90, 6, shard_map=F.RP_SHARD_BALANCED)
    ref, _, st = gpu.render(sc, replace(p, shard_map=0))
    S = max_slots(p, world)
    gathered = torch.zeros(world * S * 3, dtype=torch.float64, device="cuda")
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
    rays = 0
    n_tiles = 10 * 6
    with gpu.DeviceScene(sc) as ds:
        wss = [ds.workspace() for _ in range(world)]
        maps = []
        for r in range(world):
            sp = shard_params(p, r, world)
            n = shard_slot_count(sp)
            ds.reserve(sp, wss[r])
            ds.render_device(sp, gathered[r * S * 3:(r * S + n) * 3], ctr, workspace=wss[r])
            torch.cuda.synchronize()
            rays += int(ctr[0])
            assert int(ctr[3]) == 0
            maps.append(ds.tile_map(sp, wss[r]))
        for m in maps:
            assert np.array_equal(m, maps[0])
        order = maps[0]
        assert np.array_equal(np.sort(order), np.arange(n_tiles)) and not np.array_equal(order, np.arange(n_tiles))
        frame = torch.zeros(p.width * p.height * 3, dtype=torch.float64, device="cuda")
        pc = shard_params(p, 0, world).to_c()
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        F.check(F.rp().rp_frame_assemble_ws(ds.handle, wss[0].handle, ctypes.byref(pc), gathered.data_ptr(), 6,
                                            frame.data_ptr(), s))
        with pytest.raises(F.RPError):  # the plan-less assembly refuses a balanced frame
            F.check(F.rp().rp_frame_assemble(ctypes.byref(pc), gathered.data_ptr(), 6, frame.data_ptr(), s))
        torch.cuda.synchronize()
    got = frame.cpu().numpy().reshape(p.height, p.width, 3)
    assert np.array_equal(got, ref)
    assert np.array_equal(assemble_frame(gathered.cpu().numpy().reshape(-1, 3), p, world, order), ref)
    assert rays == st["rays"]


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("W,H", [(512, 512), (520, 488)])
def test_block_deal_matches_restatement(gpu, world, W, H):
    """Scenes dealt in Z-order (tile_order morton, on request: AUTO is the cost order) make balanced plans of square tile blocks
    (rp_api.cpp plan_block: 4 x 4 here, 4,096 tiles) from the installed cost table: the device plan equals the NumPy
    restatement (rtpotato.dist.deal_tiles with block = 4), and the shards rebuild the interleave frame bit for bit.  The
    520 x 488 grid (65 x 61 tiles) is ragged: its edge blocks hold fewer than block^2 tiles, so later units
    straddle two blocks (rp_api.cpp plan_block) -- the device must still equal the restatement and rebuild the frame."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import deal_tiles, max_slots, shard_params
    from rtpotato.scene import RenderParams, shard_slot_count
    sc = scenes.configure(scenes.bunny_full(), W, H)
    p = RenderParams(W, H, 1, 8, scenes.DEFAULT_SEED, 8, 8, shard_map=F.RP_SHARD_BALANCED)
    tx, ty = -(-W // 8), -(-H // 8)
    n = tx * ty
    rng = np.random.default_rng(3)
    xs, ys = np.meshgrid(np.arange(tx), np.arange(ty))
    cost = ((50 + 500 * (((xs - 32) ** 2 + (ys - 32) ** 2) < 400)) * rng.uniform(0.8, 1.2, xs.shape)).astype(np.uint32)
    table = np.stack([cost.reshape(-1), cost.reshape(-1) // 4])
    block = next((b for b in (4, 2) if n >= 32 * world * b * b), 1)  # rp_api.cpp plan_block
    want = deal_tiles(table[0], world, tx, block)
    S = max_slots(p, world)
    gathered = torch.zeros(world * S * 3, dtype=torch.float64, device="cuda")
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
    with gpu.DeviceScene(sc, options={"tile_order": "morton"}) as ds:
        ref, _, st = ds.render(replace(p, shard_map=0))
        wss = [ds.workspace() for _ in range(world)]
        for r in range(world):
            sp = shard_params(p, r, world)
            ds.reserve(sp, wss[r])
            ds.set_tile_costs(p, table, world, wss[r])
            ds.render_device(sp, gathered[r * S * 3:(r * S + shard_slot_count(sp)) * 3], ctr, workspace=wss[r])
            torch.cuda.synchronize()
            assert int(ctr[3]) == 0
            assert np.array_equal(ds.tile_map(sp, wss[r]), want), r
        frame = torch.zeros(W * H * 3, dtype=torch.float64, device="cuda")
        pc = shard_params(p, 0, world).to_c()
        s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        F.check(F.rp().rp_frame_assemble_ws(ds.handle, wss[0].handle, ctypes.byref(pc), gathered.data_ptr(), 6,
                                            frame.data_ptr(), s))
        torch.cuda.synchronize()
    assert np.array_equal(frame.cpu().numpy().reshape(H, W, 3), ref)
    assert (n, block) == (4096, 4) if W == 512 else (block > 1 and tx % block != 0)


def test_balanced_host_render_and_unpack(gpu):
    """rp_render of a balanced shard writes exactly the pixels of its planned tiles, equal to the full frame's; the
    interleave-only rp_shard_unpack refuses a balanced frame, rp_shard_unpack_map takes its plan."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import shard_params
    from rtpotato.render import unpack_shard
    from rtpotato.scene import shard_slot_pixels
    sc = scenes.configure(scenes.bunny_full(), 96, 64)
    p = _params(96, 64, 5, shard_map=F.RP_SHARD_BALANCED)
    with gpu.DeviceScene(sc) as ds:
        full, _, st = ds.render(replace(p, shard_map=0))
        total = 0
        for r in range(4):
            sp = shard_params(p, r, 4)
            rgb, _, sst = ds.render(sp)
            order = ds.tile_map(sp)
            pix = shard_slot_pixels(sp, order)
            m = np.zeros(96 * 64, dtype=bool)
            m[pix[pix >= 0]] = True
            m = m.reshape(64, 96)
            assert np.array_equal(rgb[m], full[m]) and not rgb[~m].any()
            assert sst["pixels"] == m.sum()
            total += sst["rays"]
            shard = np.zeros((len(pix), 3))
            shard[pix >= 0] = full.reshape(-1, 3)[pix[pix >= 0]]
            with pytest.raises(F.RPError):
                unpack_shard(sp, shard)
            assert np.array_equal(unpack_shard(sp, shard, tile_map=order)[m], full[m])
        assert total == st["rays"]


def test_balanced_plan_balances_c3_costs(gpu):
    """On config C3's frame the balanced plan's 8 shards carry nearly equal work: the per-shard ray counts of the
    real 256-spp frame are within 3 % of their mean (the interleave's are compared for the record)."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import shard_params
    scene, params = scenes.config_scene("C3")
    params = replace(params, spp=32)  # one RNG batch per pixel: the same paths as the frame's first 32 samples
    rays = {}
    with gpu.DeviceScene(scene) as ds:
        for mode in (F.RP_SHARD_INTERLEAVE, F.RP_SHARD_BALANCED):
            rays[mode] = [ds.render(shard_params(replace(params, shard_map=mode), r, 8))[2]["rays"] for r in range(8)]
    bal, inter = np.array(rays[F.RP_SHARD_BALANCED]), np.array(rays[F.RP_SHARD_INTERLEAVE])
    assert bal.sum() == inter.sum()
    assert bal.max() / bal.mean() < 1.03, (bal, inter)


def test_multi_balanced_single_device(gpu):
    """rp_render_multi with the balanced plan over device 0 equals rp_render."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.render import MultiScene
    sc = scenes.configure(scenes.bunny_full(), 64, 40)
    p = _params(64, 40, 12, shard_map=F.RP_SHARD_BALANCED)
    ref, _, st = gpu.render(sc, replace(p, shard_map=0))
    with MultiScene(sc, [0]) as ms:
        rgb, bgra, mst = ms.render(p, bgra=True)
    assert np.array_equal(rgb, ref) and mst["rays"] == st["rays"]


def _overflow_scene():
    from rtpotato import scenes
    return scenes.configure(scenes.random_mesh(200_000), 48, 32)


def test_stack_overflow_is_reported(gpu):
    """debug_stack_depth = 8 (cap 5 entries) on a tree needing ~31: every entry point reports the overflow --
    rp_render and rp_render_multi return RP_EINTERNAL, rp_render_device and rp_render_gather (1-rank RCCL
    communicator: the status word goes through the counter all-gather and its OR reduction) leave the bit in
    the counters.  The kernels never write past the stack (the frame is wrong, the process is fine)."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato.render import Comm, MultiScene, comm_unique_id
    from rtpotato.scene import shard_slot_count
    sc = _overflow_scene()
    p = _params(48, 32, 4)
    opts = {"debug_stack_depth": 8}
    with gpu.DeviceScene(sc, options=opts) as ds:
        with pytest.raises(F.RPError) as e:
            ds.render(p)
        assert e.value.code == F.RP_EINTERNAL and "overflow" in str(e.value)
        out = torch.zeros(3 * shard_slot_count(p), dtype=torch.float64, device="cuda")
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
        ds.render_device(p, out, ctr)
        torch.cuda.synchronize()
        assert int(ctr[3]) & F.RP_STATUS_STACK_OVERFLOW
        with Comm(comm_unique_id(), 1, 0, 0) as comm:
            for mode in (F.RP_SHARD_INTERLEAVE, F.RP_SHARD_BALANCED):
                q = replace(p, shard_map=mode)
                ds.reserve(q)
                frame = torch.zeros(4 * p.width * p.height, dtype=torch.uint8, device="cuda")
                ctr.zero_()
                ds.render_gather(comm, q, frame_bgra=frame, counters=ctr)
                torch.cuda.synchronize()
                assert int(ctr[3]) == F.RP_STATUS_STACK_OVERFLOW and int(ctr[0]) > 0
    with MultiScene(sc, [0], options=opts) as ms:
        with pytest.raises(F.RPError) as e:
            ms.render(p)
        assert e.value.code == F.RP_EINTERNAL and "overflow" in str(e.value)
    # the same scene with the stack the tree needs: no status
    with gpu.DeviceScene(sc) as ds:
        _, _, st = ds.render(p)
        assert st["rays"] > 0


def test_bench_refuses_overflowing_frame():
    """bench.py checks every frame's status word and refuses to report a rate for a frame that overflowed."""
    env = dict(os.environ)
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--config", "C1", "--steps", "1", "--warmup", "0",
                        "--no-cpu-baseline", "--opt", "debug_stack_depth=8"], capture_output=True, text=True,
                       timeout=300, env=env, cwd=REPO)
    assert r.returncode != 0 and "status" in r.stderr, (r.returncode, r.stderr[-2000:])
    assert '"metric"' not in r.stdout


def test_learned_tile_costs(gpu):
    """The megakernel measures every unit's duration per tile; a whole-frame render leaves a learned table the next
    frame schedules from (no probe) -- bitwise the same frame -- and an installed table (rp_workspace_set_tile_costs,
    e.g. all-zero, or reversed) changes the order only, never a pixel."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    sc = scenes.configure(scenes.bunny_full(), 128, 96)
    p = _params(128, 96, 8)
    with gpu.DeviceScene(sc) as ds:
        a, _, sa = ds.render(p)          # probe-ordered (fresh workspace), learns
        costs = ds.tile_costs(p)
        assert costs.shape == (2, 48) and (costs[0] > 0).all() and (costs[0] >= costs[1]).all()
        b, _, sb = ds.render(p)          # scheduled from the learned table
        ds.set_tile_costs(p, np.stack([costs[0][::-1], costs[1][::-1]]), 1)
        c, _, sc_ = ds.render(p)
        ds.set_tile_costs(p, np.zeros((2, 48), dtype=np.uint32), 1)
        d, _, sd = ds.render(replace(p, shard_map=F.RP_SHARD_BALANCED))
    assert np.array_equal(a, b) and np.array_equal(a, c) and np.array_equal(a, d)
    assert sa["rays"] == sb["rays"] == sc_["rays"] == sd["rays"]


def test_frames_past_the_tile_table(gpu):
    """a frame of more than TILE_SORT_MAX (16384) tiles -- 4 x 4 tiles at 640 x 480 = 19,200 -- is not
    measured (the per-tile cost table holds 16384 tiles; the kernel's atomics and the gather's cost all-gathers would
    run past it), and still renders: rp_render, and rp_render_gather on a 1-rank RCCL communicator (both shard maps:
    the balanced plan falls back to the interleave past the table), equal the 16 x 16-tile frame bit for bit --
    per-pixel seeding makes a pixel independent of the tiling."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.render import Comm, comm_unique_id
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.bunny_full(), 640, 480)
    big = RenderParams(640, 480, 1, 8, scenes.DEFAULT_SEED, 16, 16)
    small = RenderParams(640, 480, 1, 8, scenes.DEFAULT_SEED, 4, 4)
    with gpu.DeviceScene(sc) as ds:
        ref, _, st = ds.render(big)
        for _ in range(2):  # the second frame of a workspace would schedule from a learned table
            rgb, _, st2 = ds.render(small)
            assert np.array_equal(rgb, ref) and st2["rays"] == st["rays"]
        with Comm(comm_unique_id(), 1, 0, 0) as comm:
            for mode in (F.RP_SHARD_INTERLEAVE, F.RP_SHARD_BALANCED):
                q = replace(small, shard_map=mode)
                ds.reserve(q)
                frame = torch.zeros(640 * 480 * 3, dtype=torch.float64, device="cuda")
                ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
                for _ in range(2):
                    ctr.zero_()
                    ds.render_gather(comm, q, frame_rgb=frame, counters=ctr)
                    torch.cuda.synchronize()
                    assert int(ctr[3]) == 0 and int(ctr[0]) == st["rays"]
                    assert np.array_equal(frame.cpu().numpy().reshape(480, 640, 3), ref)
