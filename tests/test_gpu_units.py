"""The learned per-unit order (rp_scene_options.unit_order, rp_sched.hip; rp_device.h fetch_pixel).

A render of one frame per launch stores every unit's duration; the next frame of the same shape on the workspace hands
its units out longest first.  Units are seeded by pixel and batch, so a different schedule must give the
same frame bit for bit -- and the oracle's.  The order itself must be longest first: sorted by the previous frame's
durations in log-spaced buckets (rp_sched.hip unit_bucket: 4 per octave of 100 MHz ticks), shard order inside a bucket
(round 5's 6-bit bucket field saturated at ~0.46 ms, and its "learned" order was shard order).
"""
import numpy as np
import pytest
from dataclasses import replace

from parity import assert_parity, compare, oracle_render

pytestmark = pytest.mark.gpu


def _scene(name, w, h, spp, **kw):
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.CATALOGUE[name](**kw), w, h)
    return sc, RenderParams(w, h, spp, 8, scenes.DEFAULT_SEED)


def _bucket(c):
    """rp_sched.hip unit_bucket: 0 for a unit that never ran, else log2(c) * 4 + 1 (f32 log2), at most 254."""
    c = np.asarray(c, dtype=np.float32)
    b = np.where(c > 0, np.floor(np.log2(np.maximum(c, np.float32(1))).astype(np.float32) * np.float32(4)) + 1, 0)
    return np.minimum(b, 254).astype(np.int64)


@pytest.mark.parametrize("sps,opt", [(0, "learned"), (256, "learned"), (7, "learned"), (256, "auto")])
def test_learned_unit_order_same_frame(gpu, sps, opt):
    """The second frame on a workspace hands its units out longest first by the first frame's durations -- a different
    schedule, the same frame bit for bit (per-unit seeding), against the oracle too; with RP_UNITS_TILES no frame does.
    AUTO learns for one stream per pixel."""
    from rtpotato import _ffi as F
    sc, p = _scene("bunny_full", 72, 40, 64)
    p = replace(p, samples_per_stream=sps, tile_w=16, tile_h=16)
    with gpu.DeviceScene(sc, options={"unit_order": opt}) as ds:
        ds.reserve(p)
        a, fa, sa = ds.render(p, foreground=True)
        f1 = ds.frame_info()
        b, fb, sb = ds.render(p, foreground=True)
        f2 = ds.frame_info()
    assert not f1 & F.RP_FRAME_UNIT_ORDER and f2 & F.RP_FRAME_UNIT_ORDER, (f1, f2)
    assert np.array_equal(a, b) and np.array_equal(fa, fb) and sa["rays"] == sb["rays"]
    ref, _, ctr = oracle_render(sc, p, threads=8)
    assert_parity(compare(b, ref))
    assert sb["rays"] == ctr["rays"]
    with gpu.DeviceScene(sc, options={"unit_order": "tiles"}) as ds:
        ds.reserve(p)
        ds.render(p)
        c, _, sc_ = ds.render(p)
        assert not ds.frame_info() & F.RP_FRAME_UNIT_ORDER
    assert np.array_equal(c, b) and sc_["rays"] == sb["rays"]


def test_auto_unit_order_keeps_tiles_for_several_streams(gpu):
    """AUTO hands out 32-sample streams tile by tile (the learned order lost 4.4 % there) and never reorders a launch of
    several frames."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    sc, p = _scene("bunny_full", 64, 48, 64)
    p = replace(p, tile_w=16, tile_h=16)
    with gpu.DeviceScene(sc) as ds:
        ds.reserve(p)
        ds.render(p)
        ds.render(p)
        assert not ds.frame_info() & F.RP_FRAME_UNIT_ORDER
        q = replace(p, samples_per_stream=64)
        ds.reserve_frames(q, 2)
        ds.render(q)
        ds.render(q)
        assert ds.frame_info() & F.RP_FRAME_UNIT_ORDER
        n = shard_slot_count(q)
        out = torch.zeros(2 * 3 * n, dtype=torch.float64, device="cuda")
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
        ds.render_frames_device(q, 2, out, ctr)
        torch.cuda.synchronize()
        assert not ds.frame_info() & F.RP_FRAME_UNIT_ORDER


def test_learned_unit_order_is_longest_first(gpu):
    """glass_bunny under one stream per pixel: units (pixels) differ by orders of magnitude in duration (glass paths of
    hundreds of rays against sky pixels).  The order of the second frame is a permutation of the units whose buckets of
    the first frame's durations never increase, shard order inside a bucket, and its first unit is in the top bucket --
    and a unit that never ran (an edge-tile slot outside the frame) sorts last."""
    from rtpotato.scene import shard_slot_count
    sc, p = _scene("glass_bunny", 60, 44, 32)
    p = replace(p, samples_per_stream=32, tile_w=16, tile_h=16)  # 4 x 3 tiles: the last column and row ragged
    n = shard_slot_count(p)
    with gpu.DeviceScene(sc, options={"unit_order": "learned"}) as ds:
        ds.reserve(p)
        ds.render(p)
        dur, _ = ds.unit_order(n)
        ds.render(p)
        _, order = ds.unit_order(n)
    assert sorted(order.tolist()) == list(range(n))
    b = _bucket(dur[order])
    assert (np.diff(b) <= 0).all(), "buckets must not increase along the order"
    for k in np.unique(b):  # shard order inside a bucket (a stable sort of the unit index)
        idx = order[b == k]
        assert (np.diff(idx.astype(np.int64)) > 0).all()
    assert b[0] == _bucket(dur).max() and (dur > 0).sum() == 60 * 44
    assert b[-1] == 0 and dur[order[-1]] == 0  # the edge slots outside the 60 x 44 frame never ran
    assert _bucket(dur).max() - np.median(_bucket(dur[dur > 0])) >= 8  # the scene has long and short units (2 octaves)


@pytest.mark.parametrize("sps", [0, 48])
def test_learned_unit_order_frame_launch(gpu, sps):
    """LEARNED also orders launches of several frames (a unit's frames handed out together, each with its own seeds): the
    second launch of 3 frames on a workspace uses the order its first launch learned, and every frame of it equals its
    lone render bit for bit, counters summed."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    sc, p = _scene("bunny_full", 64, 40, 48)
    p = replace(p, samples_per_stream=sps, tile_w=16, tile_h=16)
    n, nf = shard_slot_count(p), 3
    B = -(-p.spp // (sps or F.RP_SAMPLES_PER_STREAM))
    dev = torch.device("cuda", 0)
    with gpu.DeviceScene(sc, options={"unit_order": "learned"}) as ds:
        w = ds.workspace()
        ds.reserve_frames(p, nf, w)
        out = torch.zeros(nf * 3 * n, dtype=torch.float64, device=dev)
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
        ds.render_frames_device(p, nf, out, ctr, workspace=w)
        assert not ds.frame_info(w) & F.RP_FRAME_UNIT_ORDER
        ds.render_frames_device(p, nf, out, ctr, workspace=w)
        torch.cuda.synchronize()
        assert ds.frame_info(w) & F.RP_FRAME_UNIT_ORDER
        multi = out.cpu().numpy().reshape(nf, n, 3)
        rays = 0
        with gpu.DeviceScene(sc, options={"unit_order": "tiles"}) as ref:
            for f in range(nf):
                o = torch.zeros(3 * n, dtype=torch.float64, device=dev)
                c = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
                ref.reserve(p)
                ref.render_device(replace(p, seed=p.seed + f * B * p.width * p.height), o, c)
                torch.cuda.synchronize()
                assert np.array_equal(multi[f].view(np.uint64), o.cpu().numpy().reshape(n, 3).view(np.uint64)), f
                rays += int(c[0])
        assert int(ctr[0]) == rays and int(ctr[3]) == 0
        w.close()
