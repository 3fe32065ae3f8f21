"""Several frames per persistent launch (include/rp.h rp_render_frames_device_ws, rp_device.h fetch_pixel).

Frame f of a launch of n_frames is, by the contract, the frame rp_render_device renders with seed + f * B * W * H
(B = the frame's sample batches): every unit is seeded by its pixel and its global batch, so the schedule -- units of
frames f and f + 1 in one wave, a frame's tail run by the next frame's lanes -- cannot change a pixel.  Each frame must
equal its single-frame render bit for bit, the counters must be the frames' sums, and one frame is checked against the
oracle directly.  Cases: one stream per pixel (B = 1) and multi-batch frames (B > 1, partial sums reduced per frame),
ragged tiles, shards of the interleave and of the balanced plan, spp 0 (NaN frames), argument errors.
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


def _nbatch(p):
    from rtpotato import _ffi as F
    sps = p.samples_per_stream or F.RP_SAMPLES_PER_STREAM
    return max(1, -(-p.spp // sps)) if p.spp else 1


def _frames_vs_singles(ds, p, n_frames, table=None, order="auto"):
    """(multi-frame shard buffers, single-frame shard buffers) as numpy arrays of (n_frames, slots, 3), fg the same,
    and both counter blocks."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    n = shard_slot_count(p)
    dev = torch.device("cuda", 0)
    w = ds.workspace()
    ds.reserve_frames(p, n_frames, w)
    if table is not None:
        ds.set_tile_costs(p, table, p.num_shards, w)
    out = torch.full((n_frames * 3 * max(n, 1),), -1.0, dtype=torch.float64, device=dev)
    fg = torch.full((n_frames * max(n, 1),), -1.0, dtype=torch.float32, device=dev)
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
    ds.render_frames_device(p, n_frames, out, ctr, fg=fg, workspace=w, order=order)
    torch.cuda.synchronize()
    singles, sfg, sctr = [], [], torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
    stride = _nbatch(p) * p.width * p.height
    for f in range(n_frames):
        o = torch.full((3 * max(n, 1),), -1.0, dtype=torch.float64, device=dev)
        g = torch.full((max(n, 1),), -1.0, dtype=torch.float32, device=dev)
        c = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
        ds.render_device(replace(p, seed=p.seed + f * stride), o, c, fg=g, workspace=w)
        torch.cuda.synchronize()
        singles.append(o[:3 * n].cpu().numpy())
        sfg.append(g[:n].cpu().numpy())
        sctr[:3] += c[:3]
        sctr[3] |= c[3]
    w.close()
    multi = out[:n_frames * 3 * n].cpu().numpy().reshape(n_frames, n, 3)
    mfg = fg[:n_frames * n].cpu().numpy().reshape(n_frames, n)
    return multi, np.stack(singles).reshape(n_frames, n, 3), mfg, np.stack(sfg), ctr.cpu().numpy(), sctr.cpu().numpy()


def _assert_same(multi, single, mfg, sfg, ctr, sctr):
    assert np.array_equal(multi.view(np.uint64), single.view(np.uint64))
    assert np.array_equal(mfg.view(np.uint32), sfg.view(np.uint32))
    assert ctr.tolist() == sctr.tolist(), (ctr, sctr)
    assert ctr[3] == 0


@pytest.mark.parametrize("order", ["sequential", "interleaved", "pixel"])
@pytest.mark.parametrize("sps", [48, 0, 7, 16])
@pytest.mark.parametrize("n_frames", [1, 3])
def test_frames_equal_single_renders(gpu, sps, n_frames, order):
    """bunny_full 72 x 40 at 48 spp on 16 x 16 tiles (ragged last row and column): one stream per pixel (B = 1), the
    default 32 (B = 2, a short last batch), 7 (B = 7) and 16 samples per stream (B = 3)."""
    sc, p = _scene("bunny_full", 72, 40, 48)
    p = replace(p, samples_per_stream=sps, tile_w=16, tile_h=16)
    with gpu.DeviceScene(sc) as ds:
        _assert_same(*_frames_vs_singles(ds, p, n_frames, order=order))


@pytest.mark.parametrize("name", ["variants_sky", "glass_bunny", "earth"])
def test_frames_scenes(gpu, name):
    sc, p = _scene(name, 48, 32, 24)
    with gpu.DeviceScene(sc) as ds:
        _assert_same(*_frames_vs_singles(ds, replace(p, samples_per_stream=8), 4))


@pytest.mark.parametrize("order", ["sequential", "interleaved", "pixel"])
@pytest.mark.parametrize("shard_map", [0, 1])
def test_frames_shards(gpu, shard_map, order):
    """Shard 1 of 3, interleaved and of the balanced plan.  The plan and the tile order are made once per launch, for
    all its frames; a probed plan depends on the probe's seed (frame 0's), so the balanced case installs a cost table
    (what an N-rank job does after its first gathered frame) and every render deals the same tiles."""
    sc, p = _scene("bunny_full", 64, 48, 32)
    p = replace(p, shard=1, num_shards=3, shard_map=shard_map, tile_w=8, tile_h=8, samples_per_stream=16)
    table = None
    if shard_map:
        rng = np.random.default_rng(5)
        table = rng.integers(1, 1 << 20, size=(2, 48), dtype=np.uint32)
    with gpu.DeviceScene(sc) as ds:
        _assert_same(*_frames_vs_singles(ds, p, 5, table, order))


def test_frames_against_oracle(gpu):
    """Frame 2 of a 3-frame launch is the oracle's frame of seed + 2 B W H."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    sc, p = _scene("bunny_full", 40, 24, 12)
    p = replace(p, samples_per_stream=5, tile_w=8, tile_h=8)
    n = shard_slot_count(p)
    dev = torch.device("cuda", 0)
    with gpu.DeviceScene(sc) as ds:
        ds.reserve_frames(p, 3)
        out = torch.zeros(3 * 3 * n, dtype=torch.float64, device=dev)
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
        ds.render_frames_device(p, 3, out, ctr)
        torch.cuda.synchronize()
        shard = out[2 * 3 * n:3 * 3 * n].cpu().numpy()
    q = replace(p, seed=p.seed + 2 * _nbatch(p) * p.width * p.height)
    ref, _, _ = oracle_render(sc, q, threads=8)
    from rtpotato.render import unpack_shard
    rgb = unpack_shard(q, shard)
    assert_parity(compare(rgb, ref))


def test_frames_spp0_and_errors(gpu):
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    sc, p = _scene("two_balls", 16, 16, 0)
    n = shard_slot_count(p)
    dev = torch.device("cuda", 0)
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
    with gpu.DeviceScene(sc) as ds:
        out = torch.zeros(2 * 3 * n, dtype=torch.float64, device=dev)
        ds.render_frames_device(p, 2, out, ctr)
        torch.cuda.synchronize()
        assert torch.isnan(out).all()
        q = replace(p, spp=8, samples_per_stream=2)
        with pytest.raises(F.RPError):
            ds.render_frames_device(q, 0, out, ctr)
        with pytest.raises(F.RPError):
            ds.render_frames_device(q, 2, out, ctr, order=4)
        with pytest.raises(F.RPError):
            ds.render_frames_device(q, F.RP_MAX_FRAMES + 1, torch.zeros(3 * n * 65, dtype=torch.float64, device=dev), ctr)
        ds.reserve(q)  # one frame's batch sums: two frames do not fit
        with pytest.raises(F.RPError, match="rp_workspace_reserve_frames"):
            ds.render_frames_device(q, 2, out, ctr)


def test_frame_info_flags(gpu):
    """rp_workspace_frame_info: a workspace's first frame probes its tile costs (RP_FRAME_PROBED), the next frame of the
    same geometry schedules from the learned table (RP_FRAME_LEARNED_ORDER) without a probe, and a render that launches
    nothing -- spp = 0, a refused call -- reports no scheduling at all (the flags are reset before any
    return)."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato.scene import shard_slot_count
    sc, p = _scene("bunny_full", 64, 48, 4)
    p = replace(p, tile_w=16, tile_h=16)
    n = shard_slot_count(p)
    dev = torch.device("cuda", 0)
    out = torch.zeros(3 * n, dtype=torch.float64, device=dev)
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
    with gpu.DeviceScene(sc) as ds:
        w = ds.workspace()
        ds.render_device(p, out, ctr, workspace=w)
        assert ds.frame_info(w) == F.RP_FRAME_PROBED
        ds.render_device(p, out, ctr, workspace=w)
        assert ds.frame_info(w) == F.RP_FRAME_LEARNED_ORDER
        ds.render_device(replace(p, spp=0), out, ctr, workspace=w)
        assert ds.frame_info(w) == 0
        ds.render_device(p, out, ctr, workspace=w)
        assert ds.frame_info(w) == F.RP_FRAME_LEARNED_ORDER
        with pytest.raises(F.RPError):
            ds.render_device(replace(p, max_bounce=0), out, ctr, workspace=w)
        assert ds.frame_info(w) == 0
        torch.cuda.synchronize()
        w.close()


@pytest.mark.parametrize("shard,sps", [(None, 256), (None, 0), (3, 0)])
def test_frames_c3_full_size(gpu, shard, sps):
    """bench.py's workloads at full size: C3 (1920x1080x256) rendered 8 frames to a launch in the interleaved order with
    the default queue chunks, under SURVEY.md 8c's one stream per pixel (the N = 1 headline) and in 32-sample streams --
    each of the launch's frames equals its lone render (seed + f B W H) bit for bit, with the summed counts; also shard 3
    of an 8-way balanced deal (the N = 8 per-rank work) under an installed cost table (as every rank holds one after its
    first gathered frame).  The lone renders are themselves oracle-checked at this size (test_gpu_configs.py)."""
    from rtpotato import scenes
    scene, params = scenes.config_scene("C3")
    params = replace(params, samples_per_stream=sps)
    table = None
    if shard is not None:
        n_tiles = -(-params.width // params.tile_w) * -(-params.height // params.tile_h)
        table = np.random.default_rng(11).integers(1, 1 << 20, size=(2, n_tiles), dtype=np.uint32)
        params = replace(params, shard=shard, num_shards=8, shard_map=1)
    with gpu.DeviceScene(scene) as ds:
        multi, single, mfg, sfg, ctr, sctr = _frames_vs_singles(ds, params, 8, table)
    _assert_same(multi, single, mfg, sfg, ctr, sctr)
    px = params.width * params.height // (1 if shard is None else 8)
    assert abs(int(ctr[2]) - 8 * px) <= 8 * 1024 and ctr[1] == 256 * ctr[2]  # every pixel of every frame, 256 samples
    if shard is None:
        assert ctr[2] == 8 * px


@pytest.mark.parametrize("opt", [{"node_format": "q8"}, {"node_format": "w8"}, {"lds_depth": 8},
                                 {"unit_queues": "single"}, {"tile_order": "morton"}])
def test_frames_node_formats_and_options(gpu, opt):
    """Every node format (q8: the large-scene kernel, whose hits carry no material out of the traversal; w8), the
    spilled stack, one device-wide queue and Z-order tiles: 3 interleaved frames per launch equal their lone renders."""
    sc, p = _scene("bunny_full", 64, 40, 24)
    with gpu.DeviceScene(sc, options=opt) as ds:
        _assert_same(*_frames_vs_singles(ds, replace(p, samples_per_stream=8, tile_w=16, tile_h=16), 3))


def test_frames_lens_camera(gpu):
    """three_balls (lens_radius 0.1: the UnitDisk draw moves the camera ray) and the catalogue's texture scenes."""
    for name in ("three_balls", "more_balls"):
        sc, p = _scene(name, 48, 32, 16)
        with gpu.DeviceScene(sc) as ds:
            _assert_same(*_frames_vs_singles(ds, replace(p, samples_per_stream=4), 4))


@pytest.mark.parametrize("sps", [8, 0])
def test_frames_gather_equals_per_frame_gathers(gpu, sps):
    """rp_frames_gather (one all-gather for a launch's frames) on a one-rank RCCL communicator: the n assembled BGRA8
    frames equal rp_frame_gather's of each frame's shard, byte for byte, and the counters are the launch's; without a
    frame buffer it still gathers the counters; an unreserved workspace is refused."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato.render import Comm, comm_unique_id
    from rtpotato.scene import shard_slot_count
    sc, p = _scene("bunny_full", 72, 40, 24)
    p = replace(p, samples_per_stream=sps, tile_w=16, tile_h=16)
    n = shard_slot_count(p)
    dev = torch.device("cuda", 0)
    nf = 3
    with gpu.DeviceScene(sc) as ds, Comm(comm_unique_id(), 1, 0, 0) as comm:
        w = ds.workspace()
        ds.reserve_frames(p, nf, w)
        shards = torch.zeros(3 * n * nf, dtype=torch.float64, device=dev)
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
        ds.render_frames_device(p, nf, shards, ctr, workspace=w)
        c_launch = ctr.clone()
        frames = torch.zeros(4 * p.width * p.height * nf, dtype=torch.uint8, device=dev)
        ds.frames_gather(comm, p, nf, shards, frames_bgra=frames, counters=ctr, workspace=w)
        one = torch.zeros(4 * p.width * p.height, dtype=torch.uint8, device=dev)
        c1 = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device=dev)
        per = []
        for f in range(nf):
            ds.frame_gather(comm, p, shards[3 * n * f:3 * n * (f + 1)], frame_bgra=one, counters=c1, workspace=w)
            torch.cuda.synchronize()
            per.append(one.cpu().numpy().copy())
        c2 = c_launch.clone()
        ds.frames_gather(comm, p, nf, shards, counters=c2, workspace=w)
        torch.cuda.synchronize()
        got = frames.cpu().numpy().reshape(nf, -1)
        for f in range(nf):
            assert np.array_equal(got[f], per[f]), f
        assert ctr.cpu().tolist() == c_launch.cpu().tolist() == c2.cpu().tolist()
        assert len(set(bytes(x) for x in got)) == nf  # different seeds: different frames
        w2 = ds.workspace()
        ds.reserve(p, w2)
        ds.render_frames_device(p, 1, shards, ctr, workspace=w2)
        with pytest.raises(F.RPError, match="rp_workspace_reserve_frames"):
            ds.frames_gather(comm, p, nf, shards, frames_bgra=frames, counters=ctr, workspace=w2)
        w2.close()
        w.close()
