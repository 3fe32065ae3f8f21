"""GPU parity at the BASELINE.json workloads the small tests do not reach, and the ABI around them.

C4 (the C3 scene at 1920x1080x1024 spp, tile-sharded 8 ways) and C5 (10 M random triangles at 4096x4096,
device-built LBVH + the spilling traversal stack) run at their real sizes on the GPU; the oracle re-renders
a sampled subset of tiles (per-pixel seeding makes any pixel subset comparable), and
size-independent properties cover the rest of the frame.  Also: the RNG contract's samples_per_stream
parameter (one stream per pixel), the no-allocation rule of the asynchronous calls, and the
multi-GPU entry points (rp_comm / rp_frame_gather / rp_render_gather / rp_multi) on a one-rank
communicator, bit for bit against rp_render.
"""
from dataclasses import replace

import numpy as np
import pytest

from test_gpu_parity import _sampled_shard_parity
from parity import TOL_LINF, assert_parity, compare, oracle_render, shard_mask

pytestmark = pytest.mark.gpu


@pytest.mark.slow
@pytest.mark.parametrize("shard", [0, 5])
def test_c4_shard_of_8(gpu, shard):
    """Config C4, shard `shard` of 8 at full size: 1024 spp = 32 RNG streams of 32 samples per pixel.
    (1) The oracle re-renders the shard's tiles t with t % 512 == shard (4 tiles x 1024 px x 1024 spp).
    (2) Every pixel of the shard is the batch-ordered sum of its 32 single-stream 32-spp frames (seed + b*W*H,
    x 32 -- exact, a power of two) / 1024: the multi-batch reduce at its real size, bit for bit."""
    from rtpotato import scenes
    scene, params = scenes.config_scene("C4")
    assert (params.width, params.height, params.spp) == (1920, 1080, 1024)
    W, H = params.width, params.height
    p = replace(params, shard=shard, num_shards=8)
    mask = shard_mask(p)
    with gpu.DeviceScene(scene) as ds:
        rgb, _, st = ds.render(p)
        assert st["pixels"] == mask.sum() and st["samples"] == mask.sum() * 1024
        acc = np.zeros_like(rgb)
        rays = 0
        for b in range(32):
            part, _, sb = ds.render(replace(p, spp=32, seed=params.seed + b * W * H))
            acc = acc + part * 32.0
            rays += sb["rays"]
    assert rays == st["rays"]
    assert np.array_equal(rgb[mask], (acc / 1024.0)[mask])
    sub = replace(params, shard=shard, num_shards=512)
    m = shard_mask(sub)
    assert m.sum() >= 3 * 1024 and not (m & ~mask).any()
    _sampled_shard_parity(gpu, scene, rgb, sub)


@pytest.mark.slow
def test_c5_10m_triangles(gpu):
    """Config C5 at its real size and sample count -- 10 M random triangles, 4096x4096 at 256 spp (8 RNG batches per
    pixel: the 3.7 GB batch-sum workspace, the q8 kernel's 4-block keystream ring wrapping) -- through the default
    tree (the AUTO builder: the device PLOC build at this size, 64 B quantized nodes) and the spilling traversal
    stack.  The oracle's reference median-split tree over all 10 M triangles re-renders 2 sampled tiles at 256 spp
    (parity bar, and exact ray counts against the GPU's re-render of the same tiles); 20 k rays are intersected ray
    by ray over the default tree, the device LBVH in both node formats, the host SAH tree and the host 8-wide tree."""
    from oracle import oracle_py as O
    from rtpotato import scenes
    scene, params = scenes.config_scene("C5")
    assert (params.width, params.height, params.spp) == (4096, 4096, 256)
    rng = np.random.default_rng(11)
    n = 20000
    o = np.concatenate([rng.uniform(-0.3, 0.3, size=(n, 2)), np.full((n, 1), 3.5)], axis=1)
    d = np.concatenate([rng.uniform(-1.2, 1.2, size=(n, 2)), np.full((n, 1), -3.5)], axis=1) - o * [1, 1, 0]
    rays = np.concatenate([o, d, np.full((n, 1), 1e-3), np.full((n, 1), np.inf)], axis=1)
    sub = replace(params, shard=5184, num_shards=8192)  # frame tiles 5184 and 13376 (inside the mesh), 256 spp
    m = shard_mask(sub)
    assert m.sum() == 2 * 1024
    with gpu.DeviceScene(scene) as ds:
        info = ds.info()
        assert info["prims"] == 10_000_000 and info["max_depth"] >= 12  # 43+ stack entries: the SPILL kernel
        bt = ds.build_times()
        assert bt["host_tree"] + bt["device_input"] + bt["device_build_or_upload"] < 5.0, bt  # PLOC, not host SAH
        rgb, _, st = ds.render(params)
        assert st["pixels"] == 4096 * 4096 and st["samples"] == 4096 * 4096 * 256 and np.isfinite(rgb).all()
        assert 1.0 < st["rays"] / st["samples"] < 8.0
        results = [ds.intersect(rays)]
        _sampled_shard_parity(gpu, scene, rgb, sub, ds=ds)
    for opt in ({"builder": "gpu", "node_format": "f32"}, {"builder": "gpu", "node_format": "q8"},
                {"builder": "host"}, {"node_format": "w8"}):  # w8: the host 8-wide tree
        with gpu.DeviceScene(scene, options=opt) as ds:
            results.append(ds.intersect(rays))
    desc = scene.desc()
    os_ = O.OracleScene(desc.addr(), desc)
    ref_hits, ref_mats, _ = os_.intersect(rays)
    hit = np.isfinite(ref_hits[:, 0])
    assert hit.sum() > n // 4
    for hits, mats in results:
        assert np.array_equal(np.isfinite(hits[:, 0]), hit)
        same = mats == ref_mats
        assert same.all()
        np.testing.assert_array_equal(hits[hit, :7], ref_hits[hit, :7])
    os_.close()


def test_one_stream_per_pixel_contract(gpu):
    """samples_per_stream = spp: SURVEY.md 8c's original contract (one StdRng per pixel, seed + j*W + i)
    for spp > 32 -- the GPU matches the oracle under it, and it differs from the default 32-sample batches."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.bunny_full(), 48, 30)
    p = RenderParams(48, 30, 64, 8, scenes.DEFAULT_SEED, samples_per_stream=64)
    rgb, _, st = gpu.render(sc, p)
    ref, _, ctr = oracle_render(sc, p, threads=16)
    assert_parity(compare(rgb, ref))
    assert st["rays"] == ctr["rays"]
    default, _, _ = gpu.render(sc, replace(p, samples_per_stream=0))
    assert not np.array_equal(rgb, default)
    # odd batch sizes: 64 spp in streams of 7 (a partial last batch of 1)
    p7 = replace(p, samples_per_stream=7)
    rgb7, _, st7 = gpu.render(sc, p7)
    ref7, _, ctr7 = oracle_render(sc, p7, threads=16)
    assert_parity(compare(rgb7, ref7))
    assert st7["rays"] == ctr7["rays"]


@pytest.mark.slow
def test_c3_one_stream_per_pixel_full_size(gpu):
    """SURVEY.md 8c's contract at a BASELINE config -- C3 (1920x1080x256) with samples_per_stream =
    256, i.e. ONE StdRng per pixel (seed + j*W + i) running the reference's per-pixel body (main.rs:70-86) over all
    256 samples.  The whole frame on the GPU; the oracle re-renders every 64th tile (shard 5 of 64) under the same
    contract: parity bar, and the GPU's re-render of that shard has the oracle's ray and sample counts exactly and is
    bitwise the full frame's pixels there."""
    from rtpotato import scenes
    scene, params = scenes.config_scene("C3")
    params = replace(params, samples_per_stream=256)
    with gpu.DeviceScene(scene) as ds:
        rgb, _, st = ds.render(params)
        assert st["pixels"] == params.width * params.height and st["samples"] == st["pixels"] * 256
        sub = replace(params, tile_w=32, tile_h=32, shard=5, num_shards=64)
        _sampled_shard_parity(gpu, scene, rgb, sub, ds=ds)
        default, _, sd = ds.render(replace(sub, samples_per_stream=0))
    m = shard_mask(sub)
    assert not np.array_equal(default[m], rgb[m])  # the 32-sample batches are a different (equally valid) stream set


@pytest.mark.slow
def test_c4_balanced_shard_against_oracle(gpu):
    """the deal N > 1 runs (RP_SHARD_BALANCED, bench.py's default for N > 1) at C4's full size
    (1920x1080x1024): shard 3 of 8 of a balanced plan renders its planned tiles, and the oracle re-renders the
    interleave-of-512 shard that shares the most tiles with it -- the shared pixels meet the parity bar, and the
    GPU's re-render of that oracle shard has the oracle's ray and sample counts exactly and the balanced shard's
    pixels bit for bit."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.scene import shard_slot_pixels
    scene, params = scenes.config_scene("C4")
    p = replace(params, shard=3, num_shards=8, shard_map=F.RP_SHARD_BALANCED)
    with gpu.DeviceScene(scene) as ds:
        rgb, _, st = ds.render(p)
        order = ds.tile_map(p)
        n_tiles = len(order)
        assert not np.array_equal(order, np.arange(n_tiles))
        mine = set(int(t) for t in order[3::8])
        s = max(range(512), key=lambda s: sum(t in mine for t in range(s, n_tiles, 512)))
        sub = replace(params, shard=s, num_shards=512)
        pix = shard_slot_pixels(p, order)
        m_bal = np.zeros(params.width * params.height, dtype=bool)
        m_bal[pix[pix >= 0]] = True
        m_bal = m_bal.reshape(params.height, params.width)
        assert st["pixels"] == m_bal.sum() and st["samples"] == m_bal.sum() * 1024
        m = m_bal & shard_mask(sub)
        assert m.sum() >= 1024
        ref, _, ctr = oracle_render(scene, sub, threads=16)
        assert_parity(compare(rgb, ref, m))
        sub_rgb, _, sst = ds.render(sub)
    assert np.array_equal(sub_rgb[m], rgb[m])
    assert (sst["rays"], sst["samples"]) == (ctr["rays"], ctr["samples"]), (sst, ctr)


def test_shards_of_2_31_units_are_refused(gpu):
    """The unit decode divides by launch constants with 31-bit multiply-shift magic numbers (rp_kernel.h make_div32,
    rp_device.h fetch_pixel), so rp_api.cpp refuses a shard of 2^31 or more (pixel, sample batch) units with RP_EINVAL
    before anything is launched: here 8192 x 8192 pixels x 32 batches of 32 samples on one unit queue (per-XCD queues
    hit the 2^32 queue-word limit first)."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.scene import RenderParams, shard_slot_count
    sc = scenes.configure(scenes.bunny_full(), 8192, 8192)
    p = RenderParams(8192, 8192, 1024, 8, 3)
    out = torch.zeros(3 * shard_slot_count(p), dtype=torch.float64, device="cuda")
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
    with gpu.DeviceScene(sc, options={"unit_queues": "single"}) as ds:
        with pytest.raises(F.RPError) as e:
            ds.render_device(p, out, ctr)
        assert e.value.code == F.RP_EINVAL and "2^31" in str(e.value)
    del out


def test_async_render_needs_reservation(gpu):
    """rp_render_device never allocates: a multi-batch frame without rp_workspace_reserve is refused with
    RP_EINVAL (nothing launched); after the reservation it renders the rp_render image bit for bit."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.render import unpack_shard
    from rtpotato.scene import RenderParams, shard_slot_count
    sc = scenes.configure(scenes.bunny_full(), 40, 24)
    p = RenderParams(40, 24, 70, 8, 3)
    n = shard_slot_count(p)
    out = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
    with gpu.DeviceScene(sc) as ds:
        with pytest.raises(F.RPError) as e:
            ds.render_device(p, out, ctr)
        assert e.value.code == F.RP_EINVAL and "reserve" in str(e.value)
        ds.reserve(p)
        ds.render_device(p, out, ctr)
        torch.cuda.synchronize()
        ref, _, st = ds.render(p)
    assert np.array_equal(unpack_shard(p, out.cpu().numpy()), ref)
    assert int(ctr[0]) == st["rays"] and int(ctr[3]) == 0


def test_single_rank_comm_gather(gpu):
    """rp_comm on one rank (RCCL over a 1-rank communicator): rp_render_gather's f64 frame equals rp_render
    bit for bit, its BGRA8 frame is to_srgb_u8 of it in tga::save order, and rp_frame_gather over a shard
    from rp_render_device_ws gives the same frames; counters are the render's (sum over one rank)."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.render import Comm, comm_unique_id
    from rtpotato.scene import RenderParams, shard_slot_count
    sc = scenes.configure(scenes.bunny_full(), 70, 45)
    p = RenderParams(70, 45, 40, 8, 21, 16, 16)
    npx = p.width * p.height
    with gpu.DeviceScene(sc) as ds, Comm(comm_unique_id(), 1, 0, 0) as comm:
        ref, _, st = ds.render(p)
        ds.reserve(p)
        bgra = torch.zeros(4 * npx, dtype=torch.uint8, device="cuda")
        frame = torch.zeros(3 * npx, dtype=torch.float64, device="cuda")
        ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
        ds.render_gather(comm, p, frame_bgra=bgra, frame_rgb=frame, counters=ctr)
        torch.cuda.synchronize()
        got = frame.cpu().numpy().reshape(p.height, p.width, 3)
        assert np.array_equal(got, ref)
        assert int(ctr[0]) == st["rays"] and int(ctr[1]) == st["samples"] and int(ctr[3]) == 0
        rgba = np.zeros((p.height, p.width, 4), dtype=np.uint8)
        F.host().rph_to_srgb_u8(np.ascontiguousarray(ref).ctypes.data, npx, rgba.ctypes.data)
        assert np.array_equal(bgra.cpu().numpy().reshape(p.height, p.width, 4), rgba[..., [2, 1, 0, 3]])
        # rp_frame_gather over a caller-owned shard rendered in a second workspace
        ws = ds.workspace()
        ds.reserve(p, ws)
        shard = torch.zeros(3 * shard_slot_count(p), dtype=torch.float64, device="cuda")
        ds.render_device(p, shard, ctr, workspace=ws)
        frame2 = torch.zeros_like(frame)
        ds.frame_gather(comm, p, shard, frame_rgb=frame2, workspace=ws)
        torch.cuda.synchronize()
        assert torch.equal(frame2, frame)
        with pytest.raises(F.RPError):  # the params must name this rank's shard of the communicator
            ds.frame_gather(comm, replace(p, shard=0, num_shards=2), shard, frame_rgb=frame2, workspace=ws)


def test_multi_single_device(gpu):
    """rp_multi (one process driving a device list) over device 0: the frame and its bytes equal rp_render's."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.render import MultiScene
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.bunny_full(), 64, 40)
    p = RenderParams(64, 40, 36, 8, 5)
    ref, _, st = gpu.render(sc, p)
    with MultiScene(sc, [0]) as ms:
        rgb, bgra, mst = ms.render(p, bgra=True)
    assert np.array_equal(rgb, ref)
    assert mst["rays"] == st["rays"] and mst["pixels"] == 64 * 40
    rgba = np.zeros((p.height, p.width, 4), dtype=np.uint8)
    F.host().rph_to_srgb_u8(np.ascontiguousarray(ref).ctypes.data, p.width * p.height, rgba.ctypes.data)
    assert np.array_equal(bgra, rgba[..., [2, 1, 0, 3]])
    with pytest.raises(F.RPError):
        MultiScene(sc, [0, 0])


@pytest.mark.parametrize("world", [3, 8])
def test_frame_assemble_multi_rank_layout(gpu, world):
    """rp_frame_assemble (the de-interleave step of every multi-GPU frame) with `world` ranks' shard buffers,
    all rendered on this one GPU and laid out as an all-gather leaves them (rank r at r * rp_gather_stride):
    f64 frame equal to the single-device rp_render, BGRA8 bytes equal to to_srgb_u8 of it, and both equal to
    the NumPy restatement (rtpotato.dist.assemble_frame) the CPU gloo tests use."""
    import ctypes
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.dist import assemble_frame, max_slots, shard_params
    from rtpotato.scene import RenderParams, shard_slot_count
    sc = scenes.configure(scenes.bunny_full(), 90, 50)
    p = RenderParams(90, 50, 6, 8, 13, 16, 8)
    stride = ctypes.c_uint64()
    F.check(F.rp().rp_gather_stride(ctypes.byref(shard_params(p, 0, world).to_c()), ctypes.byref(stride)))
    assert stride.value == max_slots(p, world)
    S = stride.value
    ref, _, _ = gpu.render(sc, p)
    gathered = torch.zeros(world * S * 3, dtype=torch.float64, device="cuda")
    gbgra = torch.zeros(world * S * 4, dtype=torch.uint8, device="cuda")
    ctr = torch.zeros(F.RP_COUNTERS_LEN, dtype=torch.int64, device="cuda")
    with gpu.DeviceScene(sc) as ds:
        for r in range(world):
            sp = shard_params(p, r, world)
            n = shard_slot_count(sp)
            ds.render_device(sp, gathered[r * S * 3:(r * S + n) * 3], ctr)
            ds.to_bgra8(sp, gathered[r * S * 3:(r * S + n) * 3], gbgra[r * S * 4:(r * S + n) * 4])
    frame = torch.zeros(p.width * p.height * 3, dtype=torch.float64, device="cuda")
    frame8 = torch.zeros(p.width * p.height * 4, dtype=torch.uint8, device="cuda")
    pc = shard_params(p, 0, world).to_c()
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    F.check(F.rp().rp_frame_assemble(ctypes.byref(pc), gathered.data_ptr(), 6, frame.data_ptr(), s))
    F.check(F.rp().rp_frame_assemble(ctypes.byref(pc), gbgra.data_ptr(), 1, frame8.data_ptr(), s))
    torch.cuda.synchronize()
    got = frame.cpu().numpy().reshape(p.height, p.width, 3)
    assert np.array_equal(got, ref)
    assert np.array_equal(got, assemble_frame(gathered.cpu().numpy().reshape(-1, 3), p, world))
    rgba = np.zeros((p.height, p.width, 4), dtype=np.uint8)
    F.host().rph_to_srgb_u8(np.ascontiguousarray(ref).ctypes.data, p.width * p.height, rgba.ctypes.data)
    assert np.array_equal(frame8.cpu().numpy().reshape(p.height, p.width, 4), rgba[..., [2, 1, 0, 3]])


