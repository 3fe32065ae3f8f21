"""GPU parity: librp.so (HIP, gfx950) against the CPU oracle on identical inputs and RNG seeding.

Bar (BASELINE.json north_star): per-pixel linear-RGB L-inf < 1e-3.  Ray counts must match exactly
(same paths); the fraction of pixels agreeing to 1e-12 is asserted as well (a path divergence shows
up as an O(1/spp) pixel error, far above 1e-12).
"""
import ctypes

import numpy as np
import pytest

from parity import TOL_LINF, assert_parity, compare, oracle_render, shard_mask

pytestmark = pytest.mark.gpu


def _scene(name, w, h, spp, **kw):
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.CATALOGUE[name](**kw), w, h)
    return sc, RenderParams(w, h, spp, 8, scenes.DEFAULT_SEED)


def _sampled_shard_parity(gpu, scene, full_rgb, sub, ds=None):
    """Full-size frame check on a sampled shard `sub`: the oracle renders the shard; the GPU frame's
    pixels there must meet the parity bar (no one-sided NaN, L-inf < 1e-3, >= 99.9 % exact); the GPU re-renders
    the same shard on its own -- bitwise the full frame's pixels -- and its ray and sample counts equal the
    oracle's exactly (the same paths, counted per root scene.hit, render.rs:105,133)."""
    ref, _, ctr = oracle_render(scene, sub, threads=16)
    m = shard_mask(sub)
    assert_parity(compare(full_rgb, ref, m))
    sub_rgb, _, sst = ds.render(sub) if ds is not None else gpu.render(scene, sub)
    assert np.array_equal(sub_rgb[m], full_rgb[m])
    assert (sst["rays"], sst["samples"], sst["pixels"]) == (ctr["rays"], ctr["samples"], int(m.sum())), (sst, ctr)
    return ctr


def _check(gpu, scene, params, min_exact=0.999, foreground=True, options=None):
    rgb, fg, st = gpu.render(scene, params, foreground=foreground, options=options)
    ref, ref_fg, ctr = oracle_render(scene, params, threads=8, foreground=foreground)
    mask = shard_mask(params)
    c = compare(rgb, ref, mask)
    assert c["nan_mismatch"] == 0, c
    assert c["linf"] < TOL_LINF, c
    assert c["exact_frac"] >= min_exact, c
    assert st["samples"] == ctr["samples"], (st, ctr)
    assert st["rays"] == ctr["rays"], (st, ctr)
    if foreground:
        assert np.array_equal(fg[mask], ref_fg[mask])
    return c, st


def test_c1_bunny_config(gpu):
    """Config C1: example_scenes.rs bunny(), 320x180, 4 spp -- the reference's own CPU-runnable case."""
    from rtpotato import scenes
    scene, params = scenes.config_scene("C1")
    c, st = _check(gpu, scene, params)
    assert st["pixels"] == 320 * 180


@pytest.mark.parametrize("name", ["three_balls", "more_balls", "more_balls_optimized", "two_balls", "earth",
                                  "one_triangle", "glass_bunny", "bunny", "bunny_lambert", "bunny_full", "variants",
                                  "variants_sky"])
def test_catalogue_scenes(gpu, name):
    """Every scene of example_scenes.rs, the C2/C3 material sets, and the two variant scenes: together every
    Scatter (None/Lambert/Metal/Dielectric), Absorb (Black/White/Albedo/AlbedoMap), Emit (None background in
    `variants`, DebugNormals, Color in `variants`, SkyGradient, SkySphere over Image / DebugUVs / Perlin) and
    Texture kind (Missing, DebugUVs, Solid, Image, Checker, Noise, Perlin); List and Bvh roots; lens sampling
    (three_balls, more_balls)."""
    scene, params = _scene(name, 64, 36, 4)
    _check(gpu, scene, params)


def test_c3_materials_more_spp(gpu):
    scene, params = _scene("bunny_full", 96, 54, 16)
    _check(gpu, scene, params)


def test_odd_sizes_and_tiles(gpu):
    """Ragged edge tiles, tiny frames, non-square tiles."""
    from rtpotato.scene import RenderParams
    from rtpotato import scenes
    for (w, h, tw, th) in [(1, 1, 32, 32), (37, 23, 8, 16), (70, 5, 32, 4)]:
        sc = scenes.configure(scenes.bunny_full(), w, h)
        p = RenderParams(w, h, 3, 8, 12345, tw, th)
        _check(gpu, sc, p)


@pytest.mark.parametrize("name", ["three_balls", "bunny_full"])
@pytest.mark.parametrize("spp", [1, 2, 3])
def test_small_spp(gpu, name, spp):
    """Fewer than 4 samples: a pixel's whole stream can end inside keystream block 0, so the next pixel
    on the same lane must not reuse any cached block (three_balls samples a lens)."""
    scene, params = _scene(name, 72, 40, spp)
    _check(gpu, scene, params)


@pytest.mark.parametrize("spp", [65, 130])
def test_multi_batch_streams(gpu, spp):
    """spp > RP_SAMPLES_PER_STREAM: one RNG stream per (pixel, batch of 32), batches on different lanes,
    sums reduced in batch order -- a partial last batch (65 = 2 x 32 + 1, 130 = 4 x 32 + 2)."""
    scene, params = _scene("bunny_full", 40, 24, spp)
    _check(gpu, scene, params)


def test_multi_batch_shards_bitwise(gpu):
    """Batched frames shard like single-stream ones: shards reassemble into the full frame bit for bit."""
    from rtpotato.scene import RenderParams
    from rtpotato import scenes
    sc = scenes.configure(scenes.bunny_full(), 50, 30)
    full, _, st_full = gpu.render(sc, RenderParams(50, 30, 70, 8, 3, 16, 16))
    acc = np.zeros_like(full)
    with gpu.DeviceScene(sc) as ds:
        for s in range(2):
            p = RenderParams(50, 30, 70, 8, 3, 16, 16, s, 2)
            part, _, _ = ds.render(p)
            m = shard_mask(p)
            acc[m] = part[m]
    assert np.array_equal(acc, full)
    assert st_full["pixels"] == 50 * 30


def test_max_bounce_variants(gpu):
    from rtpotato.scene import RenderParams
    from rtpotato import scenes
    sc = scenes.configure(scenes.bunny_full(), 48, 27)
    for mb in (1, 2, 3, 16):
        _check(gpu, sc, RenderParams(48, 27, 2, mb, 99))


def test_shards_cover_frame_bitwise(gpu):
    """Per-pixel seeding: shards rendered separately reassemble into the unsharded frame bit for bit."""
    from rtpotato.scene import RenderParams
    from rtpotato import scenes
    sc = scenes.configure(scenes.bunny_full(), 100, 60)
    full, _, st_full = gpu.render(sc, RenderParams(100, 60, 4, 8, 7, 16, 16))
    acc = np.zeros_like(full)
    rays = 0
    with gpu.DeviceScene(sc) as ds:
        for s in range(3):
            part, _, st = ds.render(RenderParams(100, 60, 4, 8, 7, 16, 16, s, 3))
            m = shard_mask(RenderParams(100, 60, 4, 8, 7, 16, 16, s, 3))
            acc[m] = part[m]
            rays += st["rays"]
    assert np.array_equal(acc, full)
    assert rays == st_full["rays"]


def test_determinism(gpu):
    from rtpotato import scenes
    scene, params = _scene("bunny_full", 80, 45, 8)
    with gpu.DeviceScene(scene) as ds:
        a, _, sa = ds.render(params)
        b, _, sb = ds.render(params)
    assert np.array_equal(a, b) and sa["rays"] == sb["rays"]


def test_spp_zero_is_nan_and_bad_bounce_rejected(gpu):
    """main.rs:86 divides by num_samples: 0 spp gives NaN pixels; depth 0 trips render.rs:97's assert."""
    from rtpotato.scene import RenderParams
    from rtpotato import _ffi as F
    scene, _ = _scene("bunny", 8, 8, 1)
    with gpu.DeviceScene(scene) as ds:
        rgb, _, st = ds.render(RenderParams(8, 8, 0, 8, 1))
        assert np.isnan(rgb).all() and st["rays"] == 0
        with pytest.raises(F.RPError) as e:
            ds.render(RenderParams(8, 8, 1, 0, 1))
        assert e.value.code == F.RP_EINVAL


def test_render_device_torch(gpu):
    """rp_render_device on torch's current stream into torch tensors; counters on the device."""
    import torch
    from rtpotato import scenes
    from rtpotato.scene import shard_slot_count
    from rtpotato.render import unpack_shard
    scene, params = _scene("bunny_full", 64, 40, 4)
    n = shard_slot_count(params)
    out = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
    with gpu.DeviceScene(scene) as ds:
        ds.render_device(params, out, ctr)
        torch.cuda.synchronize()
        frame = unpack_shard(params, out.cpu().numpy())
        ref, _, st = ds.render(params)
    assert np.array_equal(frame, ref)
    assert int(ctr[0]) == st["rays"] and int(ctr[3]) == 0


@pytest.mark.parametrize("fmt", ["f32", "q8", "w8"])
@pytest.mark.parametrize("builder", ["host", "gpu", "ploc"])
def test_intersect_rays(gpu, builder, fmt):
    """Hittable::hit on the root, ray by ray: t, position, normal, uv, material identical to the oracle --
    over the host SAH tree and the device-built LBVH and PLOC trees (rp_scene_options.builder), with f32 or 8-bit
    quantized child boxes, 4-wide or (host trees) 8-wide (rp_scene_options.node_format)."""
    from oracle import oracle_py as O
    from rtpotato import scenes
    from rtpotato import _ffi as F
    if builder != "host" and fmt == "w8":  # the device builders make 4-wide trees only: refused, not substituted
        with pytest.raises(F.RPError, match="4-wide"):
            gpu.DeviceScene(scenes.bunny_full(), options={"builder": builder, "node_format": "w8"})
        return
    rng = np.random.default_rng(5)
    scene = scenes.bunny_full()
    n = 20000
    o = rng.uniform(-2.5, 2.5, size=(n, 3))
    o[:, 1] = rng.uniform(-0.5, 2.5, size=n)
    target = rng.uniform(-0.8, 0.8, size=(n, 3)) + np.array([0.0, 0.7, 0.0])
    d = target - o
    rays = np.concatenate([o, d, np.full((n, 1), 1e-3), np.full((n, 1), np.inf)], axis=1)
    # edge cases: axis-parallel directions (infinite inverse components), finite t_max, origin on a slab
    rays[:200, 3:5] = 0.0
    rays[200:400, 4] = 0.0
    rays[400:600, 7] = rng.uniform(0.1, 3.0, size=200)
    rays[600:700, 0] = 0.0
    rays[600:700, 3] = 0.0
    with gpu.DeviceScene(scene, options={"builder": builder, "self_check": 1, "node_format": fmt}) as ds:
        hits, mats = ds.intersect(rays)
    d_ = scene.desc()
    os_ = O.OracleScene(d_.addr(), d_)
    ref, ref_mats, _ = os_.intersect(rays)
    hit = np.isfinite(ref[:, 0])
    assert hit.sum() > n // 4
    same_mat = mats == ref_mats
    # exact-t ties may legitimately pick a different primitive (tree shape is free); none expected here
    assert same_mat.mean() > 0.9999, np.nonzero(~same_mat)[0][:10]
    ok = same_mat
    assert np.array_equal(np.isfinite(hits[:, 0]), hit)
    assert np.array_equal(hits[ok & hit, 0], ref[ok & hit, 0])
    np.testing.assert_array_equal(hits[ok & hit, 1:7], ref[ok & hit, 1:7])
    assert np.max(np.abs(hits[ok & hit, 7:] - ref[ok & hit, 7:])) < 1e-12  # uv: OCML vs glibc atan2/asin


def test_random_mesh_deep_tree(gpu):
    """Config C5's scene type (random small triangles, Lambert, SkyGradient) at 200k triangles: a deep tree
    of many thin leaves, the HBM-bound traversal case, against the oracle's reference median-split tree."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.random_mesh(200_000), 64, 64)
    with gpu.DeviceScene(sc) as ds:
        assert ds.info()["max_depth"] >= 8
    _check(gpu, sc, RenderParams(64, 64, 4, 8, scenes.DEFAULT_SEED))


@pytest.mark.slow
def test_c2_full_size_sampled_parity(gpu):
    """Config C2 (Lambert bunny, SkyGradient, 1920x1080x64) at full size; the oracle re-renders every 64th
    tile (shard 9 of 64)."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    scene, params = scenes.config_scene("C2")
    rgb, _, st = gpu.render(scene, params)
    sub = RenderParams(params.width, params.height, params.spp, params.max_bounce, params.seed, 32, 32, 9, 64)
    _sampled_shard_parity(gpu, scene, rgb, sub)
    assert st["pixels"] == params.width * params.height


@pytest.mark.slow
def test_c3_full_size_sampled_parity(gpu):
    """Config C3 at full size (1920x1080x256): the whole frame on the GPU; the oracle re-renders every
    64th tile (shard 5 of 64) and those pixels must agree -- per-pixel seeding makes a shard of the
    oracle frame comparable to the same pixels of the GPU frame."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    scene, params = scenes.config_scene("C3")
    rgb, _, st = gpu.render(scene, params)
    sub = RenderParams(params.width, params.height, params.spp, params.max_bounce, params.seed, 32, 32, 5, 64)
    ctr = _sampled_shard_parity(gpu, scene, rgb, sub)
    assert st["pixels"] == params.width * params.height
    # size-independent property: rays per sample of the whole frame vs the sampled shard
    assert abs(st["rays"] / st["samples"] - ctr["rays"] / ctr["samples"]) < 0.25


def test_workspaces_frames_in_flight(gpu):
    """rp_render_device_ws: frames with two workspaces on two streams at once (70 spp, so the batch sums
    live in the workspaces as well) equal the scene-workspace frame bit for bit, with the same ray count."""
    import torch
    from rtpotato.scene import shard_slot_count
    scene, params = _scene("bunny_full", 64, 40, 70)
    n = shard_slot_count(params)
    with gpu.DeviceScene(scene) as ds:
        ref = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
        c0 = torch.zeros(4, dtype=torch.int64, device="cuda")
        ds.reserve(params)
        ds.render_device(params, ref, c0)
        torch.cuda.synchronize()
        wss = [ds.workspace(), ds.workspace()]
        for w in wss:
            ds.reserve(params, w)
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        outs = [torch.zeros_like(ref) for _ in range(4)]
        ctrs = [torch.zeros_like(c0) for _ in range(4)]
        for k in range(4):  # frames k and k + 2 share a workspace and its stream
            ds.render_device(params, outs[k], ctrs[k], stream=streams[k % 2], workspace=wss[k % 2])
        torch.cuda.synchronize()
        for k in range(4):
            assert torch.equal(outs[k], ref)
            assert int(ctrs[k][0]) == int(c0[0]) and int(ctrs[k][3]) == 0
        wss[0].close()  # explicit destroy before the scene; the other one is destroyed with the scene


@pytest.mark.parametrize("fmt", ["f32", "q8"])
@pytest.mark.parametrize("builder", ["gpu", "ploc"])
@pytest.mark.parametrize("name,arg", [("bunny_full", None), ("random_mesh", 200_000), ("three_balls", None),
                                      ("one_triangle", None)])
def test_device_bvh_builder(gpu, name, arg, fmt, builder):
    """Scenes over the device-built trees (rp_bvh_gpu.hip: LBVH or PLOC, then the wide collapse) in both node
    formats, with the host builder's structural self-check on the downloaded tree (options.self_check): same image
    and ray counts as the oracle."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    opt = {"builder": builder, "self_check": 1, "node_format": fmt}
    sc = scenes.configure(scenes.CATALOGUE[name](arg) if arg else scenes.CATALOGUE[name](), 64, 40)
    with gpu.DeviceScene(sc, options=opt) as ds:
        info = ds.info()
        assert info["nodes"] >= 1 and (info["max_depth"] >= 4 or name in ("three_balls", "one_triangle"))
    _check(gpu, sc, RenderParams(64, 40, 4, 8, scenes.DEFAULT_SEED), options=opt)


def test_ploc_line_aligned_node_families(gpu):
    """rp_scene_options.node_layout = RP_LAYOUT_DFS_LINE (ABI v7): the PLOC tree's 64-B quantized nodes laid out depth
    first with every family of inner children starting on a 128-B line (zero pad slots after odd families, never
    referenced).  More node slots than the packed layout, the structural self-check passes (it walks from the root),
    and the image and ray counts are the oracle's."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.random_mesh(200_000), 64, 40)
    nodes = {}
    for layout in ("dfs", "dfs_line"):
        opt = {"builder": "ploc", "node_format": "q8", "node_layout": layout, "self_check": 1}
        with gpu.DeviceScene(sc, options=opt) as ds:
            nodes[layout] = ds.info()["nodes"]
    assert nodes["dfs"] < nodes["dfs_line"] < 1.5 * nodes["dfs"], nodes
    _check(gpu, sc, RenderParams(64, 40, 4, 8, scenes.DEFAULT_SEED),
           options={"builder": "ploc", "node_format": "q8", "node_layout": "dfs_line"})


@pytest.mark.parametrize("builder", ["ploc", "gpu", "host"])
def test_nan_vertex_triangles_build_and_render(gpu, builder):
    """NaN geometry: a mesh with a run of adjacent triangles whose vertices are all NaN.  Their boxes sort
    together (Morton code 0), so PLOC's search window holds only NaN candidates; the nearest-neighbour pass ranks a NaN
    distance as +inf and still names a neighbour (it used to leave -1, which the flags pass then read out of bounds).
    The reference itself panics on such a mesh (bvh.rs:62 `partial_cmp().unwrap()` of a NaN centroid), so there is no
    image to match: every builder must build the tree and render the frame with a clean status."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.random_mesh(200_000), 32, 32)
    mesh = sc.scene_data.mesh_table[0]
    mesh.positions[3 * 1000:3 * 1012] = np.nan  # triangles 1000..1011
    with gpu.DeviceScene(sc, options={"builder": builder}) as ds:
        assert ds.info()["nodes"] >= 1
        rgb, _, st = ds.render(RenderParams(32, 32, 2, 8, scenes.DEFAULT_SEED))
    assert st["rays"] > 0 and st["pixels"] == 32 * 32 and rgb.shape == (32, 32, 3)


@pytest.mark.parametrize("fmt", ["f32", "q8"])
@pytest.mark.parametrize("collapse", ["greedy", "sah"])
def test_host_tree_collapse(gpu, collapse, fmt):
    """Both 4-wide collapses of the host SAH tree (rp_scene_options.collapse, rp_bvh.cpp CollapsePlan): the SAH-optimal
    cut gives the bunny fewer wide nodes than the greedy rule, and both render the oracle's image and ray counts."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    opt = {"builder": "host", "collapse": collapse, "node_format": fmt}
    sc = scenes.configure(scenes.bunny_full(), 64, 40)
    with gpu.DeviceScene(sc, options=opt) as ds:
        nodes = ds.info()["nodes"]
    assert (nodes < 1600) if collapse == "sah" else (nodes > 1600), nodes  # 1,451 vs 1,729 wide nodes
    _check(gpu, sc, RenderParams(64, 40, 6, 8, scenes.DEFAULT_SEED), options=opt)


@pytest.mark.parametrize("fmt", ["f32", "q8", "w8"])
@pytest.mark.parametrize("name,arg", [("bunny_full", None), ("random_mesh", 200_000)])
def test_spilled_traversal_stack(gpu, name, arg, fmt):
    """Traversal stack entries beyond the LDS part spill to the per-lane global run (the SPILL kernel that
    deep trees such as C5's use): forced here with options.lds_depth = 8 entries (the minimum), so deep traversals
    spill -- same image as the oracle."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.CATALOGUE[name](arg) if arg else scenes.CATALOGUE[name](), 64, 40)
    _check(gpu, sc, RenderParams(64, 40, 6, 8, scenes.DEFAULT_SEED), options={"lds_depth": 8, "node_format": fmt})


@pytest.mark.parametrize("fmt", ["f32", "q8"])
@pytest.mark.parametrize("name", ["bunny_full", "more_balls"])
def test_keystream_ring_sizes(gpu, name, fmt):
    """The keystream ring is a cache of the same stream: the f32-node kernel keeps 8 ChaCha12 blocks per lane
    ahead, the q8 kernel 4 in a compact slab (rp_kernel.hip RingFor).  At 40 spp (10 jitter blocks, many ring
    wraps) both give the oracle's image and ray counts."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.CATALOGUE[name](), 64, 40)
    _check(gpu, sc, RenderParams(64, 40, 40, 8, scenes.DEFAULT_SEED), options={"node_format": fmt})


@pytest.mark.parametrize("always_max", [0, 4])
def test_always_tested_primitives(gpu, always_max):
    """Primitives whose box dwarfs the rest of the scene (the C3 ground sphere) are kept out of the tree and
    tested first for every ray (options.always_max, the default 4); 0 puts them back in the tree.  Same
    image as the oracle either way, on the full-materials bunny scene (ground, two balls, bunny) and on
    two_balls (a scene of two spheres only)."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    for name in ("bunny_full", "two_balls"):
        sc = scenes.configure(scenes.CATALOGUE[name](), 64, 40)
        _check(gpu, sc, RenderParams(64, 40, 6, 8, scenes.DEFAULT_SEED), options={"always_max": int(always_max)})


@pytest.mark.parametrize("fmt", ["q8", "w8"])
@pytest.mark.parametrize("name", ["bunny_full", "more_balls", "two_balls", "earth", "variants"])
def test_quantized_nodes_scenes(gpu, name, fmt):
    """The quantized node formats (options.node_format: q8 = 64 B 4-wide, w8 = 128 B 8-wide) on the small
    catalogue scenes, whose default is the f32 format: same image and ray counts as the oracle."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.CATALOGUE[name](), 64, 40)
    _check(gpu, sc, RenderParams(64, 40, 6, 8, scenes.DEFAULT_SEED), options={"node_format": fmt})


def test_tile_orders_bitwise(gpu):
    """The unit queue's tile order (options.tile_order: plain row-major, cost-ordered by the probe launch,
    Z-order) changes the schedule only: the frames are identical bit for bit, sharded or not."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.bunny_full(), 96, 64)
    for p in (RenderParams(96, 64, 40, 8, 5, 16, 16), RenderParams(96, 64, 8, 8, 5, 8, 8, shard=1, num_shards=3)):
        frames = []
        for order in ("plain", "cost", "morton", "auto"):
            with gpu.DeviceScene(sc, options={"tile_order": order}) as ds:
                rgb, _, st = ds.render(p)
            frames.append((rgb, st["rays"]))
        for rgb, rays in frames[1:]:
            assert np.array_equal(rgb, frames[0][0]) and rays == frames[0][1]


@pytest.mark.parametrize("queues", [{"unit_queues": "single"}, {"unit_queues": "xcd_tiles"},
                                    {"unit_queues": "xcd_regions"}, {"unit_queues": "xcd_tiles", "queue_chunk": 3},
                                    {"unit_queues": "xcd_tiles", "queue_chunk": 1}])
def test_unit_queues_bitwise(gpu, queues):
    """options.unit_queues / queue_chunk (one device-wide unit queue, or one per XCD group of blocks serving
    every 8th tile, every 8th chunk of tiles or an eighth of the tile order, stealing once drained) changes the
    schedule only: identical frames --
    including frames with fewer tiles than queues, edge tiles outside the frame and multi-batch pixels."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.bunny_full(), 96, 64)
    for p in (RenderParams(96, 64, 40, 8, 5, 16, 16), RenderParams(96, 64, 8, 8, 5, 8, 8, shard=1, num_shards=3),
              RenderParams(70, 50, 3, 8, 5, 32, 32)):
        frames = []
        for q in ({"unit_queues": "single"}, queues):
            for order in ("cost", "morton"):
                with gpu.DeviceScene(sc, options={"tile_order": order, **q}) as ds:
                    rgb, _, st = ds.render(p)
                frames.append((rgb, st["rays"], st["pixels"]))
        for rgb, rays, px in frames[1:]:
            assert np.array_equal(rgb, frames[0][0]) and rays == frames[0][1] and px == frames[0][2]
