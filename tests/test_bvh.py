"""The device acceleration structure's builder (rp_bvh.cpp, CPU-only self-check through librp_host.so)
and scene validation: every index the reference would bounds-check is rejected before upload."""
import ctypes

import numpy as np
import pytest


FORMATS = [1, 2, 3]  # RP_NODES_F32, RP_NODES_Q8, RP_NODES_W8


def _selfcheck(scene, node_format=0):
    from rtpotato import _ffi as F
    d = scene.desc()
    st = (ctypes.c_uint64 * 4)()
    rc = F.host().rph_bvh_selfcheck(d.ptr(), node_format, st)
    return rc, list(st), (F.host().rph_last_error() or b"").decode()


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("name", ["bunny", "bunny_full", "glass_bunny", "three_balls", "more_balls", "two_balls",
                                  "earth", "one_triangle"])
def test_catalogue_trees_valid(name, fmt):
    """Both node formats: every stored child box (f32, or 8-bit planes in the node's frame) contains the
    exact f64 boxes of its subtree (rpb::check)."""
    from rtpotato import scenes
    rc, st, err = _selfcheck(scenes.CATALOGUE[name](), fmt)
    assert rc == 0, err
    nodes, leaves, depth, prims = st
    assert leaves >= 1 and prims == len(scenes.CATALOGUE[name]().root)


def test_bunny_tree_shape():
    """SAH with <= 4 primitives per leaf: far fewer nodes than the reference's 9,937 one-per-leaf nodes."""
    from rtpotato import scenes
    rc, (nodes, leaves, depth, prims), err = _selfcheck(scenes.bunny())
    assert rc == 0, err
    assert prims == 4969 and nodes < 4969 and depth < 40


@pytest.mark.parametrize("fmt", FORMATS)
def test_degenerate_geometry(fmt):
    """Coincident centroids (identical triangles) force the object-median fallback; a lone primitive
    becomes a root leaf next to an empty slot."""
    from rtpotato.scene import (Absorb, Emit, Hittable, Material, Mesh, Scatter, Scene, SceneData, hittables,
                                Camera, Transformation)
    cam = Camera(1.0, 1.0, 1.0, 0.0, Transformation.lookat((0, 0, 3), (0, 0, 0), (0, 1, 0)))
    mat = [Material.new(Scatter.Lambert, Absorb.Albedo((0.5, 0.5, 0.5)), Emit.None_)]
    n = 1000
    pos = np.tile(np.array([[0.0, 0, 0], [1, 0, 0], [0, 1, 0]]), (n, 1))
    mesh = Mesh(pos, np.zeros_like(pos), np.zeros((3 * n, 2)), np.arange(3 * n, dtype=np.uint32))
    sc = Scene(cam, SceneData(mat, [], [mesh]), Hittable.Triangle(mesh.iter_triangles(), 0), Emit.SkyGradient)
    rc, st, err = _selfcheck(sc, fmt)
    assert rc == 0, err
    one = Scene(cam, SceneData(mat, [], []), Hittable.Sphere((0, 0, 0), 1.0, 0), Emit.SkyGradient)
    rc, st, err = _selfcheck(one, fmt)
    assert rc == 0 and st[0] == 1 and st[1] == 1, (st, err)


@pytest.mark.parametrize("fmt", FORMATS)
def test_random_mesh_tree_valid(fmt):
    from rtpotato import scenes
    rc, st, err = _selfcheck(scenes.random_mesh(20000), fmt)
    assert rc == 0, err
    assert st[3] == 20000


@pytest.mark.parametrize("breakage", ["material", "mesh", "triangle", "texture", "checker_cycle", "bvh_empty",
                                      "vertex_index"])
def test_validation_rejects(breakage):
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.scene import Texture
    sc = scenes.bunny_full()
    if breakage == "material":
        sc.root["material"][-1] = 99
    elif breakage == "mesh":
        sc.root["mesh"][0] = 3
    elif breakage == "triangle":
        sc.root["triangle"][0] = 3 * 4968
    elif breakage == "texture":
        sc.background = type(sc.background)(sc.background.kind, texture=7)
    elif breakage == "checker_cycle":
        sc.scene_data.texture_table.append(Texture.Checker(2, 2))
    elif breakage == "bvh_empty":
        sc.root = sc.root[:0]
    elif breakage == "vertex_index":
        m = sc.scene_data.mesh_table[0]
        from rtpotato.scene import Mesh
        idx = m.indices.copy()
        idx[5] = 1 << 20
        sc.scene_data.mesh_table = [Mesh(m.positions, m.normals, m.uvs, idx)]
    rc, _, err = _selfcheck(sc)
    assert rc == F.RP_EINVAL and err, err


def test_list_root_with_no_hittables_is_valid():
    """hit_list over an empty list returns None (every ray sees the background)."""
    from rtpotato import scenes
    from rtpotato import _ffi as F
    sc = scenes.three_balls()
    sc.root = sc.root[:0]
    rc, st, err = _selfcheck(sc)
    assert rc == 0, err


def _rays_for(scene, n, seed, adversarial=True):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-2.5, 2.5, size=(n, 3))
    o[:, 1] = rng.uniform(-0.5, 2.5, size=n)
    d = rng.uniform(-0.8, 0.8, size=(n, 3)) + np.array([0.0, 0.7, 0.0]) - o
    rays = np.concatenate([o, d, np.full((n, 1), 1e-3), np.full((n, 1), np.inf)], axis=1)
    if adversarial:
        k = n // 10
        rays[:k, 3:5] = 0.0                       # axis-parallel (infinite inverse components)
        rays[k:2 * k, 4] = 0.0
        rays[2 * k:3 * k, 7] = rng.uniform(0.05, 3.0, size=k)  # finite t_max
        # origins exactly on box planes of the bunny's vertices
        m = scene.scene_data.mesh_table[0] if scene.scene_data.mesh_table else None
        if m is not None:
            v = m.positions[rng.integers(0, len(m.positions), size=k)]
            rays[3 * k:4 * k, 0:3] = v + np.array([0.0, 0.0, 1.0]) * rng.integers(0, 2, size=(k, 1))
            rays[3 * k:4 * k, 3:6] = rng.normal(size=(k, 3))
        # grazing rays along triangle edges
        if m is not None:
            idx = m.indices.reshape(-1, 3)[rng.integers(0, len(m.indices) // 3, size=k)]
            a, b = m.positions[idx[:, 0]], m.positions[idx[:, 1]]
            rays[4 * k:5 * k, 0:3] = a - 2.0 * (b - a)
            rays[4 * k:5 * k, 3:6] = b - a
    return rays


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("name", ["bunny_full", "more_balls", "one_triangle", "two_balls"])
def test_conservative_f32_traversal_finds_reference_hits(oracle, name, fmt):
    """The device traversal model (4-wide tree, conservative f32 child boxes or 8-bit quantized ones, fma
    slab form) returns the same closest primitive as the oracle's reference traversal (median-split tree,
    exact f64 boxes) on random and adversarial rays -- the stored boxes never cull a primitive the f64 test
    would hit."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    scene = scenes.CATALOGUE[name]()
    rays = _rays_for(scene, 40000, 3)
    d = scene.desc()
    out = np.zeros((len(rays), 3), dtype=np.uint64)
    F.check_host(F.host().rph_bvh_traversal_stats(d.ptr(), rays.ctypes.data, len(rays), fmt, out.ctypes.data))
    os_ = oracle.OracleScene(d.addr(), d)
    hits, mats, _ = os_.intersect(rays)
    ref_hit = np.isfinite(hits[:, 0])
    got_hit = out[:, 2] != np.uint64(2**64 - 1)
    bad = np.nonzero(ref_hit != got_hit)[0]
    k = len(rays) // 10
    # Everything agrees except rays constructed to run exactly along a mesh edge through two vertices
    # ([4k, 5k)): there the reference's per-primitive f64 box test can reject, by one rounding, a
    # corner-touching hit its exact triangle test accepts (the measure-zero case of SURVEY.md 8a A9).
    assert np.all((bad >= 4 * k) & (bad < 5 * k)), bad[:10]
    assert len(bad) <= k // 100, len(bad)
    assert ref_hit.sum() > 1000


def test_wide_tree_is_shallow():
    from rtpotato import _ffi as F
    from rtpotato import scenes
    import ctypes
    d = scenes.bunny_full().desc()
    st = (ctypes.c_uint64 * 4)()
    assert F.host().rph_bvh_selfcheck(d.ptr(), 0, st) == 0
    nodes, leaves, depth, prims = list(st)
    # 4 971 hittables: the 4-wide SAH tree (node cost 0.7 of a primitive test, rp_bvh.h) has ~1 700 nodes
    # at depth 8; the reference's binary median tree has 9 937 nodes at depth 14
    assert depth <= 12 and nodes < 2000, list(st)


@pytest.mark.parametrize("fmt", FORMATS)
def test_giant_primitives_tested_first(fmt):
    """The host builder keeps primitives whose box dwarfs the rest of the scene out of the tree and tests
    them first for every ray (rp_bvh.h BuildOptions::always_max): in the C3 scene the ground sphere
    (r = 1000) is tested by every ray, including rays that miss every box of the tree; in earth (one
    sphere, nothing to single out) a ray that misses the root tests nothing."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    for name, always in (("bunny_full", True), ("earth", False)):
        scene = scenes.CATALOGUE[name]()
        rays = _rays_for(scene, 2000, 9)
        rays[:1000, 3:6] = np.array([0.0, 1.0, 0.0])  # straight up: misses the bunny and both balls
        rays[:1000, 0:3] = np.array([0.0, 5.0, 0.0])
        d = scene.desc()
        out = np.zeros((len(rays), 3), dtype=np.uint64)
        F.check_host(F.host().rph_bvh_traversal_stats(d.ptr(), rays.ctypes.data, len(rays), fmt, out.ctypes.data))
        if always:
            assert (out[:, 1] >= 1).all()
        else:
            assert (out[:1000, 1] == 0).all()


def test_quantized_nodes_cost_few_extra_visits():
    """The 8-bit child boxes are rounded outward to a grid of 1/255 of the node's extent: the same closest hits,
    at most a few percent more node visits and primitive tests than the f32 boxes (bunny and a 200 k mesh)."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    for scene in (scenes.bunny_full(), scenes.random_mesh(200_000)):
        rays = _rays_for(scene, 20000, 5, adversarial=False)
        d = scene.desc()
        res = []
        for fmt in FORMATS:
            out = np.zeros((len(rays), 3), dtype=np.uint64)
            F.check_host(F.host().rph_bvh_traversal_stats(d.ptr(), rays.ctypes.data, len(rays), fmt, out.ctypes.data))
            res.append(out)
        assert (res[0][:, 2] == res[1][:, 2]).all()
        assert res[1][:, 0].mean() <= 1.05 * res[0][:, 0].mean()
        assert res[1][:, 1].mean() <= 1.10 * res[0][:, 1].mean()


def test_quantized_frames_refuse_huge_coordinates():
    """Node frames need |coordinate| <= 2^54 (rp_layout.h COORD_MAX): larger scenes are refused, not mis-culled."""
    from rtpotato import _ffi as F
    from rtpotato.scene import Camera, Emit, Hittable, Material, Scatter, Absorb, Scene, SceneData, Transformation
    cam = Camera(1.0, 1.0, 1.0, 0.0, Transformation.lookat((0, 0, 3), (0, 0, 0), (0, 1, 0)))
    mat = [Material.new(Scatter.Lambert, Absorb.Albedo((0.5, 0.5, 0.5)), Emit.None_)]
    far = Scene(cam, SceneData(mat, [], []), Hittable.Sphere((0, 0, 0), 1e17, 0), Emit.SkyGradient)
    rc, _, err = _selfcheck(far, 2)
    assert rc == F.RP_EINVAL and "2^54" in err
    for fmt in (0, 1):  # auto falls back to the f32 nodes
        rc, _, err = _selfcheck(far, fmt)
        assert rc == 0, err


@pytest.mark.parametrize("fmt", FORMATS)
def test_parallel_host_build_is_deterministic(fmt):
    """The host SAH build splits the top of the tree across threads and builds the subtrees on a pool; the
    spliced tree (node records, leaf order) is the single-threaded build's bit for bit."""
    from rtpotato import _ffi as F
    from rtpotato import scenes
    d = scenes.random_mesh(150_000).desc()
    hs = []
    for threads in (1, 3, 8):
        h = ctypes.c_uint64()
        F.check_host(F.host().rph_bvh_tree_hash(d.ptr(), fmt, threads, ctypes.byref(h)))
        hs.append(h.value)
    assert hs[0] == hs[1] == hs[2], hs


@pytest.mark.parametrize("fmt", [1, 2])  # RP_NODES_F32, RP_NODES_Q8 (the 8-wide collapse keeps its own rule)
def test_sah_collapse_cuts_node_visits(oracle, fmt):
    """rp_scene_options.collapse (rp_bvh.cpp CollapsePlan): the SAH-optimal cut of the binary tree into 4-wide nodes
    makes the bunny scene's tree smaller (1,451 vs 1,729 wide nodes) and its rays visit ~7 % fewer nodes than the greedy
    largest-area rule, with the same closest hits; on a uniform triangle soup it never does worse."""
    import ctypes
    from rtpotato import _ffi as F
    from rtpotato import scenes
    for scene, gain in ((scenes.bunny_full(), 0.95), (scenes.random_mesh(100_000), 1.0)):
        rays = _rays_for(scene, 20000, 11, adversarial=False)
        d = scene.desc()
        res, nodes = {}, {}
        for c in (F.RP_COLLAPSE_GREEDY, F.RP_COLLAPSE_SAH):
            st = (ctypes.c_uint64 * 4)()
            assert F.host().rph_bvh_selfcheck_ex(d.ptr(), fmt, c, st) == 0  # structural check of the packed tree
            nodes[c] = st[0]
            out = np.zeros((len(rays), 3), dtype=np.uint64)
            F.check_host(F.host().rph_bvh_traversal_stats_ex(d.ptr(), rays.ctypes.data, len(rays), fmt, c, out.ctypes.data))
            res[c] = out
        g, s = res[F.RP_COLLAPSE_GREEDY], res[F.RP_COLLAPSE_SAH]
        assert (g[:, 2] == s[:, 2]).all()
        assert nodes[F.RP_COLLAPSE_SAH] <= nodes[F.RP_COLLAPSE_GREEDY]
        assert s[:, 0].mean() <= gain * g[:, 0].mean(), (s[:, 0].mean(), g[:, 0].mean())
        assert s[:, 1].mean() <= 1.02 * g[:, 1].mean()
