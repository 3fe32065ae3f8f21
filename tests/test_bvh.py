"""The device acceleration structure's builder (rp_bvh.cpp, CPU-only self-check through librp_host.so)
and scene validation: every index the reference would bounds-check is rejected before upload."""
import ctypes

import numpy as np
import pytest


def _selfcheck(scene):
    from rtpotato import _ffi as F
    d = scene.desc()
    st = (ctypes.c_uint64 * 4)()
    rc = F.host().rph_bvh_selfcheck(d.ptr(), st)
    return rc, list(st), (F.host().rph_last_error() or b"").decode()


@pytest.mark.parametrize("name", ["bunny", "bunny_full", "glass_bunny", "three_balls", "more_balls", "two_balls",
                                  "earth", "one_triangle"])
def test_catalogue_trees_valid(name):
    from rtpotato import scenes
    rc, st, err = _selfcheck(scenes.CATALOGUE[name]())
    assert rc == 0, err
    nodes, leaves, depth, prims = st
    assert leaves >= 1 and prims == len(scenes.CATALOGUE[name]().root)


def test_bunny_tree_shape():
    """SAH with <= 4 primitives per leaf: far fewer nodes than the reference's 9,937 one-per-leaf nodes."""
    from rtpotato import scenes
    rc, (nodes, leaves, depth, prims), err = _selfcheck(scenes.bunny())
    assert rc == 0, err
    assert prims == 4969 and nodes < 4969 and depth < 40


def test_degenerate_geometry():
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
    rc, st, err = _selfcheck(sc)
    assert rc == 0, err
    one = Scene(cam, SceneData(mat, [], []), Hittable.Sphere((0, 0, 0), 1.0, 0), Emit.SkyGradient)
    rc, st, err = _selfcheck(one)
    assert rc == 0 and st[0] == 1 and st[1] == 1, (st, err)


def test_random_mesh_tree_valid():
    from rtpotato import scenes
    rc, st, err = _selfcheck(scenes.random_mesh(20000))
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
