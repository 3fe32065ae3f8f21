"""Host-side mirror of the reference's scene surface, lowered to the C-ABI (include/rp.h).

Names and argument meaning follow the Rust crate so scene code reads like example_scenes.rs:

    Material.new(Scatter.Metal(fuzziness=0.05), Absorb.Albedo(rgb(0.8, 0.8, 0.8)), Emit.None_)
    Hittable.Sphere(center=(0, -1000, -1), radius=1000, material=MaterialId(1))
    Texture.Image(image)          # image.rs Array2d<[u8; 4]> as an (h, w, 4) uint8 array, row 0 = bottom
    Transformation.lookat(position, target, up)
    Camera(aspect_ratio, fov, focal_dist, lens_radius, transformation)

References: hittable.rs:10-15, mesh.rs:7-35, material.rs:19-111, texture.rs:10-18, render.rs:10-25,
utility.rs:159-192, example_scenes.rs:14-19.  Triangles of a mesh are kept as numpy arrays (a 10M
triangle mesh never becomes Python objects).
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _ffi as F

PI = math.pi
TAU = 2.0 * math.pi
FRAC_PI_2 = math.pi / 2.0
FRAC_PI_4 = math.pi / 4.0


def rgb(r: float, g: float, b: float):
    return (float(r), float(g), float(b))


def vector(*xs):
    return tuple(float(x) for x in xs)


def MaterialId(i: int) -> int:
    return int(i)


def TextureId(i: int) -> int:
    return int(i)


def MeshId(i: int) -> int:
    return int(i)


def TriangleId(i: int) -> int:
    return int(i)


# ---- material.rs ---------------------------------------------------------------------------------

@dataclass(frozen=True)
class _Scatter:
    kind: int
    param: float = 0.0


class Scatter:
    None_ = _Scatter(F.RP_SCATTER_NONE)
    Lambert = _Scatter(F.RP_SCATTER_LAMBERT)

    @staticmethod
    def Metal(fuzziness: float) -> _Scatter:
        return _Scatter(F.RP_SCATTER_METAL, float(fuzziness))

    @staticmethod
    def Dielectric(refraction_index: float) -> _Scatter:
        return _Scatter(F.RP_SCATTER_DIELECTRIC, float(refraction_index))


@dataclass(frozen=True)
class _Absorb:
    kind: int
    color: tuple = (0.0, 0.0, 0.0)
    texture: int = 0


class Absorb:
    BlackBody = _Absorb(F.RP_ABSORB_BLACK_BODY)
    WhiteBody = _Absorb(F.RP_ABSORB_WHITE_BODY)

    @staticmethod
    def Albedo(color) -> _Absorb:
        return _Absorb(F.RP_ABSORB_ALBEDO, tuple(float(c) for c in color))

    @staticmethod
    def AlbedoMap(texture: int) -> _Absorb:
        return _Absorb(F.RP_ABSORB_ALBEDO_MAP, texture=int(texture))


@dataclass(frozen=True)
class _Emit:
    kind: int
    color: tuple = (0.0, 0.0, 0.0)
    texture: int = 0

    def to_c(self) -> F.rp_emit:
        e = F.rp_emit()
        e.kind, e.texture = self.kind, self.texture
        e.color[:] = self.color
        return e


class Emit:
    None_ = _Emit(F.RP_EMIT_NONE)
    DebugNormals = _Emit(F.RP_EMIT_DEBUG_NORMALS)
    SkyGradient = _Emit(F.RP_EMIT_SKY_GRADIENT)

    @staticmethod
    def Color(color) -> _Emit:
        return _Emit(F.RP_EMIT_COLOR, tuple(float(c) for c in color))

    @staticmethod
    def SkySphere(texture: int) -> _Emit:
        return _Emit(F.RP_EMIT_SKY_SPHERE, texture=int(texture))


@dataclass(frozen=True)
class Material:
    scatter: _Scatter
    absorb: _Absorb
    emit: _Emit

    @staticmethod
    def new(scatter, absorb, emit) -> "Material":  # material.rs:100-102
        return Material(scatter, absorb, emit)

    def to_c(self) -> F.rp_material:
        m = F.rp_material()
        m.scatter.kind, m.scatter.param = self.scatter.kind, self.scatter.param
        m.absorb.kind, m.absorb.texture = self.absorb.kind, self.absorb.texture
        m.absorb.color[:] = self.absorb.color
        m.emit.kind, m.emit.texture = self.emit.kind, self.emit.texture
        m.emit.color[:] = self.emit.color
        return m


# ---- texture.rs ----------------------------------------------------------------------------------

@dataclass
class _Texture:
    kind: int
    color: tuple = (0.0, 0.0, 0.0)
    odd: int = 0
    even: int = 0
    seed: int = 0
    image: Optional[np.ndarray] = None  # (h, w, 4) uint8, row 0 = bottom


class Texture:
    Missing = _Texture(F.RP_TEXTURE_MISSING)
    DebugUVs = _Texture(F.RP_TEXTURE_DEBUG_UVS)

    @staticmethod
    def Solid(color) -> _Texture:
        return _Texture(F.RP_TEXTURE_SOLID, tuple(float(c) for c in color))

    @staticmethod
    def Image(image: np.ndarray) -> _Texture:
        img = np.ascontiguousarray(image, dtype=np.uint8)
        assert img.ndim == 3 and img.shape[2] == 4, "Image texture expects an (h, w, 4) RGBA8 array"
        return _Texture(F.RP_TEXTURE_IMAGE, image=img)

    @staticmethod
    def Checker(odd: int, even: int) -> _Texture:
        return _Texture(F.RP_TEXTURE_CHECKER, odd=int(odd), even=int(even))

    @staticmethod
    def Noise(seed: int) -> _Texture:
        return _Texture(F.RP_TEXTURE_NOISE, seed=int(seed))

    @staticmethod
    def Perlin(seed: int) -> _Texture:
        return _Texture(F.RP_TEXTURE_PERLIN, seed=int(seed))


# ---- mesh.rs -------------------------------------------------------------------------------------

@dataclass
class Mesh:
    positions: np.ndarray  # (n, 3) f64
    normals: np.ndarray    # (n, 3) f64
    uvs: np.ndarray        # (n, 2) f64
    indices: np.ndarray    # (3k,) u32
    material: int = 0      # MaterialId(0) as obj::load sets it (mesh.rs:181)

    def __post_init__(self):
        self.positions = np.ascontiguousarray(self.positions, dtype=np.float64).reshape(-1, 3)
        self.normals = np.ascontiguousarray(self.normals, dtype=np.float64).reshape(-1, 3)
        self.uvs = np.ascontiguousarray(self.uvs, dtype=np.float64).reshape(-1, 2)
        self.indices = np.ascontiguousarray(self.indices, dtype=np.uint32).reshape(-1)

    def iter_triangles(self) -> np.ndarray:  # mesh.rs:32-34 -> TriangleId(3 * i)
        return (3 * np.arange(len(self.indices) // 3, dtype=np.uint32)).astype(np.uint32)


# ---- hittable.rs ---------------------------------------------------------------------------------

class Hittable:
    """Leaf hittables, built as rows of the rp_hittable numpy dtype."""

    @staticmethod
    def Sphere(center, radius: float, material: int) -> np.ndarray:
        a = np.zeros(1, dtype=F.hittable_dtype())
        a["kind"] = F.RP_HITTABLE_SPHERE
        a["material"] = material
        a["center"][0] = center
        a["radius"] = radius
        return a

    @staticmethod
    def Triangle(triangle, mesh: int) -> np.ndarray:
        t = np.atleast_1d(np.asarray(triangle, dtype=np.uint32))
        a = np.zeros(len(t), dtype=F.hittable_dtype())
        a["kind"] = F.RP_HITTABLE_TRIANGLE
        a["mesh"] = mesh
        a["triangle"] = t
        return a


def hittables(*parts: np.ndarray) -> np.ndarray:
    return np.concatenate([np.asarray(p, dtype=F.hittable_dtype()) for p in parts]) if parts else \
        np.zeros(0, dtype=F.hittable_dtype())


# ---- utility.rs Transformation, render.rs Camera / SceneData -------------------------------------

@dataclass
class Transformation:
    orientation: tuple  # column-major 3x3 (nalgebra)
    position: tuple

    @staticmethod
    def lookat(position, target, up) -> "Transformation":
        """utility.rs:172-177 (same f64 operation order as nalgebra: normalize divides, cross)."""
        p, t, u = [tuple(float(x) for x in v) for v in (position, target, up)]
        z = (p[0] - t[0], p[1] - t[1], p[2] - t[2])
        n = math.sqrt((z[0] * z[0] + z[1] * z[1]) + z[2] * z[2])
        z = (z[0] / n, z[1] / n, z[2] / n)
        x = (u[1] * z[2] - u[2] * z[1], u[2] * z[0] - u[0] * z[2], u[0] * z[1] - u[1] * z[0])
        y = (z[1] * x[2] - z[2] * x[1], z[2] * x[0] - z[0] * x[2], z[0] * x[1] - z[1] * x[0])
        return Transformation(x + y + z, p)


@dataclass
class Camera:
    aspect_ratio: float
    fov: float
    focal_dist: float
    lens_radius: float
    transformation: Transformation

    def to_c(self) -> F.rp_camera:
        c = F.rp_camera()
        c.aspect_ratio, c.fov, c.focal_dist, c.lens_radius = (float(self.aspect_ratio), float(self.fov),
                                                              float(self.focal_dist), float(self.lens_radius))
        c.orientation[:] = self.transformation.orientation
        c.position[:] = self.transformation.position
        return c


@dataclass
class SceneData:
    material_table: List[Material] = field(default_factory=list)
    texture_table: List[_Texture] = field(default_factory=list)
    mesh_table: List[Mesh] = field(default_factory=list)


@dataclass
class Scene:
    """example_scenes.rs:14-19 ExampleScene: camera, scene data, root (Bvh or List of leaves), background."""
    camera: Camera
    scene_data: SceneData
    root: np.ndarray           # rp_hittable rows
    background: _Emit
    root_kind: int = F.RP_ROOT_BVH
    name: str = ""

    def desc(self) -> "SceneDesc":
        return SceneDesc(self)


class SceneDesc:
    """An rp_scene_desc whose pointed-to arrays are kept alive by this object."""

    def __init__(self, scene: Scene):
        sd = scene.scene_data
        self._keep = []
        self.hittables = np.ascontiguousarray(scene.root, dtype=F.hittable_dtype())
        meshes = (F.rp_mesh * max(1, len(sd.mesh_table)))()
        for i, m in enumerate(sd.mesh_table):
            self._keep += [m.positions, m.normals, m.uvs, m.indices]
            meshes[i].n_vertices = len(m.positions)
            meshes[i].n_indices = len(m.indices)
            meshes[i].positions = m.positions.ctypes.data
            meshes[i].normals = m.normals.ctypes.data
            meshes[i].uvs = m.uvs.ctypes.data
            meshes[i].indices = m.indices.ctypes.data
            meshes[i].material = m.material
        mats = (F.rp_material * max(1, len(sd.material_table)))()
        for i, m in enumerate(sd.material_table):
            mats[i] = m.to_c()
        texs = (F.rp_texture * max(1, len(sd.texture_table)))()
        for i, t in enumerate(sd.texture_table):
            c = texs[i]
            c.kind, c.odd, c.even, c.seed = t.kind, t.odd, t.even, t.seed
            c.color[:] = t.color
            if t.image is not None:
                img = np.ascontiguousarray(t.image, dtype=np.uint8)
                self._keep.append(img)
                c.height, c.width = img.shape[0], img.shape[1]
                c.rgba = img.ctypes.data
        self._meshes, self._mats, self._texs = meshes, mats, texs
        d = F.rp_scene_desc()
        d.root_kind = scene.root_kind
        d.n_hittables = len(self.hittables)
        d.hittables = self.hittables.ctypes.data if len(self.hittables) else None
        d.n_meshes = len(sd.mesh_table)
        d.meshes = ctypes.cast(meshes, ctypes.POINTER(F.rp_mesh))
        d.n_materials = len(sd.material_table)
        d.materials = ctypes.cast(mats, ctypes.POINTER(F.rp_material))
        d.n_textures = len(sd.texture_table)
        d.textures = ctypes.cast(texs, ctypes.POINTER(F.rp_texture))
        d.background = scene.background.to_c()
        self.c = d

    def ptr(self):
        return ctypes.byref(self.c)

    def addr(self) -> int:
        return ctypes.addressof(self.c)


@dataclass
class RenderParams:
    """Multisampler (render.rs:58-62) + max_bounce (main.rs:25) + the RNG-contract seed + sharding."""
    width: int
    height: int
    spp: int
    max_bounce: int = 8
    seed: int = 0x5EED0001
    tile_w: int = 32
    tile_h: int = 32
    shard: int = 0
    num_shards: int = 1
    samples_per_stream: int = 0  # RNG contract batch size (0 -> RP_SAMPLES_PER_STREAM = 32; >= spp: one stream)
    shard_map: int = 0  # RP_SHARD_INTERLEAVE (tile t -> shard t % num_shards) or RP_SHARD_BALANCED (cost plan)

    def to_c(self) -> F.rp_render_params:
        p = F.rp_render_params()
        p.width, p.height, p.spp, p.max_bounce = self.width, self.height, self.spp, self.max_bounce
        p.seed = self.seed & 0xFFFFFFFFFFFFFFFF
        p.tile_w, p.tile_h, p.shard, p.num_shards = self.tile_w, self.tile_h, self.shard, self.num_shards
        p.samples_per_stream = self.samples_per_stream
        p.shard_map = self.shard_map
        return p


def shard_slot_count(params: RenderParams) -> int:
    """Length in pixels of the compact shard buffer: (shard's tiles) * tile_w * tile_h."""
    tiles_x = -(-params.width // params.tile_w)
    tiles_y = -(-params.height // params.tile_h)
    n_tiles = tiles_x * tiles_y
    n_shard_tiles = max(0, -(-(n_tiles - params.shard) // params.num_shards)) if n_tiles > params.shard else 0
    return n_shard_tiles * params.tile_w * params.tile_h


def shard_slot_pixels(params: RenderParams, tile_map=None) -> np.ndarray:
    """(slot -> flat pixel index j*W + i, or -1 for slots outside the frame) for the compact shard buffer.
    tile_map: the frame's deal order (rp_workspace_tile_map) of a balanced frame, None = the interleave."""
    tw, th = params.tile_w, params.tile_h
    tiles_x = -(-params.width // tw)
    n = shard_slot_count(params)
    slot = np.arange(n, dtype=np.int64)
    k, local = slot // (tw * th), slot % (tw * th)
    t = params.shard + k * params.num_shards
    if tile_map is not None:
        t = np.asarray(tile_map, dtype=np.int64)[t]
    i = (t % tiles_x) * tw + local % tw
    j = (t // tiles_x) * th + local // tw
    ok = (i < params.width) & (j < params.height)
    return np.where(ok, j * params.width + i, -1)
