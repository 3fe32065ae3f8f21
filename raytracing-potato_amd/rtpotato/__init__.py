"""rtpotato -- host-side Python mirror of alucas2/raytracing-potato over the MI355X hot path (librp.so).

The package directory `raytracing-potato_amd/` is not an importable name; add it to sys.path:

    sys.path.insert(0, "<repo>/raytracing-potato_amd"); import rtpotato
"""
from . import _ffi  # noqa: F401
from .scene import (FRAC_PI_2, FRAC_PI_4, PI, TAU, Absorb, Camera, Emit, Hittable, Material, MaterialId,  # noqa
                    Mesh, MeshId, RenderParams, Scatter, Scene, SceneData, Texture, TextureId, Transformation,
                    TriangleId, hittables, rgb, shard_slot_count, shard_slot_pixels, vector)

__all__ = ["Absorb", "Camera", "Emit", "Hittable", "Material", "Mesh", "RenderParams", "Scatter", "Scene",
           "SceneData", "Texture", "Transformation", "hittables", "rgb"]
