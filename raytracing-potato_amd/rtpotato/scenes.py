"""The reference's scene catalogue (example_scenes.rs) and the benchmark configurations.

Every constructor returns a `Scene` (camera with aspect 1.0 as in the reference; `configure()` sets the
aspect to width / height as main.rs:22 does).  Configs:
  C1  bunny() exactly (example_scenes.rs:309-350), 320x180, 4 spp
  C2  bunny Lambert-only, SkyGradient, 1920x1080, 64 spp
  C3  bunny full materials + earthmap + sky panorama, 1920x1080, 256 spp        (the headline metric)
  C4  C3 scene, 1920x1080, 1024 spp, sharded across GPUs
  C5  synthetic 10M-triangle random mesh, 4096x4096, 256 spp
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace

import numpy as np

from . import _ffi as F
from .assets import load_image, load_mesh, sky_panorama
from .rng import StdRng
from .scene import (FRAC_PI_2, FRAC_PI_4, PI, Absorb, Camera, Emit, Hittable, Material, Mesh, RenderParams,
                    Scatter, Scene, SceneData, Texture, Transformation, hittables, rgb)

DEFAULT_SEED = 0x5EED0001  # SURVEY.md 8d base seed of the RNG contract


def _cam(fov, focal, lens, pos, target, up=(0.0, 1.0, 0.0)) -> Camera:
    return Camera(1.0, fov, focal, lens, Transformation.lookat(pos, target, up))


def three_balls() -> Scene:  # example_scenes.rs:22-60
    textures = [Texture.Solid(rgb(0.8, 0.8, 0.0)), Texture.Solid(rgb(0.1, 0.2, 0.5))]
    materials = [
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(0), Emit.None_),
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(1), Emit.None_),
        Material.new(Scatter.Dielectric(1.5), Absorb.WhiteBody, Emit.None_),
        Material.new(Scatter.Metal(0.0), Absorb.Albedo(rgb(0.8, 0.6, 0.2)), Emit.None_),
    ]
    root = hittables(Hittable.Sphere((0.0, -100.5, -1.0), 100.0, 0), Hittable.Sphere((0.0, 0.0, -1.0), 0.5, 1),
                     Hittable.Sphere((-1.0, 0.0, -1.0), 0.5, 2), Hittable.Sphere((1.0, 0.0, -1.0), 0.5, 3))
    cam = _cam(FRAC_PI_2, 3.46, 0.1, (-2.0, 2.0, 1.0), (0.0, 0.0, -1.0))
    return Scene(cam, SceneData(materials, textures, []), root, Emit.SkyGradient, F.RP_ROOT_LIST, "three_balls")


def more_balls() -> Scene:  # example_scenes.rs:63-138
    textures = [Texture.Checker(1, 2), Texture.Solid(rgb(0.2, 0.3, 0.1)), Texture.Solid(rgb(0.9, 0.9, 0.9))]
    materials = [
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(0), Emit.None_),
        Material.new(Scatter.Lambert, Absorb.Albedo(rgb(0.1, 0.2, 0.5)), Emit.None_),
        Material.new(Scatter.Metal(0.0), Absorb.Albedo(rgb(0.8, 0.6, 0.2)), Emit.None_),
        Material.new(Scatter.Dielectric(1.5), Absorb.WhiteBody, Emit.None_),
    ]
    parts = [Hittable.Sphere((0.0, -1000.0, -1.0), 1000.0, 0), Hittable.Sphere((-4.0, 1.8, 0.0), 1.8, 1),
             Hittable.Sphere((4.0, 1.8, 0.0), 1.8, 2), Hittable.Sphere((0.0, 1.8, 0.0), 1.8, 3)]
    rng = StdRng.from_seed(bytes([249] * 32))
    for x in range(-31, 31):
        for z in range(-31, 31):
            if z == 0:
                continue
            radius = rng.closed_range(0.1, 0.3)
            cx = x + rng.closed_range(-0.5 + radius, 0.5 - radius)
            cz = z + rng.closed_range(-0.5 + radius, 0.5 - radius)
            parts.append(Hittable.Sphere((float(cx), radius, float(cz)), radius, len(materials)))
            albedo = rgb(rng.gen(), rng.gen(), rng.gen())
            if rng.bernoulli(0.7):
                materials.append(Material.new(Scatter.Lambert, Absorb.Albedo(albedo), Emit.None_))
            elif rng.bernoulli(0.7):
                materials.append(Material.new(Scatter.Metal(rng.gen()), Absorb.Albedo(albedo), Emit.None_))
            else:
                materials.append(Material.new(Scatter.Dielectric(1.5), Absorb.WhiteBody, Emit.None_))
    cam = _cam(FRAC_PI_2, 7.5, 0.02, (6.0, 2.0, 4.0), (0.0, 0.0, 0.0))
    return Scene(cam, SceneData(materials, textures, []), hittables(*parts), Emit.SkyGradient, F.RP_ROOT_LIST,
                 "more_balls")


def more_balls_optimized() -> Scene:  # example_scenes.rs:141-150
    s = more_balls()
    return replace(s, root_kind=F.RP_ROOT_BVH, name="more_balls_optimized")


def two_balls() -> Scene:  # example_scenes.rs:153-187
    textures = [Texture.Solid(rgb(0.2, 0.2, 0.2)), Texture.Solid(rgb(0.9, 0.0, 0.5)), Texture.Checker(0, 1),
                Texture.Perlin(0)]
    materials = [Material.new(Scatter.Lambert, Absorb.AlbedoMap(2), Emit.None_),
                 Material.new(Scatter.Lambert, Absorb.AlbedoMap(3), Emit.None_)]
    root = hittables(Hittable.Sphere((0.0, -10.0, 0.0), 10.0, 0), Hittable.Sphere((0.0, 10.0, 0.0), 10.0, 1))
    cam = _cam(FRAC_PI_2, 7.5, 0.0, (6.0, 0.0, 4.0), (0.0, 0.0, 0.0))
    return Scene(cam, SceneData(materials, textures, []), root, Emit.SkyGradient, F.RP_ROOT_BVH, "two_balls")


def earth() -> Scene:  # example_scenes.rs:190-219
    textures = [Texture.Image(load_image("earthmap"))]
    materials = [Material.new(Scatter.Lambert, Absorb.AlbedoMap(0), Emit.None_)]
    root = Hittable.Sphere((0.0, 0.0, 0.0), 2.0, 0)
    cam = _cam(PI / 9.0, 1.0, 0.0, (13.0, 7.0, 3.0), (0.0, 0.0, 0.0))
    return Scene(cam, SceneData(materials, textures, []), root, Emit.SkyGradient, F.RP_ROOT_BVH, "earth")


def one_triangle() -> Scene:  # example_scenes.rs:222-262
    norm = math.sqrt((1.0 * 1.0 + 1.0 * 1.0) + 1.0 * 1.0)  # vector![1,1,1].normalize(): component / norm
    normal = (1.0 / norm, 1.0 / norm, 1.0 / norm)
    mesh = Mesh(np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]), np.array([normal] * 3),
                np.zeros((3, 2)), np.array([0, 1, 2], dtype=np.uint32), material=0)
    materials = [Material.new(Scatter.None_, Absorb.BlackBody, Emit.DebugNormals),
                 Material.new(Scatter.Lambert, Absorb.Albedo(rgb(0.1, 0.2, 0.5)), Emit.None_)]
    root = hittables(Hittable.Triangle(0, 0), Hittable.Sphere((0.0, -1000.0, -1.0), 1000.0, 1))
    cam = _cam(FRAC_PI_2, 1.0, 0.0, (2.0, 0.5, 1.0), (0.0, 0.0, 0.0))
    return Scene(cam, SceneData(materials, [], [mesh]), root, Emit.SkyGradient, F.RP_ROOT_BVH, "one_triangle")


def _bunny_scene(mesh_name: str, materials, textures, background, extra=(), name="") -> Scene:
    mesh = load_mesh(mesh_name)
    root = hittables(Hittable.Triangle(mesh.iter_triangles(), 0),
                     Hittable.Sphere((0.0, -1000.0, -1.0), 1000.0, 1), *extra)
    cam = _cam(FRAC_PI_4, 1.0, 0.0, (-1.5, 1.5, 2.5), (0.0, 0.5, 0.0))
    return Scene(cam, SceneData(materials, textures, [mesh]), root, background, F.RP_ROOT_BVH, name)


def glass_bunny() -> Scene:  # example_scenes.rs:265-306
    materials = [Material.new(Scatter.Dielectric(1.5), Absorb.Albedo(rgb(0.7, 0.8, 0.7)), Emit.None_),
                 Material.new(Scatter.Metal(0.05), Absorb.Albedo(rgb(0.8, 0.8, 0.8)), Emit.None_)]
    return _bunny_scene("bunny_flat", materials, [Texture.Image(sky_panorama())], Emit.SkySphere(0),
                        name="glass_bunny")


def bunny() -> Scene:  # example_scenes.rs:309-350 (config C1)
    materials = [Material.new(Scatter.None_, Absorb.BlackBody, Emit.DebugNormals),
                 Material.new(Scatter.Metal(0.05), Absorb.Albedo(rgb(0.8, 0.8, 0.8)), Emit.None_)]
    return _bunny_scene("bunny", materials, [Texture.Image(sky_panorama())], Emit.SkySphere(0), name="bunny")


def bunny_lambert() -> Scene:  # config C2
    materials = [Material.new(Scatter.Lambert, Absorb.Albedo(rgb(0.8, 0.8, 0.8)), Emit.None_),
                 Material.new(Scatter.Lambert, Absorb.Albedo(rgb(0.5, 0.5, 0.5)), Emit.None_)]
    return _bunny_scene("bunny", materials, [], Emit.SkyGradient, name="bunny_lambert")


def bunny_full() -> Scene:  # config C3 / C4
    materials = [
        Material.new(Scatter.Dielectric(1.5), Absorb.Albedo(rgb(0.7, 0.8, 0.7)), Emit.None_),  # glass bunny
        Material.new(Scatter.Metal(0.05), Absorb.Albedo(rgb(0.8, 0.8, 0.8)), Emit.None_),      # ground
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(1), Emit.None_),                        # earth ball
        Material.new(Scatter.Metal(0.0), Absorb.Albedo(rgb(0.8, 0.6, 0.2)), Emit.None_),       # mirror ball
    ]
    textures = [Texture.Image(sky_panorama()), Texture.Image(load_image("earthmap"))]
    extra = (Hittable.Sphere((1.2, 0.5, -0.8), 0.5, 2), Hittable.Sphere((-1.2, 0.4, -0.6), 0.4, 3))
    return _bunny_scene("bunny", materials, textures, Emit.SkySphere(0), extra, name="bunny_full")


def variants() -> Scene:
    """Not in example_scenes.rs: the material and texture variants no catalogue scene uses, in one small
    scene -- Emit::Color as a light and on a scattering surface (material.rs:52), Texture::Noise with a
    positive and a negative seed (texture.rs:62-68), Texture::DebugUVs on a sphere and on an uv-mapped
    triangle (texture.rs:24), Texture::Missing (texture.rs:23) and an Emit::None background (material.rs:51):
    all light comes from the emissive sphere."""
    textures = [Texture.Noise(7), Texture.DebugUVs, Texture.Missing, Texture.Noise(-3)]
    materials = [
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(0), Emit.None_),                             # ground: Noise
        Material.new(Scatter.None_, Absorb.BlackBody, Emit.Color(rgb(4.0, 3.5, 3.0))),               # light
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(1), Emit.None_),                             # DebugUVs
        Material.new(Scatter.Metal(0.3), Absorb.AlbedoMap(2), Emit.Color(rgb(0.25, 0.125, 0.0625))),  # Missing
        Material.new(Scatter.Dielectric(1.3), Absorb.AlbedoMap(3), Emit.None_),                     # Noise(-3)
    ]
    mesh = Mesh(np.array([[-3.0, -0.5, -3.0], [3.0, -0.5, -3.0], [0.0, 3.0, -3.5]]),
                np.array([[0.0, 0.0, 1.0]] * 3), np.array([[0.0, 0.0], [1.0, 0.0], [0.5, 1.0]]),
                np.array([0, 1, 2], dtype=np.uint32), material=2)
    root = hittables(Hittable.Sphere((0.0, -100.5, -1.0), 100.0, 0), Hittable.Sphere((0.0, 2.2, -1.2), 0.8, 1),
                     Hittable.Sphere((-1.1, 0.0, -1.0), 0.5, 2), Hittable.Sphere((0.0, 0.0, -1.0), 0.5, 3),
                     Hittable.Sphere((1.1, 0.0, -1.0), 0.5, 4), Hittable.Triangle(0, 0))
    cam = _cam(FRAC_PI_2, 1.0, 0.0, (0.0, 1.0, 2.5), (0.0, 0.2, -1.0))
    return Scene(cam, SceneData(materials, textures, [mesh]), root, Emit.None_, F.RP_ROOT_BVH, "variants")


def variants_sky() -> Scene:
    """Not in example_scenes.rs: Emit::SkySphere over a non-image texture (DebugUVs) as the background, a
    surface that reads two textures in one hit (Absorb::AlbedoMap of a Checker of Noise / DebugUVs and
    Emit::SkySphere of a Perlin texture, sampled at the hit record: material.rs:59), on a List root."""
    textures = [Texture.DebugUVs, Texture.Noise(11), Texture.Checker(0, 1), Texture.Perlin(5), Texture.Missing]
    materials = [
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(2), Emit.SkySphere(3)),
        Material.new(Scatter.Metal(0.1), Absorb.AlbedoMap(4), Emit.SkySphere(0)),
        Material.new(Scatter.Lambert, Absorb.AlbedoMap(1), Emit.None_),
    ]
    root = hittables(Hittable.Sphere((0.0, -50.5, -1.0), 50.0, 2), Hittable.Sphere((-0.6, 0.1, -1.0), 0.6, 0),
                     Hittable.Sphere((0.7, 0.0, -1.3), 0.5, 1))
    cam = _cam(FRAC_PI_2, 1.0, 0.0, (0.0, 0.8, 1.8), (0.0, 0.0, -1.0))
    return Scene(cam, SceneData(materials, textures, []), root, Emit.SkySphere(0), F.RP_ROOT_LIST, "variants_sky")


def random_mesh(n_triangles: int = 10_000_000, seed: int = 0xC5) -> Scene:
    """Config C5: n random small triangles.  Per triangle, in draw order: centroid (3 x ClosedRange(-1, 1)),
    then 9 offsets ClosedRange(-0.005, 0.005) for vertices a, b, c; flat normal normalize((b-a) x (c-a))."""
    rng = StdRng.seed_from_u64(seed)
    g = rng.gen_f64_array(12 * n_triangles).reshape(n_triangles, 12)
    c = -1.0 + g[:, 0:3] * (1.0 - -1.0)
    off = -0.005 + g[:, 3:12] * (0.005 - -0.005)
    v = c[:, None, :] + off.reshape(n_triangles, 3, 3)
    e1 = v[:, 1] - v[:, 0]
    e2 = v[:, 2] - v[:, 0]
    n = np.cross(e1, e2)
    n = n / np.sqrt((n[:, 0] * n[:, 0] + n[:, 1] * n[:, 1]) + n[:, 2] * n[:, 2])[:, None]
    pos = v.reshape(-1, 3)
    nrm = np.repeat(n, 3, axis=0)
    mesh = Mesh(pos, nrm, np.zeros((len(pos), 2)), np.arange(3 * n_triangles, dtype=np.uint32), material=0)
    materials = [Material.new(Scatter.Lambert, Absorb.Albedo(rgb(0.7, 0.7, 0.7)), Emit.None_)]
    root = Hittable.Triangle(mesh.iter_triangles(), 0)
    cam = _cam(PI / 3.0, 1.0, 0.0, (0.0, 0.0, 3.5), (0.0, 0.0, 0.0))
    return Scene(cam, SceneData(materials, [], [mesh]), root, Emit.SkyGradient, F.RP_ROOT_BVH, "random_mesh")


CATALOGUE = {
    "three_balls": three_balls, "more_balls": more_balls, "more_balls_optimized": more_balls_optimized,
    "two_balls": two_balls, "earth": earth, "one_triangle": one_triangle, "glass_bunny": glass_bunny,
    "bunny": bunny, "bunny_lambert": bunny_lambert, "bunny_full": bunny_full, "random_mesh": random_mesh,
    "variants": variants, "variants_sky": variants_sky,
}


@dataclass(frozen=True)
class Config:
    name: str
    scene: str
    width: int
    height: int
    spp: int
    gpus: int
    description: str


CONFIGS = {
    "C1": Config("C1", "bunny", 320, 180, 4, 0, "example_scenes bunny(), 320x180, 4 spp (reference CPU case)"),
    "C2": Config("C2", "bunny_lambert", 1920, 1080, 64, 1, "bunny Lambert-only, 1920x1080x64, SkyGradient"),
    "C3": Config("C3", "bunny_full", 1920, 1080, 256, 1,
                 "bunny full materials + earthmap + sky panorama, 1920x1080x256"),
    "C4": Config("C4", "bunny_full", 1920, 1080, 1024, 8, "C3 scene, 1920x1080x1024, tile-sharded, RCCL gather"),
    "C5": Config("C5", "random_mesh", 4096, 4096, 256, 8, "synthetic 10M-triangle mesh, 4096x4096x256"),
}


def configure(scene: Scene, width: int, height: int) -> Scene:
    """main.rs:22: camera.aspect_ratio = width / height."""
    cam = replace(scene.camera, aspect_ratio=float(width) / float(height))
    return replace(scene, camera=cam)


def config_scene(name: str, **kw) -> tuple:
    cfg = CONFIGS[name]
    scene = configure(CATALOGUE[cfg.scene](**kw), cfg.width, cfg.height)
    return scene, RenderParams(cfg.width, cfg.height, cfg.spp, 8, DEFAULT_SEED)
