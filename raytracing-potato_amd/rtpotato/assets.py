"""Scene assets: packed fixtures of the reference's assets, host loaders, the synthesised sky panorama.

The reference's assets (bunny.obj, bunny_flat.obj, earthmap.tga) are input data; /root/reference is not
present on the GPU box, so they ship here as compressed numpy fixtures produced by `make_assets.py`
through this package's own loaders (rph_obj_load / rph_tga_load, i.e. mesh.rs obj::load and image.rs
tga::load semantics).  tests/test_host.py re-derives them from the reference files where those exist.
assets/sky_panorama.tga is missing from the reference mount (.MISSING_LARGE_BLOBS:1): sky_panorama()
synthesises a deterministic stand-in (documented deviation).
"""
from __future__ import annotations

import ctypes
import functools
import os

import numpy as np

from . import _ffi as F
from .scene import Mesh

ASSET_DIR = os.path.join(F.PKG_DIR, "assets")
REFERENCE_ASSETS = "/root/reference/assets"
SKY_W, SKY_H = 2048, 1024


def obj_load(path: str) -> Mesh:
    """mesh.rs:145-183 obj::load through librp_host.so."""
    m = F.rph_mesh()
    F.check_host(F.host().rph_obj_load(path.encode(), ctypes.byref(m)))
    try:
        nv, ni = m.n_vertices, m.n_indices
        pos = np.ctypeslib.as_array(m.positions, shape=(max(1, 3 * nv),))[:3 * nv].copy() if nv else np.zeros(0)
        nrm = np.ctypeslib.as_array(m.normals, shape=(max(1, 3 * nv),))[:3 * nv].copy() if nv else np.zeros(0)
        uv = np.ctypeslib.as_array(m.uvs, shape=(max(1, 2 * nv),))[:2 * nv].copy() if nv else np.zeros(0)
        idx = np.ctypeslib.as_array(m.indices, shape=(max(1, ni),))[:ni].copy() if ni else np.zeros(0, np.uint32)
    finally:
        F.host().rph_mesh_free(ctypes.byref(m))
    return Mesh(pos, nrm, uv, idx, material=0)


def tga_load(path: str) -> np.ndarray:
    """image.rs:73-114 tga::load -> (h, w, 4) uint8, row 0 = bottom."""
    w, h = ctypes.c_uint32(), ctypes.c_uint32()
    buf = ctypes.POINTER(ctypes.c_uint8)()
    F.check_host(F.host().rph_tga_load(path.encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(buf)))
    try:
        n = w.value * h.value * 4
        arr = np.ctypeslib.as_array(buf, shape=(max(1, n),))[:n].copy()
    finally:
        F.host().rph_free(buf)
    return arr.reshape(h.value, w.value, 4)


def tga_save(path: str, image: np.ndarray) -> None:
    """image.rs:116-137 tga::save of an (h, w, 4) uint8 image (row 0 = bottom)."""
    img = np.ascontiguousarray(image, dtype=np.uint8)
    F.check_host(F.host().rph_tga_save(path.encode(), img.shape[1], img.shape[0], img.ctypes.data))


def to_srgb_u8(rgb: np.ndarray) -> np.ndarray:
    """utility.rs:212-220 over an (h, w, 3) f64 image -> (h, w, 4) uint8."""
    src = np.ascontiguousarray(rgb, dtype=np.float64)
    out = np.empty(src.shape[:-1] + (4,), dtype=np.uint8)
    F.host().rph_to_srgb_u8(src.ctypes.data, src.size // 3, out.ctypes.data)
    return out


@functools.lru_cache(maxsize=4)
def sky_panorama(width: int = SKY_W, height: int = SKY_H) -> np.ndarray:
    img = np.empty((height, width, 4), dtype=np.uint8)
    F.check_host(F.host().rph_sky_panorama(width, height, img.ctypes.data))
    img.setflags(write=False)
    return img


def _fixture(name: str) -> str:
    return os.path.join(ASSET_DIR, name + ".npz")


@functools.lru_cache(maxsize=8)
def load_mesh(name: str) -> Mesh:
    """Packed fixture of assets/<name>.obj (e.g. "bunny", "bunny_flat")."""
    path = _fixture(name)
    if not os.path.exists(path):
        ref = os.path.join(REFERENCE_ASSETS, name + ".obj")
        if os.path.exists(ref):
            return obj_load(ref)
        raise FileNotFoundError(path)
    z = np.load(path, allow_pickle=False)
    return Mesh(z["positions"], z["normals"], z["uvs"], z["indices"], material=0)


@functools.lru_cache(maxsize=8)
def load_image(name: str) -> np.ndarray:
    """Packed fixture of assets/<name>.tga (e.g. "earthmap") as (h, w, 4) uint8, row 0 = bottom."""
    path = _fixture(name)
    if not os.path.exists(path):
        ref = os.path.join(REFERENCE_ASSETS, name + ".tga")
        if os.path.exists(ref):
            return tga_load(ref)
        raise FileNotFoundError(path)
    img = np.load(path, allow_pickle=False)["rgba"]
    img.setflags(write=False)
    return img
