"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of oracle/liboracle.so (the CPU restatement of the reference).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.  It takes
the same rp_scene_desc (include/rp.h) the product consumes, so both see identical inputs.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")            # parity checker (-O2, per-event counters)
LIB_FAST = os.path.join(HERE, "liboracle_fast.so")  # timed CPU baseline (-O3, no per-event counters)
N_COUNTERS = 7  # rays, box tests, triangle tests, sphere tests, samples, triangle hits, texel fetches
COUNTER_NAMES = ["rays", "box_tests", "tri_tests", "sphere_tests", "samples", "tri_hits", "texels"]

_libs = {}


class _Rng(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint32 * 8), ("counter", ctypes.c_uint64), ("buf", ctypes.c_uint32 * 64),
                ("index", ctypes.c_uint32), ("rounds", ctypes.c_uint32)]


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib(fast: bool = False) -> ctypes.CDLL:
    if fast in _libs:
        return _libs[fast]
    path = LIB_FAST if fast else LIB
    if os.environ.get("OR_LIB"):  # the sanitizer build of the oracle (tools/sanitize.sh)
        path = os.environ["OR_LIB"]
    if not os.path.exists(path):
        build()
    L = ctypes.CDLL(path)
    vp, u64, u32, i32, dbl = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_double
    L.or_chacha_block.argtypes = [vp, u64, u64, u32, vp]
    L.or_chacha_block.restype = None
    L.or_rng_from_seed.argtypes = [vp, vp, u32]
    L.or_rng_seed_from_u64.argtypes = [vp, u64]
    L.or_rng_next_u32.argtypes = [vp]
    L.or_rng_next_u32.restype = u32
    L.or_rng_next_u64.argtypes = [vp]
    L.or_rng_next_u64.restype = u64
    L.or_rng_fill_bytes.argtypes = [vp, vp, u64]
    L.or_rng_gen_f64.argtypes = [vp]
    L.or_rng_gen_f64.restype = dbl
    L.or_stream_u64.argtypes = [u64, u64, vp]
    L.or_stream_u64.restype = None
    for n in ("or_sample_unit_disk", "or_sample_unit_ball", "or_sample_unit_sphere"):
        getattr(L, n).argtypes = [vp, vp]
        getattr(L, n).restype = None
    L.or_sample_bernoulli.argtypes = [vp, dbl]
    L.or_noise_integer.argtypes = [ctypes.c_int64] * 4
    L.or_noise_integer.restype = ctypes.c_int64
    L.or_noise_real.argtypes = [ctypes.c_int64] * 4
    L.or_noise_real.restype = dbl
    L.or_lookat.argtypes = [vp, vp, vp, vp]
    L.or_lookat.restype = None
    L.or_scene_create.argtypes = [vp]
    L.or_scene_create.restype = vp
    L.or_scene_destroy.argtypes = [vp]
    L.or_scene_destroy.restype = None
    L.or_scene_info.argtypes = [vp, vp, vp]
    L.or_intersect.argtypes = [vp, vp, u64, vp, vp, vp]
    L.or_render.argtypes = [vp, vp, vp, vp, vp, vp, i32]
    L.or_render_baseline.argtypes = [vp, vp, u32, u32, u32, u32, u32, u32, u64, vp, vp]
    L.or_render_baseline.restype = dbl
    L.or_obj_load.argtypes = [ctypes.c_char_p, vp]
    L.or_mesh_free.argtypes = [vp]
    L.or_mesh_free.restype = None
    L.or_tga_load.argtypes = [ctypes.c_char_p, vp, vp, vp]
    L.or_tga_save.argtypes = [ctypes.c_char_p, u32, u32, vp]
    L.or_free.argtypes = [vp]
    L.or_free.restype = None
    L.or_to_srgb_u8.argtypes = [vp, u64, vp]
    L.or_to_srgb_u8.restype = None
    _libs[fast] = L
    return L


class Rng:
    """rand 0.8 StdRng as restated by the oracle (for known-answer tests)."""

    def __init__(self, seed_u64: int | None = None, seed_bytes: bytes | None = None, rounds: int = 12):
        self.s = _Rng()
        if seed_bytes is not None:
            lib().or_rng_from_seed(ctypes.byref(self.s), seed_bytes, rounds)
        else:
            lib().or_rng_seed_from_u64(ctypes.byref(self.s), seed_u64 & (2**64 - 1))

    def next_u32(self):
        return lib().or_rng_next_u32(ctypes.byref(self.s))

    def next_u64(self):
        return lib().or_rng_next_u64(ctypes.byref(self.s))

    def gen(self):
        return lib().or_rng_gen_f64(ctypes.byref(self.s))

    def fill_bytes(self, n: int) -> bytes:
        b = (ctypes.c_uint8 * n)()
        lib().or_rng_fill_bytes(ctypes.byref(self.s), b, n)
        return bytes(b)

    def unit_disk(self):
        o = (ctypes.c_double * 2)()
        lib().or_sample_unit_disk(ctypes.byref(self.s), o)
        return tuple(o)

    def unit_ball(self):
        o = (ctypes.c_double * 3)()
        lib().or_sample_unit_ball(ctypes.byref(self.s), o)
        return tuple(o)

    def unit_sphere(self):
        o = (ctypes.c_double * 3)()
        lib().or_sample_unit_sphere(ctypes.byref(self.s), o)
        return tuple(o)

    def bernoulli(self, p: float) -> bool:
        return bool(lib().or_sample_bernoulli(ctypes.byref(self.s), p))


def chacha_block(key, counter: int, stream: int = 0, rounds: int = 20):
    k = (ctypes.c_uint32 * 8)(*key)
    o = (ctypes.c_uint32 * 16)()
    lib().or_chacha_block(k, counter, stream, rounds, o)
    return list(o)


def stream_u64(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.uint64)
    lib().or_stream_u64(seed & (2**64 - 1), n, out.ctypes.data)
    return out


class OracleScene:
    """or_scene built from an rp_scene_desc (ctypes struct address, e.g. rtpotato SceneDesc.addr())."""

    def __init__(self, desc_addr: int, keepalive=None, fast: bool = False):
        """fast: the -O3 build without per-event counters (the timed CPU baseline)."""
        self._keep = keepalive
        self._lib = lib(fast)
        self.h = self._lib.or_scene_create(desc_addr)
        if not self.h:
            raise ValueError("or_scene_create failed")

    def close(self):
        if self.h:
            self._lib.or_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        nn, d = ctypes.c_uint32(), ctypes.c_uint32()
        self._lib.or_scene_info(self.h, ctypes.byref(nn), ctypes.byref(d))
        return {"nodes": nn.value, "depth": d.value}

    def intersect(self, rays: np.ndarray):
        r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 8)
        hits = np.empty((len(r), 9))
        mats = np.empty(len(r), dtype=np.uint32)
        ctr = np.zeros(N_COUNTERS, dtype=np.uint64)
        self._lib.or_intersect(self.h, r.ctypes.data, len(r), hits.ctypes.data, mats.ctypes.data, ctr.ctypes.data)
        return hits, mats, dict(zip(COUNTER_NAMES, ctr.tolist()))

    def render(self, camera_addr: int, params_addr: int, width: int, height: int, threads: int = 8,
               foreground: bool = False):
        rgb = np.zeros((height, width, 3))
        fg = np.zeros((height, width), dtype=np.float32) if foreground else None
        ctr = np.zeros(N_COUNTERS, dtype=np.uint64)
        rc = self._lib.or_render(self.h, camera_addr, params_addr, rgb.ctypes.data,
                             fg.ctypes.data if fg is not None else None, ctr.ctypes.data, threads)
        if rc != 0:
            raise ValueError("or_render failed")
        return rgb, fg, dict(zip(COUNTER_NAMES, ctr.tolist()))

    def baseline(self, camera_addr: int, width: int, height: int, spp: int, max_bounce: int = 8, tile: int = 32,
                 workers: int = 4, seed: int = 0, want_image: bool = False):
        """The reference driver (main.rs:36-106) timed: (seconds, counters, image or None)."""
        img = np.zeros((height, width, 3)) if want_image else None
        ctr = np.zeros(N_COUNTERS, dtype=np.uint64)
        secs = self._lib.or_render_baseline(self.h, camera_addr, width, height, spp, max_bounce, tile, workers, seed,
                                        img.ctypes.data if img is not None else None, ctr.ctypes.data)
        return secs, dict(zip(COUNTER_NAMES, ctr.tolist())), img


class _MeshData(ctypes.Structure):
    _fields_ = [("n_vertices", ctypes.c_uint32), ("n_indices", ctypes.c_uint32),
                ("positions", ctypes.POINTER(ctypes.c_double)), ("normals", ctypes.POINTER(ctypes.c_double)),
                ("uvs", ctypes.POINTER(ctypes.c_double)), ("indices", ctypes.POINTER(ctypes.c_uint32))]


def obj_load(path: str):
    m = _MeshData()
    rc = lib().or_obj_load(path.encode(), ctypes.byref(m))
    if rc != 0:
        raise ValueError(f"or_obj_load failed ({rc})")
    try:
        nv, ni = m.n_vertices, m.n_indices
        arr = lambda p, n: np.ctypeslib.as_array(p, shape=(max(n, 1),))[:n].copy()
        return (arr(m.positions, 3 * nv).reshape(-1, 3), arr(m.normals, 3 * nv).reshape(-1, 3),
                arr(m.uvs, 2 * nv).reshape(-1, 2), arr(m.indices, ni))
    finally:
        lib().or_mesh_free(ctypes.byref(m))


def tga_load(path: str) -> np.ndarray:
    w, h = ctypes.c_uint32(), ctypes.c_uint32()
    p = ctypes.POINTER(ctypes.c_uint8)()
    rc = lib().or_tga_load(path.encode(), ctypes.byref(w), ctypes.byref(h), ctypes.byref(p))
    if rc != 0:
        raise ValueError(f"or_tga_load failed ({rc})")
    try:
        n = w.value * h.value * 4
        return np.ctypeslib.as_array(p, shape=(max(n, 1),))[:n].copy().reshape(h.value, w.value, 4)
    finally:
        lib().or_free(p)


def tga_save(path: str, img: np.ndarray) -> None:
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if lib().or_tga_save(path.encode(), a.shape[1], a.shape[0], a.ctypes.data) != 0:
        raise ValueError("or_tga_save failed")


def to_srgb_u8(rgb: np.ndarray) -> np.ndarray:
    src = np.ascontiguousarray(rgb, dtype=np.float64)
    out = np.empty(src.shape[:-1] + (4,), dtype=np.uint8)
    lib().or_to_srgb_u8(src.ctypes.data, src.size // 3, out.ctypes.data)
    return out


def lookat(position, target, up):
    o = (ctypes.c_double * 9)()
    lib().or_lookat((ctypes.c_double * 3)(*position), (ctypes.c_double * 3)(*target),
                    (ctypes.c_double * 3)(*up), o)
    return tuple(o)
