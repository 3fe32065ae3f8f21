"""ctypes bindings of include/rp.h (librp.so, the HIP hot path) and include/rp_host.h (librp_host.so).

librp.so must share the HIP runtime with PyTorch when both live in one process: torch's own
libamdhip64.so is loaded under the NEEDED name "libamdhip64.so" and would not be recognised as the
same library if librp.so (NEEDED "libamdhip64.so.7") pulled /opt/rocm's copy in first.  So `import
torch` happens before librp.so is opened (SONAMEs match, the loader then reuses torch's runtime).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import (POINTER, Structure, c_char_p, c_double, c_float, c_int, c_int64, c_uint8, c_uint32,
                    c_uint64, c_void_p)

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(PKG_DIR, "lib")

RP_OK, RP_EINVAL, RP_EHIP, RP_ENOMEM, RP_ENODEV, RP_EINTERNAL, RP_ERCCL = 0, -1, -2, -3, -4, -5, -6
RP_HITTABLE_SPHERE, RP_HITTABLE_TRIANGLE = 0, 1
RP_SCATTER_NONE, RP_SCATTER_LAMBERT, RP_SCATTER_METAL, RP_SCATTER_DIELECTRIC = 0, 1, 2, 3
RP_ABSORB_BLACK_BODY, RP_ABSORB_WHITE_BODY, RP_ABSORB_ALBEDO, RP_ABSORB_ALBEDO_MAP = 0, 1, 2, 3
(RP_EMIT_NONE, RP_EMIT_DEBUG_NORMALS, RP_EMIT_COLOR, RP_EMIT_SKY_GRADIENT, RP_EMIT_SKY_SPHERE) = range(5)
(RP_TEXTURE_MISSING, RP_TEXTURE_DEBUG_UVS, RP_TEXTURE_SOLID, RP_TEXTURE_IMAGE, RP_TEXTURE_CHECKER,
 RP_TEXTURE_NOISE, RP_TEXTURE_PERLIN) = range(7)
RP_ROOT_BVH, RP_ROOT_LIST = 0, 1
RP_COUNTERS_LEN = 4  # device counter block: rays, samples, pixels, status (include/rp.h)
RP_SAMPLES_PER_STREAM = 32
RP_COMM_ID_BYTES = 128
RP_BUILDER_AUTO, RP_BUILDER_HOST, RP_BUILDER_DEVICE, RP_BUILDER_PLOC = 0, 1, 2, 3
RP_NODES_AUTO, RP_NODES_F32, RP_NODES_Q8, RP_NODES_W8 = 0, 1, 2, 3
RP_TILES_AUTO, RP_TILES_PLAIN, RP_TILES_COST, RP_TILES_MORTON, RP_TILES_PROBE = 0, 1, 2, 3, 4
RP_QUEUES_AUTO, RP_QUEUES_SINGLE, RP_QUEUES_XCD_TILES, RP_QUEUES_XCD_REGIONS = 0, 1, 2, 3
RP_COLLAPSE_AUTO, RP_COLLAPSE_GREEDY, RP_COLLAPSE_SAH = 0, 1, 2
RP_LAYOUT_AUTO, RP_LAYOUT_DFS, RP_LAYOUT_DFS_LINE = 0, 1, 2
RP_UNITS_AUTO, RP_UNITS_TILES, RP_UNITS_LEARNED = 0, 1, 2
RP_FRAME_LEARNED_ORDER, RP_FRAME_PROBED, RP_FRAME_UNIT_ORDER = 2, 4, 8
RP_SHARD_INTERLEAVE, RP_SHARD_BALANCED = 0, 1
RP_STATUS_STACK_OVERFLOW, RP_STATUS_PLAN_MISMATCH = 1, 2
RP_ABI_VERSION = 9
RP_MAX_FRAMES = 64
RP_FRAME_ORDER_AUTO, RP_FRAME_ORDER_SEQUENTIAL, RP_FRAME_ORDER_INTERLEAVED, RP_FRAME_ORDER_PIXEL = 0, 1, 2, 3


class rp_hittable(Structure):
    _fields_ = [("kind", c_uint32), ("material", c_uint32), ("mesh", c_uint32), ("triangle", c_uint32),
                ("center", c_double * 3), ("radius", c_double)]


class rp_mesh(Structure):
    _fields_ = [("n_vertices", c_uint32), ("n_indices", c_uint32), ("positions", c_void_p),
                ("normals", c_void_p), ("uvs", c_void_p), ("indices", c_void_p), ("material", c_uint32),
                ("reserved", c_uint32)]


class rp_scatter(Structure):
    _fields_ = [("kind", c_uint32), ("reserved", c_uint32), ("param", c_double)]


class rp_absorb(Structure):
    _fields_ = [("kind", c_uint32), ("texture", c_uint32), ("color", c_double * 3)]


class rp_emit(Structure):
    _fields_ = [("kind", c_uint32), ("texture", c_uint32), ("color", c_double * 3)]


class rp_material(Structure):
    _fields_ = [("scatter", rp_scatter), ("absorb", rp_absorb), ("emit", rp_emit)]


class rp_texture(Structure):
    _fields_ = [("kind", c_uint32), ("odd", c_uint32), ("even", c_uint32), ("width", c_uint32),
                ("height", c_uint32), ("reserved", c_uint32), ("seed", c_int64), ("color", c_double * 3),
                ("rgba", c_void_p)]


class rp_scene_desc(Structure):
    _fields_ = [("root_kind", c_uint32), ("n_hittables", c_uint32), ("hittables", c_void_p),
                ("n_meshes", c_uint32), ("meshes", POINTER(rp_mesh)), ("n_materials", c_uint32),
                ("materials", POINTER(rp_material)), ("n_textures", c_uint32),
                ("textures", POINTER(rp_texture)), ("background", rp_emit)]


class rp_camera(Structure):
    _fields_ = [("aspect_ratio", c_double), ("fov", c_double), ("focal_dist", c_double),
                ("lens_radius", c_double), ("orientation", c_double * 9), ("position", c_double * 3)]


class rp_render_params(Structure):
    _fields_ = [("width", c_uint32), ("height", c_uint32), ("spp", c_uint32), ("max_bounce", c_uint32),
                ("seed", c_uint64), ("tile_w", c_uint32), ("tile_h", c_uint32), ("shard", c_uint32),
                ("num_shards", c_uint32), ("samples_per_stream", c_uint32), ("shard_map", c_uint32)]


class rp_scene_options(Structure):
    _fields_ = [("builder", c_uint32), ("max_leaf", c_uint32), ("cost_traverse", c_double),
                ("always_max", ctypes.c_int32), ("lds_depth", c_uint32), ("self_check", c_uint32),
                ("trav_threshold", c_uint32), ("tile_order", c_uint32), ("probe_n", c_uint32),
                ("node_format", c_uint32), ("leaf_break", c_uint32),
                ("unit_queues", c_uint32), ("queue_chunk", c_uint32), ("debug_stack_depth", c_uint32),
                ("collapse", c_uint32), ("node_layout", c_uint32), ("unit_order", c_uint32)]


class rp_stats(Structure):
    _fields_ = [("rays", c_uint64), ("samples", c_uint64), ("pixels", c_uint64), ("seconds", c_double)]


class rph_mesh(Structure):
    _fields_ = [("n_vertices", c_uint32), ("n_indices", c_uint32), ("positions", POINTER(c_double)),
                ("normals", POINTER(c_double)), ("uvs", POINTER(c_double)), ("indices", POINTER(c_uint32))]


# numpy dtype with exactly rp_hittable's layout (48 B), so large meshes never become Python objects
def hittable_dtype():
    import numpy as np
    return np.dtype({"names": ["kind", "material", "mesh", "triangle", "center", "radius"],
                     "formats": ["<u4", "<u4", "<u4", "<u4", ("<f8", (3,)), "<f8"],
                     "offsets": [0, 4, 8, 12, 16, 40], "itemsize": 48})


class RPError(RuntimeError):
    def __init__(self, code: int, message: str):
        super().__init__(f"rp error {code}: {message}")
        self.code = code


_rp = None
_host = None

RP_SYMBOLS = ["rp_abi_version", "rp_last_error", "rp_device_count", "rp_scene_create", "rp_scene_destroy",
              "rp_scene_info", "rp_shard_pixel_count", "rp_shard_unpack", "rp_render", "rp_render_device",
              "rp_intersect", "rp_diagnostics", "rp_workspace_create", "rp_workspace_destroy",
              "rp_render_device_ws", "rp_shard_to_bgra8", "rp_srgb_thresholds", "rp_scene_options_init",
              "rp_scene_create_ex", "rp_workspace_reserve", "rp_comm_unique_id", "rp_comm_create", "rp_comm_destroy",
              "rp_comm_info", "rp_frame_gather", "rp_gather_stride", "rp_frame_assemble", "rp_render_gather", "rp_multi_create", "rp_multi_destroy",
              "rp_render_multi", "rp_shard_unpack_map", "rp_workspace_tile_map", "rp_frame_assemble_ws", "rp_build_id",
              "rp_workspace_tile_costs", "rp_workspace_set_tile_costs", "rp_scene_build_times",
              "rp_workspace_frame_info", "rp_workspace_reserve_frames", "rp_render_frames_device_ws", "rp_frames_gather",
              "rp_workspace_unit_order", "rp_frames_block_words", "rp_frames_pack", "rp_frames_unpack"]
HOST_SYMBOLS = ["rph_obj_load", "rph_mesh_free", "rph_tga_load", "rph_tga_save", "rph_free", "rph_to_srgb_u8",
                "rph_lookat", "rph_sky_panorama", "rph_bvh_selfcheck", "rph_bvh_traversal_stats", "rph_bvh_selfcheck_ex", "rph_bvh_traversal_stats_ex", "rph_bvh_tree_hash", "rph_last_error",
                "rph_stdrng_u64", "rph_make_div32"]


def rp_lib_path() -> str:
    return os.path.join(LIB_DIR, "librp.so")


def host_lib_path() -> str:
    return os.path.join(LIB_DIR, "librp_host.so")


def rp() -> ctypes.CDLL:
    """librp.so (the HIP hot path).  Raises if it is missing: there is no CPU fallback."""
    global _rp
    if _rp is not None:
        return _rp
    path = os.environ.get("RP_LIB") or rp_lib_path()  # RP_LIB: lib/librp_diag.so (diagnostic counters)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `make -C raytracing-potato_amd` "
                           "(or __graft_entry__.build()); there is no CPU fallback for the render path")
    try:
        import torch  # noqa: F401  (share torch's HIP runtime, see module docstring)
    except Exception:
        pass
    lib = ctypes.CDLL(path)
    lib.rp_abi_version.restype = c_int
    lib.rp_last_error.restype = c_char_p
    lib.rp_build_id.restype = c_char_p
    lib.rp_device_count.argtypes = [POINTER(c_int)]
    lib.rp_scene_create.argtypes = [POINTER(rp_scene_desc), c_int, POINTER(c_void_p)]
    lib.rp_scene_destroy.argtypes = [c_void_p]
    lib.rp_scene_destroy.restype = None
    lib.rp_scene_info.argtypes = [c_void_p, POINTER(c_uint64), POINTER(c_uint64), POINTER(c_uint32),
                                  POINTER(c_uint64), POINTER(c_uint64)]
    lib.rp_shard_pixel_count.argtypes = [POINTER(rp_render_params), POINTER(c_uint64)]
    lib.rp_shard_unpack.argtypes = [POINTER(rp_render_params), c_void_p, c_uint32, c_void_p]
    lib.rp_render.argtypes = [c_void_p, POINTER(rp_camera), POINTER(rp_render_params), c_void_p, c_void_p,
                              POINTER(rp_stats)]
    lib.rp_render_device.argtypes = [c_void_p, POINTER(rp_camera), POINTER(rp_render_params), c_void_p, c_void_p,
                                     c_void_p, c_void_p]
    lib.rp_workspace_create.argtypes = [c_void_p, POINTER(c_void_p)]
    lib.rp_workspace_destroy.argtypes = [c_void_p]
    lib.rp_workspace_destroy.restype = None
    lib.rp_render_device_ws.argtypes = [c_void_p, c_void_p, POINTER(rp_camera), POINTER(rp_render_params), c_void_p,
                                        c_void_p, c_void_p, c_void_p]
    lib.rp_shard_to_bgra8.argtypes = [c_void_p, POINTER(rp_render_params), c_void_p, c_void_p, c_void_p]
    lib.rp_srgb_thresholds.argtypes = [c_void_p]
    lib.rp_intersect.argtypes = [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p]
    lib.rp_diagnostics.argtypes = [c_void_p, c_void_p, c_uint32, c_int]
    lib.rp_scene_options_init.argtypes = [POINTER(rp_scene_options)]
    lib.rp_scene_create_ex.argtypes = [POINTER(rp_scene_desc), c_int, POINTER(rp_scene_options), POINTER(c_void_p)]
    lib.rp_workspace_reserve.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params)]
    lib.rp_comm_unique_id.argtypes = [c_void_p]
    lib.rp_comm_create.argtypes = [c_void_p, c_int, c_int, c_int, POINTER(c_void_p)]
    lib.rp_comm_destroy.argtypes = [c_void_p]
    lib.rp_comm_destroy.restype = None
    lib.rp_comm_info.argtypes = [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]
    lib.rp_frame_gather.argtypes = [c_void_p, c_void_p, c_void_p, POINTER(rp_render_params), c_void_p, c_void_p,
                                    c_void_p, c_void_p, c_void_p]
    lib.rp_gather_stride.argtypes = [POINTER(rp_render_params), POINTER(c_uint64)]
    lib.rp_frame_assemble.argtypes = [POINTER(rp_render_params), c_void_p, c_uint32, c_void_p, c_void_p]
    lib.rp_render_gather.argtypes = [c_void_p, c_void_p, c_void_p, POINTER(rp_camera), POINTER(rp_render_params),
                                     c_void_p, c_void_p, c_void_p, c_void_p]
    lib.rp_multi_create.argtypes = [POINTER(rp_scene_desc), c_void_p, c_int, POINTER(rp_scene_options),
                                    POINTER(c_void_p)]
    lib.rp_multi_destroy.argtypes = [c_void_p]
    lib.rp_multi_destroy.restype = None
    lib.rp_render_multi.argtypes = [c_void_p, POINTER(rp_camera), POINTER(rp_render_params), c_void_p, c_void_p,
                                    POINTER(rp_stats)]
    lib.rp_shard_unpack_map.argtypes = [POINTER(rp_render_params), c_void_p, c_void_p, c_uint32, c_void_p]
    lib.rp_workspace_tile_map.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params), c_void_p, c_uint32]
    lib.rp_scene_build_times.argtypes = [c_void_p, c_void_p, c_uint32]
    lib.rp_workspace_tile_costs.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params), c_void_p, c_uint32]
    lib.rp_workspace_frame_info.argtypes = [c_void_p, c_void_p, POINTER(c_uint32)]
    lib.rp_workspace_unit_order.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_uint64]
    lib.rp_frames_block_words.argtypes = [POINTER(rp_render_params), c_uint32, POINTER(c_uint64)]
    lib.rp_frames_pack.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params), c_uint32, c_void_p, c_void_p, c_void_p,
                                   c_void_p]
    lib.rp_frames_unpack.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params), c_uint32, c_void_p, c_void_p, c_void_p,
                                     c_void_p]
    lib.rp_workspace_reserve_frames.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params), c_uint32]
    lib.rp_frames_gather.argtypes = [c_void_p, c_void_p, c_void_p, POINTER(rp_render_params), c_uint32, c_void_p, c_void_p,
                                     c_void_p, c_void_p]
    lib.rp_render_frames_device_ws.argtypes = [c_void_p, c_void_p, POINTER(rp_camera), POINTER(rp_render_params),
                                               c_uint32, c_uint32, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.rp_workspace_set_tile_costs.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params), c_void_p, c_uint32]
    lib.rp_frame_assemble_ws.argtypes = [c_void_p, c_void_p, POINTER(rp_render_params), c_void_p, c_uint32, c_void_p,
                                         c_void_p]
    if lib.rp_abi_version() != RP_ABI_VERSION:
        raise RuntimeError(f"{path}: ABI version {lib.rp_abi_version()}, bindings expect {RP_ABI_VERSION} (rebuild)")
    _rp = lib
    return lib


def host() -> ctypes.CDLL:
    global _host
    if _host is not None:
        return _host
    path = os.environ.get("RP_HOST_LIB") or host_lib_path()  # RP_HOST_LIB: the sanitizer build (tools/sanitize.sh)
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `make -C raytracing-potato_amd`")
    lib = ctypes.CDLL(path)
    lib.rph_obj_load.argtypes = [c_char_p, POINTER(rph_mesh)]
    lib.rph_mesh_free.argtypes = [POINTER(rph_mesh)]
    lib.rph_mesh_free.restype = None
    lib.rph_tga_load.argtypes = [c_char_p, POINTER(c_uint32), POINTER(c_uint32), POINTER(POINTER(c_uint8))]
    lib.rph_tga_save.argtypes = [c_char_p, c_uint32, c_uint32, c_void_p]
    lib.rph_free.argtypes = [c_void_p]
    lib.rph_free.restype = None
    lib.rph_to_srgb_u8.argtypes = [c_void_p, c_uint64, c_void_p]
    lib.rph_to_srgb_u8.restype = None
    lib.rph_lookat.argtypes = [c_double * 3, c_double * 3, c_double * 3, c_double * 9]
    lib.rph_lookat.restype = None
    lib.rph_sky_panorama.argtypes = [c_uint32, c_uint32, c_void_p]
    lib.rph_bvh_selfcheck.argtypes = [POINTER(rp_scene_desc), c_uint32, POINTER(c_uint64)]
    lib.rph_bvh_traversal_stats.argtypes = [POINTER(rp_scene_desc), c_void_p, c_uint64, c_uint32, c_void_p]
    lib.rph_bvh_selfcheck_ex.argtypes = [POINTER(rp_scene_desc), c_uint32, c_uint32, POINTER(c_uint64)]
    lib.rph_bvh_traversal_stats_ex.argtypes = [POINTER(rp_scene_desc), c_void_p, c_uint64, c_uint32, c_uint32, c_void_p]
    lib.rph_bvh_tree_hash.argtypes = [POINTER(rp_scene_desc), c_uint32, c_uint32, POINTER(c_uint64)]
    lib.rph_last_error.restype = c_char_p
    lib.rph_stdrng_u64.argtypes = [c_void_p, c_uint64, c_uint64, c_void_p]
    lib.rph_make_div32.argtypes = [c_uint32, POINTER(c_uint32), POINTER(c_uint32)]
    _host = lib
    return lib


def check(code: int, lib: ctypes.CDLL | None = None) -> None:
    if code != RP_OK:
        lib = lib or rp()
        fn = lib.rp_last_error if hasattr(lib, "rp_last_error") else lib.rph_last_error
        raise RPError(code, (fn() or b"").decode(errors="replace"))


def check_host(code: int) -> None:
    if code != RP_OK:
        raise RPError(code, (host().rph_last_error() or b"").decode(errors="replace"))


__all__ = [n for n in dir() if not n.startswith("__")]
