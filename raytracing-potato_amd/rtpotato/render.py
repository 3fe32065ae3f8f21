"""render(): the drop-in for the reference's per-pixel worker loop (main.rs:61-92 calling
render.rs:94 trace_path), on MI355X through librp.so.  No CPU fallback: a missing or failing HIP
library raises.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _ffi as F
from .scene import RenderParams, Scene, shard_slot_count


def scene_options(**kw) -> F.rp_scene_options:
    """rp_scene_options with the library defaults (rp_scene_options_init), fields overridden by keyword:
    builder ("auto" | "host" | "gpu" (LBVH) | "ploc" or RP_BUILDER_*), max_leaf, cost_traverse, always_max, lds_depth,
    self_check, trav_threshold, tile_order, probe_n,
    node_format ("auto" | "f32" | "q8" | "w8" or RP_NODES_*), tile_order ("auto" | "plain" | "cost" | "morton" | "probe"), leaf_break,
    unit_queues ("auto" | "single" | "xcd_tiles" | "xcd_regions" or RP_QUEUES_*), collapse ("auto" | "greedy" | "sah" or
    RP_COLLAPSE_*), node_layout ("auto" | "dfs" | "dfs_line" or RP_LAYOUT_*), unit_order ("auto" | "tiles" | "learned" or
    RP_UNITS_*)."""
    o = F.rp_scene_options()
    F.check(F.rp().rp_scene_options_init(ctypes.byref(o)))
    for k, v in kw.items():
        if k == "builder" and isinstance(v, str):
            v = {"auto": F.RP_BUILDER_AUTO, "host": F.RP_BUILDER_HOST, "gpu": F.RP_BUILDER_DEVICE,
                 "ploc": F.RP_BUILDER_PLOC}[v]
        if k == "tile_order" and isinstance(v, str):
            v = {"auto": F.RP_TILES_AUTO, "plain": F.RP_TILES_PLAIN, "cost": F.RP_TILES_COST,
                 "morton": F.RP_TILES_MORTON, "probe": F.RP_TILES_PROBE}[v]
        if k == "node_format" and isinstance(v, str):
            v = {"auto": F.RP_NODES_AUTO, "f32": F.RP_NODES_F32, "q8": F.RP_NODES_Q8, "w8": F.RP_NODES_W8}[v]
        if k == "unit_queues" and isinstance(v, str):
            v = {"auto": F.RP_QUEUES_AUTO, "single": F.RP_QUEUES_SINGLE, "xcd_tiles": F.RP_QUEUES_XCD_TILES,
                 "xcd_regions": F.RP_QUEUES_XCD_REGIONS}[v]
        if k == "collapse" and isinstance(v, str):
            v = {"auto": F.RP_COLLAPSE_AUTO, "greedy": F.RP_COLLAPSE_GREEDY, "sah": F.RP_COLLAPSE_SAH}[v]
        if k == "node_layout" and isinstance(v, str):
            v = {"auto": F.RP_LAYOUT_AUTO, "dfs": F.RP_LAYOUT_DFS, "dfs_line": F.RP_LAYOUT_DFS_LINE}[v]
        if k == "unit_order" and isinstance(v, str):
            v = {"auto": F.RP_UNITS_AUTO, "tiles": F.RP_UNITS_TILES, "learned": F.RP_UNITS_LEARNED}[v]
        if not hasattr(o, k):
            raise KeyError(f"unknown scene option {k!r}")
        setattr(o, k, v)
    return o


class DeviceScene:
    """rp_scene: the scene's acceleration structure and tables resident in one GPU's HBM.  `options`: a dict of
    rp_scene_options fields (scene_options())."""

    def __init__(self, scene: Scene, device: int = 0, options: dict | None = None):
        self.scene = scene
        self.device = device
        self._desc = scene.desc()
        h = ctypes.c_void_p()
        opt = scene_options(**(options or {}))
        F.check(F.rp().rp_scene_create_ex(self._desc.ptr(), device, ctypes.byref(opt), ctypes.byref(h)))
        self.handle = h

    def info(self) -> dict:
        nn, nl, np_, nb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        md = ctypes.c_uint32()
        F.check(F.rp().rp_scene_info(self.handle, ctypes.byref(nn), ctypes.byref(nl), ctypes.byref(md),
                                     ctypes.byref(np_), ctypes.byref(nb)))
        return {"nodes": nn.value, "leaves": nl.value, "max_depth": md.value, "prims": np_.value,
                "device_bytes": nb.value}

    def build_times(self) -> dict:
        """rp_scene_build_times: host seconds of the scene_create phases."""
        t = np.zeros(6)
        F.check(F.rp().rp_scene_build_times(self.handle, t.ctypes.data, 6))
        return dict(zip(("validate", "host_tree", "device_input", "device_build_or_upload", "tables_upload",
                         "workspace"), t.round(4).tolist()))

    def close(self) -> None:
        for w in list(getattr(self, "_workspaces", ())):
            w.close()
        if getattr(self, "handle", None):
            F.rp().rp_scene_destroy(self.handle)
            self.handle = None

    def workspace(self) -> "Workspace":
        """A second (third, ...) per-frame workspace: frames rendered with different workspaces may run
        concurrently on different streams (rp_workspace_create)."""
        w = Workspace(self)
        self.__dict__.setdefault("_workspaces", []).append(w)
        return w

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def reserve(self, params: RenderParams, workspace: "Workspace | None" = None) -> None:
        """rp_workspace_reserve: device memory the asynchronous renders (and frame gathers) of `params`' shape
        need, in `workspace` (default: the scene's own)."""
        p = params.to_c()
        F.check(F.rp().rp_workspace_reserve(self.handle, workspace.handle if workspace else None, ctypes.byref(p)))

    def reserve_frames(self, params: RenderParams, n_frames: int, workspace: "Workspace | None" = None) -> None:
        """rp_workspace_reserve_frames: rp_workspace_reserve, plus the batch sums of n_frames frames per launch."""
        p = params.to_c()
        F.check(F.rp().rp_workspace_reserve_frames(self.handle, workspace.handle if workspace else None,
                                                   ctypes.byref(p), n_frames))

    def tile_map(self, params: RenderParams, workspace: "Workspace | None" = None) -> np.ndarray:
        """rp_workspace_tile_map: the frame's deal order (shard s's k-th tile = map[s + k * num_shards]) -- the
        balanced plan the last render of this frame in `workspace` made, or the interleave's identity."""
        tiles = -(-params.width // params.tile_w) * -(-params.height // params.tile_h)
        out = np.empty(tiles, dtype=np.uint32)
        p = params.to_c()
        F.check(F.rp().rp_workspace_tile_map(self.handle, workspace.handle if workspace else None, ctypes.byref(p),
                                             out.ctypes.data, tiles))
        return out

    def tile_costs(self, params: RenderParams, workspace: "Workspace | None" = None) -> np.ndarray:
        """rp_workspace_tile_costs: (2, shard tiles) measured costs of the last render in `workspace` -- summed unit
        durations per shard tile, then the longest unit."""
        from .scene import shard_slot_count
        n = shard_slot_count(params) // (params.tile_w * params.tile_h)
        out = np.zeros(2 * max(n, 1), dtype=np.uint32)
        p = params.to_c()
        F.check(F.rp().rp_workspace_tile_costs(self.handle, workspace.handle if workspace else None, ctypes.byref(p),
                                               out.ctypes.data, len(out)))
        return out[:2 * n].reshape(2, n)

    def frame_info(self, workspace: "Workspace | None" = None) -> int:
        """rp_workspace_frame_info: RP_FRAME_* bits of the last render enqueued with `workspace` (None = the scene's)."""
        f = ctypes.c_uint32()
        F.check(F.rp().rp_workspace_frame_info(self.handle, workspace.handle if workspace else None, ctypes.byref(f)))
        return f.value

    def unit_order(self, n: int, workspace: "Workspace | None" = None) -> tuple:
        """rp_workspace_unit_order: (durations, order) of the last render's n units (uint32 arrays; order valid when
        frame_info has RP_FRAME_UNIT_ORDER)."""
        dur = np.zeros(n, dtype=np.uint32)
        order = np.zeros(n, dtype=np.uint32)
        F.check(F.rp().rp_workspace_unit_order(self.handle, workspace.handle if workspace else None, dur.ctypes.data,
                                               order.ctypes.data, n))
        return dur, order

    def set_tile_costs(self, params: RenderParams, costs: np.ndarray, ranks: int,
                       workspace: "Workspace | None" = None) -> None:
        """rp_workspace_set_tile_costs: install a frame's learned cost table, (2, frame tiles) by frame tile."""
        c = np.ascontiguousarray(costs, dtype=np.uint32).reshape(-1)
        p = params.to_c()
        F.check(F.rp().rp_workspace_set_tile_costs(self.handle, workspace.handle if workspace else None,
                                                   ctypes.byref(p), c.ctypes.data, ranks))

    # ---- synchronous host-buffer render -----------------------------------------------------------
    def render(self, params: RenderParams, camera=None, foreground: bool = False):
        """Full frame (only the shard's pixels written, others zero): (rgb (h, w, 3) f64,
        foreground (h, w) f32 or None, stats dict)."""
        cam = (camera or self.scene.camera).to_c()
        p = params.to_c()
        rgb = np.zeros((params.height, params.width, 3), dtype=np.float64)
        fg = np.zeros((params.height, params.width), dtype=np.float32) if foreground else None
        st = F.rp_stats()
        F.check(F.rp().rp_render(self.handle, ctypes.byref(cam), ctypes.byref(p), rgb.ctypes.data,
                                 fg.ctypes.data if fg is not None else None, ctypes.byref(st)))
        return rgb, fg, {"rays": st.rays, "samples": st.samples, "pixels": st.pixels, "seconds": st.seconds}

    # ---- asynchronous device render (torch tensors, torch's current stream) ------------------------
    def render_device(self, params: RenderParams, out, counters, fg=None, camera=None, stream=None,
                      workspace: "Workspace | None" = None) -> None:
        """Render the shard into `out` (torch f64 tensor, >= shard_slot_count*3 elements) on `stream`
        (torch stream; default: current).  counters: torch int64 tensor of RP_COUNTERS_LEN elements.
        workspace: one from self.workspace() (default: the scene's own, rp_render_device); frames of more
        than one sample batch need self.reserve(params, workspace) first."""
        import torch
        cam = (camera or self.scene.camera).to_c()
        p = params.to_c()
        assert out.dtype == torch.float64 and out.is_cuda and out.numel() >= 3 * shard_slot_count(params)
        assert counters.dtype == torch.int64 and counters.numel() >= F.RP_COUNTERS_LEN
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        fgp = fg.data_ptr() if fg is not None else None
        if workspace is None:
            F.check(F.rp().rp_render_device(self.handle, ctypes.byref(cam), ctypes.byref(p), out.data_ptr(), fgp,
                                            counters.data_ptr(), ctypes.c_void_p(s.cuda_stream)))
        else:
            assert workspace.scene is self and workspace.handle
            F.check(F.rp().rp_render_device_ws(self.handle, workspace.handle, ctypes.byref(cam), ctypes.byref(p),
                                               out.data_ptr(), fgp, counters.data_ptr(),
                                               ctypes.c_void_p(s.cuda_stream)))

    def render_frames_device(self, params: RenderParams, n_frames: int, out, counters, fg=None, camera=None,
                             stream=None, workspace: "Workspace | None" = None, order="auto") -> None:
        """rp_render_frames_device_ws: n_frames frames in one launch -- frame f is render_device's frame of `params` with
        seed + f * ceil(spp / samples_per_stream) * width * height.  out: torch f64, >= n_frames * 3 * shard_slot_count
        elements (frame f at f * 3 * slots); fg: n_frames * slots floats or None; counters: the frames' sums.  The
        workspace needs reserve_frames(params, n_frames) when the frame has more than one sample batch.  order: "auto" |
        "sequential" | "interleaved" (RP_FRAME_ORDER_*)."""
        import torch
        cam = (camera or self.scene.camera).to_c()
        p = params.to_c()
        n = shard_slot_count(params)
        assert out.dtype == torch.float64 and out.is_cuda and out.numel() >= 3 * n * n_frames
        assert fg is None or fg.numel() >= n * n_frames
        assert counters.dtype == torch.int64 and counters.numel() >= F.RP_COUNTERS_LEN
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        F.check(F.rp().rp_render_frames_device_ws(self.handle, workspace.handle if workspace else None,
                                                  ctypes.byref(cam), ctypes.byref(p), n_frames,
                                                  {"auto": F.RP_FRAME_ORDER_AUTO, "sequential": F.RP_FRAME_ORDER_SEQUENTIAL,
                                                   "interleaved": F.RP_FRAME_ORDER_INTERLEAVED,
                                                   "pixel": F.RP_FRAME_ORDER_PIXEL}.get(order, order),
                                                  out.data_ptr(),
                                                  fg.data_ptr() if fg is not None else None, counters.data_ptr(),
                                                  ctypes.c_void_p(s.cuda_stream)))

    def to_bgra8(self, params: RenderParams, shard_rgb, out, stream=None) -> None:
        """Output stage on the device (rp_shard_to_bgra8): the shard's linear f64 RGB (`shard_rgb`, torch
        f64) -> to_srgb_u8 bytes in TGA order B, G, R, A into `out` (torch uint8, >= 4 * slots)."""
        import torch
        n = shard_slot_count(params)
        assert shard_rgb.dtype == torch.float64 and shard_rgb.is_cuda and shard_rgb.numel() >= 3 * n
        assert out.dtype == torch.uint8 and out.is_cuda and out.numel() >= 4 * n
        s = stream if stream is not None else torch.cuda.current_stream(out.device)
        p = params.to_c()
        F.check(F.rp().rp_shard_to_bgra8(self.handle, ctypes.byref(p), shard_rgb.data_ptr(), out.data_ptr(),
                                         ctypes.c_void_p(s.cuda_stream)))

    def frame_gather(self, comm: "Comm", params: RenderParams, shard_rgb, frame_bgra=None, frame_rgb=None,
                     counters=None, stream=None, workspace: "Workspace | None" = None) -> None:
        """rp_frame_gather: this rank's finished shard (`shard_rgb`, torch f64) all-gathered over RCCL with the
        other ranks' and de-interleaved into frame order: `frame_bgra` (torch uint8, W*H*4: to_srgb_u8 in
        tga::save order) and/or `frame_rgb` (torch f64, W*H*3); `counters` (int64, 4) summed over ranks."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(shard_rgb.device)
        n = params.width * params.height
        if frame_bgra is not None:
            assert frame_bgra.dtype == torch.uint8 and frame_bgra.is_cuda and frame_bgra.numel() >= 4 * n
        if frame_rgb is not None:
            assert frame_rgb.dtype == torch.float64 and frame_rgb.is_cuda and frame_rgb.numel() >= 3 * n
        p = params.to_c()
        F.check(F.rp().rp_frame_gather(comm.handle, self.handle, workspace.handle if workspace else None,
                                       ctypes.byref(p), shard_rgb.data_ptr(),
                                       frame_bgra.data_ptr() if frame_bgra is not None else None,
                                       frame_rgb.data_ptr() if frame_rgb is not None else None,
                                       counters.data_ptr() if counters is not None else None,
                                       ctypes.c_void_p(s.cuda_stream)))

    def frames_gather(self, comm: "Comm", params: RenderParams, n_frames: int, shard_rgb, frames_bgra=None,
                      counters=None, stream=None, workspace: "Workspace | None" = None) -> None:
        """rp_frames_gather: the n_frames shards of one render_frames_device launch (`shard_rgb`, back to back) in one
        all-gather; `frames_bgra` (torch uint8, n_frames * W*H*4) receives the assembled frames back to back."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(shard_rgb.device)
        n = params.width * params.height
        if frames_bgra is not None:
            assert frames_bgra.dtype == torch.uint8 and frames_bgra.is_cuda and frames_bgra.numel() >= 4 * n * n_frames
        assert shard_rgb.dtype == torch.float64 and shard_rgb.numel() >= 3 * shard_slot_count(params) * n_frames
        p = params.to_c()
        F.check(F.rp().rp_frames_gather(comm.handle, self.handle, workspace.handle if workspace else None,
                                        ctypes.byref(p), n_frames, shard_rgb.data_ptr(),
                                        frames_bgra.data_ptr() if frames_bgra is not None else None,
                                        counters.data_ptr() if counters is not None else None,
                                        ctypes.c_void_p(s.cuda_stream)))

    def frames_block_words(self, params: RenderParams, n_frames: int) -> int:
        """rp_frames_block_words: 32-bit words of one rank's packed block for a launch of n_frames frames (the same on
        every rank of the job)."""
        p = params.to_c()
        w = ctypes.c_uint64()
        F.check(F.rp().rp_frames_block_words(ctypes.byref(p), n_frames, ctypes.byref(w)))
        return w.value

    def frames_pack(self, params: RenderParams, n_frames: int, shard_rgb, counters, send, stream=None,
                    workspace: "Workspace | None" = None) -> None:
        """rp_frames_pack: this rank's half of rp_frames_gather without the collective -- the launch's n_frames shards
        (output stage to BGRA8) and its counters into `send` (torch int32, frames_block_words words), for a caller's
        own all-gather."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(shard_rgb.device)
        assert send.dtype == torch.int32 and send.is_cuda and send.numel() >= self.frames_block_words(params, n_frames)
        p = params.to_c()
        F.check(F.rp().rp_frames_pack(self.handle, workspace.handle if workspace else None, ctypes.byref(p), n_frames,
                                      shard_rgb.data_ptr(), counters.data_ptr(), send.data_ptr(),
                                      ctypes.c_void_p(s.cuda_stream)))

    def frames_unpack(self, params: RenderParams, n_frames: int, recv, frames_bgra, counters=None, stream=None,
                      workspace: "Workspace | None" = None) -> None:
        """rp_frames_unpack: the all-gathered blocks of every rank (`recv`, rank-major) de-interleaved into the n_frames
        assembled BGRA8 frames and the counters summed over the ranks."""
        import torch
        s = stream if stream is not None else torch.cuda.current_stream(recv.device)
        n = params.width * params.height
        assert frames_bgra.is_cuda and frames_bgra.numel() * frames_bgra.element_size() >= 4 * n * n_frames
        p = params.to_c()
        F.check(F.rp().rp_frames_unpack(self.handle, workspace.handle if workspace else None, ctypes.byref(p), n_frames,
                                        recv.data_ptr(), frames_bgra.data_ptr(),
                                        counters.data_ptr() if counters is not None else None,
                                        ctypes.c_void_p(s.cuda_stream)))

    def render_gather(self, comm: "Comm", params: RenderParams, frame_bgra=None, frame_rgb=None, counters=None,
                      camera=None, stream=None, workspace: "Workspace | None" = None) -> None:
        """rp_render_gather: render this rank's shard and gather the frame (see frame_gather)."""
        import torch
        dev = (frame_bgra if frame_bgra is not None else frame_rgb).device
        s = stream if stream is not None else torch.cuda.current_stream(dev)
        cam = (camera or self.scene.camera).to_c()
        p = params.to_c()
        F.check(F.rp().rp_render_gather(comm.handle, self.handle, workspace.handle if workspace else None,
                                        ctypes.byref(cam), ctypes.byref(p),
                                        frame_bgra.data_ptr() if frame_bgra is not None else None,
                                        frame_rgb.data_ptr() if frame_rgb is not None else None,
                                        counters.data_ptr() if counters is not None else None,
                                        ctypes.c_void_p(s.cuda_stream)))

    def intersect(self, rays: np.ndarray):
        """Hittable::hit on the root for (n, 8) rays -> ((n, 9) hits, (n,) material ids)."""
        r = np.ascontiguousarray(rays, dtype=np.float64).reshape(-1, 8)
        hits = np.empty((len(r), 9), dtype=np.float64)
        mats = np.empty(len(r), dtype=np.uint32)
        F.check(F.rp().rp_intersect(self.handle, r.ctypes.data, len(r), hits.ctypes.data, mats.ctypes.data))
        return hits, mats


class Workspace:
    """rp_workspace: per-frame device state (keystream cache, queue counters, probe buffers, batch sums)."""

    def __init__(self, scene: DeviceScene):
        h = ctypes.c_void_p()
        F.check(F.rp().rp_workspace_create(scene.handle, ctypes.byref(h)))
        self.scene = scene
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None):
            F.rp().rp_workspace_destroy(self.handle)
            self.handle = None
            ws = self.scene.__dict__.get("_workspaces", [])
            if self in ws:
                ws.remove(self)


def comm_unique_id() -> bytes:
    """rp_comm_unique_id: the RCCL id rank 0 makes and shares with the other ranks out of band."""
    buf = (ctypes.c_uint8 * F.RP_COMM_ID_BYTES)()
    F.check(F.rp().rp_comm_unique_id(buf))
    return bytes(buf)


class Comm:
    """rp_comm: this rank's RCCL communicator (one process per GPU)."""

    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int):
        assert len(unique_id) == F.RP_COMM_ID_BYTES
        h = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * F.RP_COMM_ID_BYTES).from_buffer_copy(unique_id)
        F.check(F.rp().rp_comm_create(buf, nranks, rank, device, ctypes.byref(h)))
        self.handle = h
        self.nranks, self.rank, self.device = nranks, rank, device

    def close(self) -> None:
        if getattr(self, "handle", None):
            F.rp().rp_comm_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class MultiScene:
    """rp_multi: one process driving several GPUs (a scene copy per device, one RCCL communicator)."""

    def __init__(self, scene: Scene, devices, options: dict | None = None):
        self.scene = scene
        self._desc = scene.desc()
        devs = (ctypes.c_int * len(devices))(*devices)
        opt = scene_options(**(options or {}))
        h = ctypes.c_void_p()
        F.check(F.rp().rp_multi_create(self._desc.ptr(), devs, len(devices), ctypes.byref(opt), ctypes.byref(h)))
        self.handle = h
        self.devices = list(devices)

    def render(self, params: RenderParams, camera=None, rgb: bool = True, bgra: bool = False):
        """rp_render_multi: (rgb (h, w, 3) f64 or None, bgra (h, w, 4) u8 or None, stats)."""
        cam = (camera or self.scene.camera).to_c()
        p = params.to_c()
        out = np.zeros((params.height, params.width, 3)) if rgb else None
        ob = np.zeros((params.height, params.width, 4), dtype=np.uint8) if bgra else None
        st = F.rp_stats()
        F.check(F.rp().rp_render_multi(self.handle, ctypes.byref(cam), ctypes.byref(p),
                                       out.ctypes.data if out is not None else None,
                                       ob.ctypes.data if ob is not None else None, ctypes.byref(st)))
        return out, ob, {"rays": st.rays, "samples": st.samples, "pixels": st.pixels, "seconds": st.seconds}

    def close(self) -> None:
        if getattr(self, "handle", None):
            F.rp().rp_multi_destroy(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def unpack_shard(params: RenderParams, shard_buf: np.ndarray, channels: int = 3,
                 frame: np.ndarray | None = None, tile_map=None) -> np.ndarray:
    """Scatter a compact shard buffer into a full (h, w, channels) frame (rp_shard_unpack; with `tile_map`, the
    deal order of a balanced frame, rp_shard_unpack_map)."""
    if frame is None:
        frame = np.zeros((params.height, params.width, channels), dtype=np.float64)
    src = np.ascontiguousarray(shard_buf, dtype=np.float64)
    p = params.to_c()
    if tile_map is None:
        F.check(F.rp().rp_shard_unpack(ctypes.byref(p), src.ctypes.data, channels, frame.ctypes.data))
    else:
        m = np.ascontiguousarray(tile_map, dtype=np.uint32)
        F.check(F.rp().rp_shard_unpack_map(ctypes.byref(p), m.ctypes.data, src.ctypes.data, channels,
                                           frame.ctypes.data))
    return frame


def srgb_thresholds() -> np.ndarray:
    """The 256-entry threshold table of the device output stage (rp_srgb_thresholds; host only)."""
    t = np.empty(256, dtype=np.float64)
    F.check(F.rp().rp_srgb_thresholds(t.ctypes.data))
    return t


def tga_bytes(width: int, height: int, bgra) -> bytes:
    """tga::save (image.rs:116-137): 18-byte header (uncompressed true colour, 32 bpp) + the frame's
    B, G, R, A bytes in row order, row 0 = bottom -- the file rph_tga_save writes."""
    hd = bytearray(18)
    hd[2] = 2
    hd[12:14] = int(width).to_bytes(2, "little")
    hd[14:16] = int(height).to_bytes(2, "little")
    hd[16] = 32
    body = np.ascontiguousarray(bgra, dtype=np.uint8).reshape(-1)
    assert body.size == 4 * width * height
    return bytes(hd) + body.tobytes()


def device_count() -> int:
    n = ctypes.c_int()
    rc = F.rp().rp_device_count(ctypes.byref(n))
    return n.value if rc == F.RP_OK else 0


def render(scene: Scene, params: RenderParams, device: int = 0, foreground: bool = False,
           options: dict | None = None):
    """One-shot: upload the scene, render the frame, return (rgb, fg, stats)."""
    with DeviceScene(scene, device, options) as ds:
        return ds.render(params, foreground=foreground)
