"""Output stage (utility.rs:212-220 to_srgb_u8, image.rs:116-137 tga::save): the device looks each channel
up in the 255 thresholds of to_srgb_u8's step function, built on the host with the host libm's pow.  CPU
tests: the table against the host restatement rph_to_srgb_u8 (the reference expression in C++), the
device's binary search emulated in numpy, and the TGA byte layout.  GPU test: rp_shard_to_bgra8."""
import ctypes
import os

import numpy as np
import pytest


def _host_bytes(x):
    """rph_to_srgb_u8 on a flat array of channel values (R of each pixel)."""
    from rtpotato import _ffi as F
    x = np.ascontiguousarray(x, dtype=np.float64)
    rgb = np.zeros((x.size, 3))
    rgb[:, 0] = x
    rgba = np.zeros((x.size, 4), dtype=np.uint8)
    F.host().rph_to_srgb_u8(rgb.ctypes.data, x.size, rgba.ctypes.data)
    return rgba[:, 0]


def _device_search(thr, x):
    """The kernel's 8-step search: k += step while x >= thr[k + step] (NaN compares false -> 0)."""
    k = np.zeros(x.shape, dtype=np.int64)
    with np.errstate(invalid="ignore"):
        for step in (128, 64, 32, 16, 8, 4, 2, 1):
            k += np.where(x >= thr[k + step], step, 0)
    return k


def test_thresholds_are_the_step_points_of_to_srgb_u8():
    from rtpotato.render import srgb_thresholds
    thr = srgb_thresholds()
    assert thr[0] == -np.inf and 0.0 < thr[1] and thr[255] <= 1.0
    assert np.all(np.diff(thr[1:]) > 0)
    at = _host_bytes(thr[1:])
    below = _host_bytes(np.nextafter(thr[1:], -np.inf))
    k = np.arange(1, 256)
    assert np.all(at >= k) and np.all(below < k)


def test_lookup_equals_to_srgb_u8():
    from rtpotato.render import srgb_thresholds
    thr = srgb_thresholds()
    rng = np.random.default_rng(212)
    k = np.arange(256) / 255.0
    x = np.concatenate([
        rng.uniform(-0.2, 1.3, 1_000_000),
        10.0 ** rng.uniform(-12, 0, 200_000),
        k, k ** 2.2, np.nextafter(k ** 2.2, np.inf), np.nextafter(k ** 2.2, -np.inf),
        thr[1:], np.nextafter(thr[1:], -np.inf),
        [0.0, -0.0, 1.0, np.nan, np.inf, -np.inf, 5e-324, 1e300, -1e300],
    ])
    assert np.array_equal(_device_search(thr, x), _host_bytes(x).astype(np.int64))


def test_tga_bytes_match_rph_tga_save(tmp_path):
    from rtpotato import _ffi as F
    from rtpotato.render import tga_bytes
    rng = np.random.default_rng(3)
    w, h = 7, 5
    rgba = rng.integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    path = str(tmp_path / "x.tga")
    assert F.host().rph_tga_save(path.encode(), w, h, rgba.ctypes.data) == 0
    bgra = rgba[..., [2, 1, 0, 3]]
    assert open(path, "rb").read() == tga_bytes(w, h, bgra)


@pytest.mark.gpu
def test_shard_to_bgra8_matches_host(gpu):
    """rp_shard_to_bgra8 on a rendered frame (sharded, ragged tiles) = rph_to_srgb_u8 of the same linear
    values, in TGA byte order; the world-1 frame assembly gives the reference's output.tga bytes."""
    import torch
    from rtpotato import _ffi as F
    from rtpotato import scenes
    from rtpotato.render import tga_bytes, unpack_shard
    from rtpotato.scene import RenderParams, shard_slot_count
    sc = scenes.configure(scenes.bunny_full(), 70, 45)
    for params in (RenderParams(70, 45, 8, 8, 11, 16, 16), RenderParams(70, 45, 8, 8, 11, 16, 16, 1, 3)):
        n = shard_slot_count(params)
        rgb = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
        ctr = torch.zeros(4, dtype=torch.int64, device="cuda")
        out = torch.zeros(4 * n, dtype=torch.uint8, device="cuda")
        with gpu.DeviceScene(sc) as ds:
            ds.render_device(params, rgb, ctr)
            ds.to_bgra8(params, rgb, out)
            torch.cuda.synchronize()
        lin = rgb.cpu().numpy()
        ref = np.zeros((n, 4), dtype=np.uint8)
        F.host().rph_to_srgb_u8(lin.ctypes.data, n, ref.ctypes.data)
        got = out.cpu().numpy().reshape(n, 4)
        assert np.array_equal(got, ref[:, [2, 1, 0, 3]])
        if params.num_shards == 1:
            import ctypes
            fr = torch.zeros(params.width * params.height * 4, dtype=torch.uint8, device="cuda")
            F.check(F.rp().rp_frame_assemble(ctypes.byref(params.to_c()), out.data_ptr(), 1, fr.data_ptr(),
                                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
            torch.cuda.synchronize()
            frame = fr.cpu().numpy().reshape(params.height, params.width, 4)
            full = unpack_shard(params, lin)
            rgba = np.zeros((params.height, params.width, 4), dtype=np.uint8)
            F.host().rph_to_srgb_u8(np.ascontiguousarray(full).ctypes.data, params.width * params.height,
                                    rgba.ctypes.data)
            assert tga_bytes(params.width, params.height, frame) == tga_bytes(params.width, params.height,
                                                                              rgba[..., [2, 1, 0, 3]])
