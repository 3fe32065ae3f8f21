"""The coherent primary pass (rp_scene_options.primary, rp_kernel.hip primary_kernel).

With lens_radius = 0 a camera ray depends only on its jitter words (render.rs:36-44,74-82), so the library traces every
camera ray of the frame first, in waves of 64 neighbouring rays, and the path loop starts each sample from that closest
hit.  The closest hit does not depend on the order rays are traced (up to exact-t ties), so the frame
must be the path-loop frame: same rays, same samples, pixels equal -- and the oracle's.  Cases: both node formats and
the 8-wide one, the spilled stack, odd tiles and frame sizes, spp not a multiple of the pass's 16 samples, RNG streams
whose length is not a multiple of 4 (the pass's per-lane ChaCha path instead of the quad one), multi-batch frames,
shards of the balanced plan, and lens cameras (no pass).
"""
import numpy as np
import pytest
from dataclasses import replace

from parity import assert_parity, compare, oracle_render, shard_mask

pytestmark = pytest.mark.gpu


def _scene(name, w, h, spp, **kw):
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    sc = scenes.configure(scenes.CATALOGUE[name](**kw), w, h)
    return sc, RenderParams(w, h, spp, 8, scenes.DEFAULT_SEED)


def _render(gpu, sc, p, **opt):
    with gpu.DeviceScene(sc, options=opt or None) as ds:
        rgb, fg, st = ds.render(p, foreground=True)
        flags = ds.frame_info()
    return rgb, fg, st, flags


def _on_off(gpu, sc, p, **opt):
    """The frame with the pass (ON) and without it (OFF): identical counts, pixels to the parity bar (bitwise but for
    exact-t ties), foreground identical."""
    from rtpotato import _ffi as F
    on, fg_on, st_on, f_on = _render(gpu, sc, p, primary="on", **opt)
    off, fg_off, st_off, f_off = _render(gpu, sc, p, primary="off", **opt)
    assert f_on & F.RP_FRAME_PRIMARY_PASS and not f_off & F.RP_FRAME_PRIMARY_PASS, (f_on, f_off)
    assert (st_on["rays"], st_on["samples"], st_on["pixels"]) == (st_off["rays"], st_off["samples"], st_off["pixels"])
    m = shard_mask(p)
    c = compare(on, off, m)
    assert_parity(c, min_exact=0.9999)
    assert np.array_equal(fg_on[m], fg_off[m])
    return on, st_on


@pytest.mark.parametrize("name", ["bunny_full", "variants", "variants_sky", "earth", "one_triangle", "glass_bunny",
                                  "two_balls"])
def test_primary_pass_equals_path_loop(gpu, name):
    sc, p = _scene(name, 64, 36, 8)
    _on_off(gpu, sc, p)


@pytest.mark.parametrize("fmt", ["f32", "q8", "w8"])
def test_primary_pass_node_formats_and_spill(gpu, fmt):
    """Every node format, with the stack split into LDS + a global spill run (lds_depth 8)."""
    sc, p = _scene("bunny_full", 80, 48, 12)
    _on_off(gpu, sc, p, node_format=fmt)
    _on_off(gpu, sc, p, node_format=fmt, lds_depth=8)


def test_primary_pass_against_oracle_odd_shapes(gpu):
    """Odd frame and tile sizes (quads cut by tile and frame edges), spp 21 (a partial 16-sample group), streams of 7
    samples (not a multiple of 4: the per-lane ChaCha path) and of 12 (quad path, batches not 16-aligned), a shard of
    a balanced 3-way frame: against the oracle, exact ray counts."""
    from rtpotato import _ffi as F
    sc, p0 = _scene("bunny_full", 53, 37, 21)
    for sps in (7, 12, 0):
        for tw, th in ((7, 5), (32, 32)):
            p = replace(p0, samples_per_stream=sps, tile_w=tw, tile_h=th)
            rgb, fg, st, flags = _render(gpu, sc, p, primary="on")
            assert flags & F.RP_FRAME_PRIMARY_PASS
            ref, ref_fg, ctr = oracle_render(sc, p, threads=8, foreground=True)
            m = shard_mask(p)
            assert_parity(compare(rgb, ref, m))
            assert (st["rays"], st["samples"]) == (ctr["rays"], ctr["samples"]), (sps, tw, st, ctr)
            assert np.array_equal(fg[m], ref_fg[m])
    p = replace(p0, shard=1, num_shards=3, tile_w=8, tile_h=8)
    rgb, _, st, flags = _render(gpu, sc, p, primary="on")
    assert flags & F.RP_FRAME_PRIMARY_PASS
    ref, _, ctr = oracle_render(sc, p, threads=8)
    assert_parity(compare(rgb, ref, shard_mask(p)))
    assert st["rays"] == ctr["rays"]


def test_primary_pass_skipped_for_lens_cameras(gpu):
    """three_balls has lens_radius 0.1: camera rays depend on the main stream's UnitDisk draw, so no pass runs; the frame
    equals the oracle's."""
    from rtpotato import _ffi as F
    sc, p = _scene("three_balls", 48, 32, 4)
    assert sc.camera.lens_radius > 0
    rgb, _, st, flags = _render(gpu, sc, p, primary="on")
    assert not flags & F.RP_FRAME_PRIMARY_PASS
    ref, _, ctr = oracle_render(sc, p, threads=8)
    assert_parity(compare(rgb, ref))
    assert st["rays"] == ctr["rays"]


def test_primary_pass_auto_is_off(gpu):
    """AUTO resolves to OFF (the pass lost on both configs): no pass, no hint buffer use."""
    from rtpotato import _ffi as F
    sc, p = _scene("bunny_full", 32, 32, 4)
    _, _, _, flags = _render(gpu, sc, p)
    assert not flags & F.RP_FRAME_PRIMARY_PASS


def test_primary_pass_c3_tile_full_spp(gpu):
    """C3's scene at its full 256 spp on a 96 x 64 crop, default streams and one stream per pixel: pass on = off."""
    sc, p = _scene("bunny_full", 96, 64, 256)
    _on_off(gpu, sc, p)
    _on_off(gpu, sc, replace(p, samples_per_stream=256))


@pytest.mark.parametrize("sps", [0, 256, 7])
def test_learned_unit_order_same_frame(gpu, sps):
    """rp_scene_options.unit_order (rp_sched.hip): the second frame on a workspace hands its units out longest first by
    the first frame's durations -- a different schedule, the same frame bit for bit (per-unit seeding), against the
    oracle too; with RP_UNITS_TILES no frame does."""
    from rtpotato import _ffi as F
    sc, p = _scene("bunny_full", 72, 40, 64)
    p = replace(p, samples_per_stream=sps, tile_w=16, tile_h=16)
    with gpu.DeviceScene(sc, options={"unit_order": "learned"}) as ds:
        a, fa, sa = ds.render(p, foreground=True)
        f1 = ds.frame_info()
        b, fb, sb = ds.render(p, foreground=True)
        f2 = ds.frame_info()
    assert not f1 & F.RP_FRAME_UNIT_ORDER and f2 & F.RP_FRAME_UNIT_ORDER, (f1, f2)
    assert np.array_equal(a, b) and np.array_equal(fa, fb) and sa["rays"] == sb["rays"]
    ref, _, ctr = oracle_render(sc, p, threads=8)
    assert_parity(compare(b, ref))
    assert sb["rays"] == ctr["rays"]
    with gpu.DeviceScene(sc, options={"unit_order": "tiles"}) as ds:
        ds.render(p)
        c, _, sc_ = ds.render(p)
        assert not ds.frame_info() & F.RP_FRAME_UNIT_ORDER
    assert np.array_equal(c, b) and sc_["rays"] == sb["rays"]
