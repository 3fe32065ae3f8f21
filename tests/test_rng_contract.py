"""The RNG contract's sample batching (include/rp.h "Determinism"), on the CPU oracle.

Batch b of pixel (i, j) is its own stream seed_from_u64(seed + b*W*H + j*W + i) over samples Sb..Sb+S-1 (S = RP_SAMPLES_PER_STREAM = 32),
so batch 1 of a frame with seed X is batch 0 of the same pixel in a frame with seed X + W*H: an (S+6)-spp
frame must equal the spp-weighted mean of an S-spp frame (seed X) and a 6-spp frame (seed X + W*H).
Frames with spp <= S are the single per-pixel stream, which the golden fixtures pin.
"""
from dataclasses import replace

import numpy as np

from parity import oracle_render

SAMPLES_PER_STREAM = 32  # include/rp.h RP_SAMPLES_PER_STREAM


def test_batches_compose_from_single_stream_frames():
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    w, h = 20, 12
    scene = scenes.configure(scenes.bunny_full(), w, h)
    seed = 777
    S = SAMPLES_PER_STREAM
    full, fg_full, c_full = oracle_render(scene, RenderParams(w, h, S + 6, 8, seed), threads=8, foreground=True)
    a, fg_a, c_a = oracle_render(scene, RenderParams(w, h, S, 8, seed), threads=8, foreground=True)
    b, fg_b, c_b = oracle_render(scene, RenderParams(w, h, 6, 8, seed + w * h), threads=8, foreground=True)
    np.testing.assert_allclose(full, (a * S + b * 6) / (S + 6), rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(fg_full, (fg_a.astype(np.float64) * S + fg_b * 6) / (S + 6), rtol=1e-6)
    assert c_full["rays"] == c_a["rays"] + c_b["rays"]
    assert c_full["samples"] == (S + 6) * w * h


def test_single_batch_frames_are_the_per_pixel_stream():
    """spp <= S: one stream per pixel, seed + j*W + i -- a pixel's value does not depend on spp's batch
    count and a sub-rectangle shard agrees with the full frame (per-pixel seeding)."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    w, h = 16, 10
    scene = scenes.configure(scenes.bunny_full(), w, h)
    p = RenderParams(w, h, SAMPLES_PER_STREAM, 8, 5)
    full, _, _ = oracle_render(scene, p, threads=4)
    shard, _, _ = oracle_render(scene, replace(p, tile_w=8, tile_h=8, shard=1, num_shards=2), threads=4)
    m = np.any(shard != 0, axis=2)
    assert m.sum() > 0
    assert np.array_equal(full[m], shard[m])


def test_samples_per_stream_parameter():
    """rp_render_params.samples_per_stream N: N >= spp is SURVEY.md 8c's one stream per pixel whatever N is;
    N = 1 makes sample s its own stream seed + s*W*H (the mean of spp one-sample frames)."""
    from rtpotato import scenes
    from rtpotato.scene import RenderParams
    w, h, spp, seed = 12, 8, 40, 31
    scene = scenes.configure(scenes.bunny_full(), w, h)
    one, _, c1 = oracle_render(scene, RenderParams(w, h, spp, 8, seed, samples_per_stream=spp), threads=8)
    big, _, c2 = oracle_render(scene, RenderParams(w, h, spp, 8, seed, samples_per_stream=1000), threads=8)
    assert np.array_equal(one, big) and c1["rays"] == c2["rays"]
    default, _, _ = oracle_render(scene, RenderParams(w, h, spp, 8, seed), threads=8)
    assert not np.array_equal(one, default)  # 40 > 32: the default splits the pixel into two streams
    single, _, c3 = oracle_render(scene, RenderParams(w, h, 3, 8, seed, samples_per_stream=1), threads=8)
    parts = [oracle_render(scene, RenderParams(w, h, 1, 8, seed + b * w * h), threads=8) for b in range(3)]
    np.testing.assert_allclose(single, sum(p[0] for p in parts) / 3, rtol=1e-12, atol=1e-14)
    assert c3["rays"] == sum(p[2]["rays"] for p in parts)
