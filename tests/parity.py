"""Shared parity helpers (test infrastructure): run the CPU oracle on the same inputs as librp.so and
compare.  The contract (BASELINE.json north_star): per-pixel linear RGB L-inf < 1e-3 against the
reference CPU render under identical RNG seeding.  Paths are expected to be the reference's exactly,
so in practice almost every pixel agrees to ~1e-15 (the GPU accumulates the path throughput forward,
the reference recursively: last-ulp differences only).
"""
from __future__ import annotations

import ctypes

import numpy as np

TOL_LINF = 1e-3    # north_star tolerance on linear RGB per pixel
TOL_EXACT = 1e-12  # "same path" threshold used for the diagnostic bit-close fraction


def oracle_render(scene, params, threads: int = 8, foreground: bool = False):
    from oracle import oracle_py as O
    d = scene.desc()
    os_ = O.OracleScene(d.addr(), d)
    cam = scene.camera.to_c()
    p = params.to_c()
    try:
        return os_.render(ctypes.addressof(cam), ctypes.addressof(p), params.width, params.height, threads,
                          foreground)
    finally:
        os_.close()


def shard_mask(params) -> np.ndarray:
    from rtpotato.scene import shard_slot_pixels
    idx = shard_slot_pixels(params)
    m = np.zeros(params.width * params.height, dtype=bool)
    m[idx[idx >= 0]] = True
    return m.reshape(params.height, params.width)


def compare(gpu_rgb: np.ndarray, ref_rgb: np.ndarray, mask: np.ndarray | None = None) -> dict:
    a, b = gpu_rgb, ref_rgb
    if mask is not None:
        a, b = a[mask], b[mask]
    diff = np.abs(a - b)
    both_nan = np.isnan(a) & np.isnan(b)
    diff = np.where(both_nan, 0.0, diff)
    per_px = diff.reshape(-1, 3).max(axis=1)
    nan_px = np.isnan(per_px)  # NaN on one side only (both-NaN channels count 0 above)
    return {
        # a one-sided NaN is an infinite error: it fails the L-inf bar by itself
        "linf": (float("inf") if nan_px.any() else float(per_px.max())) if per_px.size else 0.0,
        "nan_mismatch": int(np.sum(np.isnan(per_px))),
        "pixels": int(per_px.size),
        "bad": int(np.sum(per_px >= TOL_LINF)),
        "not_exact": int(np.sum(per_px > TOL_EXACT)),
        "exact_frac": float(np.mean(per_px <= TOL_EXACT)) if per_px.size else 1.0,
    }


def assert_parity(c: dict, min_exact: float = 0.999) -> None:
    """The parity bar on a compare() result: no one-sided NaN, per-pixel L-inf < TOL_LINF, and at least
    `min_exact` of the pixels equal to 1e-12 (the same paths)."""
    assert c["nan_mismatch"] == 0, c
    assert c["linf"] < TOL_LINF, c
    assert c["exact_frac"] >= min_exact, c
