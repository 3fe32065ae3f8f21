"""Host-side pieces (librp_host.so) against the oracle's restatements and the reference's own assets:
obj::load (mesh.rs:145-183), tga::load/save (image.rs:73-137), to_srgb_u8 (utility.rs:212-220),
Transformation::lookat (utility.rs:172-177), and the packed asset fixtures used on the GPU box.
"""
import os

import numpy as np
import pytest

from conftest import HAVE_REFERENCE, REFERENCE

ref_only = pytest.mark.skipif(not HAVE_REFERENCE, reason="reference assets not mounted")


@ref_only
@pytest.mark.parametrize("name", ["bunny", "bunny_flat"])
def test_obj_load_matches_oracle_and_fixture(oracle, name):
    from rtpotato import assets
    path = os.path.join(REFERENCE, "assets", name + ".obj")
    m = assets.obj_load(path)
    p, n, uv, idx = oracle.obj_load(path)
    assert np.array_equal(m.positions, p) and np.array_equal(m.normals, n)
    assert np.array_equal(m.uvs, uv) and np.array_equal(m.indices, idx)
    fx = np.load(os.path.join(assets.ASSET_DIR, name + ".npz"))
    assert np.array_equal(fx["positions"], m.positions) and np.array_equal(fx["indices"], m.indices)
    assert np.array_equal(fx["normals"], m.normals) and np.array_equal(fx["uvs"], m.uvs)


@ref_only
def test_obj_bunny_shape():
    """bunny.obj has 2,503 v, 2,503 vn, 0 vt, 4,968 tris of `f a//a` -> 2,503 unique
    (p, n, t) vertices; bunny_flat.obj dedups to 14,902 vertices."""
    from rtpotato import assets
    m = assets.load_mesh("bunny")
    assert m.positions.shape == (2503, 3) and m.indices.shape == (4968 * 3,)
    assert np.all(m.uvs == 0.0)
    assert assets.load_mesh("bunny_flat").positions.shape == (14902, 3)


def test_obj_edge_cases(tmp_path, oracle):
    from rtpotato import assets
    from rtpotato import _ffi as F
    src = ("# comment\no obj\nv 0 0 0\nv 1.5e0 0 0\nv 0 -1. 0\nv  0 0 2\nvt 0.25 0.75\nvn 0 0 1\ns off\n"
           "f 1/1/1 2/1/1 3/1/1\nf 1 2 4 \nf 2//1 3//1 4//1\n  f 1 2 3\nf 4/1 3/1 2/1\n")
    p = tmp_path / "m.obj"
    p.write_text(src)
    m = assets.obj_load(str(p))
    op, on, ouv, oidx = oracle.obj_load(str(p))
    assert np.array_equal(m.positions, op) and np.array_equal(m.indices, oidx)
    assert np.array_equal(m.normals, on) and np.array_equal(m.uvs, ouv)
    assert len(m.indices) == 12  # the indented face line is not parsed (mesh.rs:117-120 skips it)
    assert m.positions[1, 0] == 1.5 and m.uvs[0].tolist() == [0.25, 0.75]
    quad = tmp_path / "q.obj"
    quad.write_text("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nf 1 2 3 4\n")
    with pytest.raises(F.RPError):
        assets.obj_load(str(quad))  # "Non-triangular face are not supported"
    bad = tmp_path / "b.obj"
    bad.write_text("v 0 0 0\nf 1 2 3\n")
    with pytest.raises(F.RPError):
        assets.obj_load(str(bad))  # index out of bounds: the reference panics


def test_tga_roundtrip_and_flip(tmp_path, oracle):
    from rtpotato import assets
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(7, 11, 4), dtype=np.uint8)
    p = str(tmp_path / "a.tga")
    assets.tga_save(p, img)
    assert np.array_equal(assets.tga_load(p), img)
    assert np.array_equal(oracle.tga_load(p), img)
    raw = open(p, "rb").read()
    assert raw[2] == 2 and raw[16] == 32 and raw[17] == 0  # tga::save header (image.rs:121-124)
    # a 24-bit top-left-origin file: rows flipped into bottom-row-first storage, alpha 0xff
    hdr = bytearray(18)
    hdr[2], hdr[12], hdr[14], hdr[16], hdr[17] = 2, 3, 2, 24, 0x20
    body = bytes([1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18])
    q = str(tmp_path / "b.tga")
    open(q, "wb").write(bytes(hdr) + body)
    got = assets.tga_load(q)
    assert np.array_equal(got, oracle.tga_load(q))
    assert got[1, 0].tolist() == [3, 2, 1, 255] and got[0, 0].tolist() == [12, 11, 10, 255]


@ref_only
def test_earthmap_fixture():
    from rtpotato import assets
    img = assets.tga_load(os.path.join(REFERENCE, "assets", "earthmap.tga"))
    assert img.shape == (512, 1024, 4)
    assert np.array_equal(img, assets.load_image("earthmap"))


def test_srgb_and_lookat_match_oracle(oracle):
    from rtpotato import assets
    from rtpotato.scene import Transformation
    rng = np.random.default_rng(2)
    x = rng.uniform(-0.2, 1.2, size=(50, 40, 3))
    x[0, 0] = [np.nan, 0.0, 1.0]
    assert np.array_equal(assets.to_srgb_u8(x), oracle.to_srgb_u8(x))
    for pos, tgt in [((-1.5, 1.5, 2.5), (0.0, 0.5, 0.0)), ((13.0, 7.0, 3.0), (0, 0, 0)), ((6, 2, 4), (0, 0, 0))]:
        t = Transformation.lookat(pos, tgt, (0.0, 1.0, 0.0))
        assert t.orientation == oracle.lookat(pos, tgt, (0.0, 1.0, 0.0))


def test_sky_panorama_deterministic():
    """The synthesised stand-in for the missing sky_panorama.tga is a pure function of (w, h)."""
    import hashlib
    from rtpotato import assets
    a = assets.sky_panorama(256, 128)
    b = np.empty_like(a)
    from rtpotato import _ffi as F
    F.check_host(F.host().rph_sky_panorama(256, 128, b.ctypes.data))
    assert np.array_equal(a, b)
    assert a[..., 3].min() == 255
    assert a[0].mean() < a[-1].mean()  # nadir (row 0) darker than the zenith
    full = assets.sky_panorama()
    assert full.shape == (1024, 2048, 4)
    digest = hashlib.sha256(full.tobytes()).hexdigest()
    golden = os.path.join(os.path.dirname(__file__), "golden", "sky_panorama.sha256")
    if os.path.exists(golden):
        assert open(golden).read().strip() == digest


def test_u8_unit_division_free_is_exact():
    """rp_kernel.hip u8_unit(): x/255.0 for every byte x as fl(x*fl(1/255)) plus one FMA residual
    correction -- bit-identical to the correctly rounded division texture.rs:47 performs."""
    import ctypes
    import struct
    libm = ctypes.CDLL("libm.so.6")
    libm.fma.restype = ctypes.c_double
    libm.fma.argtypes = [ctypes.c_double] * 3
    R = 1.0 / 255.0
    for x in range(256):
        q0 = float(x) * R
        q = libm.fma(libm.fma(-q0, 255.0, float(x)), R, q0)
        assert struct.pack("<d", q) == struct.pack("<d", float(x) / 255.0), x


def test_bulk_stdrng_matches_oracle_stream(oracle):
    """rph_stdrng_u64 (the threaded host generator behind rtpotato.rng bulk draws, used to build the C5
    mesh) is rand 0.8 StdRng's stream: equal to the oracle's next_u64 sequence, from any start draw."""
    import numpy as np
    from rtpotato.rng import BULK_DRAWS, StdRng
    for seed in (0xC5, 0, 2**64 - 1):
        ref = oracle.stream_u64(seed, 3000)
        r = StdRng.seed_from_u64(seed)
        assert np.array_equal(r.next_u64_array(BULK_DRAWS)[:3000], ref)
        r = StdRng.seed_from_u64(seed)
        r.next_u64_array(777)
        assert np.array_equal(r.next_u64_array(BULK_DRAWS)[:3000 - 777], ref[777:])
