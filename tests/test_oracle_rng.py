"""Pins the oracle's RNG (the reference's randomness.rs on rand 0.8 StdRng) with known-answer vectors.

- ChaCha20 block function: RFC 7539 section 2.3.2 test vector and the all-zero key/nonce keystream
  (the values rand_chacha 0.3's own `test_chacha_true_values_a` checks), optionally cross-checked
  against `openssl enc -chacha20` on random keys.
- StdRng (ChaCha12): rand 0.8's value-stability test `test_stdrng_construction` (src/rngs/std.rs):
  from_seed([1,0,0,0, 23,0,0,0, 200,1,0,0, 210,30,0,0, 0...]) -> next_u64 = 10719222850664546238, then
  StdRng::from_rng(rng0) -> next_u64 = 14064965282130556830.  This pins ChaCha12, the 64-bit counter
  layout, BlockRng's u64 assembly and fill_bytes.
- seed_from_u64 (rand_core 0.6 PCG32 expansion) is restated from the published algorithm: no vector
  exists; it is cross-checked against the independent host implementation (rtpotato.rng).
"""
import shutil
import subprocess

import numpy as np
import pytest


def test_chacha20_rfc7539_block(oracle):
    key = [int.from_bytes(bytes(range(4 * i, 4 * i + 4)), "little") for i in range(8)]
    # RFC 7539 2.3.2: counter = 1, nonce = 00:00:00:09:00:00:00:4a:00:00:00:00 (96-bit layout ==
    # 64-bit counter word 13 = 0x09000000, stream word 14 = 0x4a000000)
    out = oracle.chacha_block(key, 1 | (0x09000000 << 32), 0x4A000000, 20)
    assert out == [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204,
                   0x4E6CD4C3, 0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE,
                   0xE883D0CB, 0x4E3C50A2]


def test_chacha20_zero_key_keystream(oracle):
    assert oracle.chacha_block([0] * 8, 0, 0, 20) == [
        0xADE0B876, 0x903DF1A0, 0xE56A5D40, 0x28BD8653, 0xB819D2BD, 0x1AED8DA0, 0xCCEF36A8, 0xC70D778B,
        0x7C5941DA, 0x8D485751, 0x3FE02477, 0x374AD8B8, 0xF4B8436A, 0x1CA11815, 0x69B687C3, 0x8665EEB2]
    assert oracle.chacha_block([0] * 8, 1, 0, 20) == [
        0xBEE7079F, 0x7A385155, 0x7C97BA98, 0x0D082D73, 0xA0290FCB, 0x6965E348, 0x3E53C612, 0xED7AEE32,
        0x7621B729, 0x434EE69C, 0xB03371D5, 0xD539D874, 0x281FED31, 0x45FB0A51, 0x1F0AE1AC, 0x6F4D794B]


@pytest.mark.skipif(shutil.which("openssl") is None, reason="openssl not available")
def test_chacha20_against_openssl(oracle):
    rng = np.random.default_rng(1)
    for _ in range(4):
        key = rng.integers(0, 2**32, size=8, dtype=np.uint64).astype(np.uint32)
        ctr = int(rng.integers(0, 2**31))
        nonce = int(rng.integers(0, 2**63))
        kb = key.astype("<u4").tobytes()
        iv = ctr.to_bytes(4, "little") + (0).to_bytes(4, "little") + nonce.to_bytes(8, "little")
        # openssl's 16-byte IV = 32-bit counter || 96-bit nonce; our 64-bit counter's high word is the
        # first nonce word (0 here), the 64-bit stream id the rest.
        ks = subprocess.run(["openssl", "enc", "-chacha20", "-K", kb.hex(), "-iv", iv.hex()],
                            input=bytes(64), capture_output=True, check=True).stdout
        expect = list(np.frombuffer(ks, dtype="<u4"))
        assert oracle.chacha_block(list(key), ctr, nonce, 20) == expect


def test_stdrng_value_stability(oracle):
    seed = bytes([1, 0, 0, 0, 23, 0, 0, 0, 200, 1, 0, 0, 210, 30, 0, 0] + [0] * 16)
    r0 = oracle.Rng(seed_bytes=seed)
    x0 = r0.next_u64()
    r1 = oracle.Rng(seed_bytes=r0.fill_bytes(32))
    x1 = r1.next_u64()
    assert [x0, x1] == [10719222850664546238, 14064965282130556830]


def test_blockrng_u32_u64_mixing(oracle):
    """BlockRng::next_u64 straddling the 64-word buffer end (index 63) takes the last word as the low half
    and word 0 of the next refill as the high half."""
    a = oracle.Rng(seed_u64=42)
    words = [a.next_u32() for _ in range(130)]
    b = oracle.Rng(seed_u64=42)
    for _ in range(63):
        b.next_u32()
    x = b.next_u64()
    assert x == (words[64] << 32) | words[63]
    assert b.next_u32() == words[65]


def test_gen_f64_is_top_53_bits(oracle):
    a = oracle.Rng(seed_u64=7)
    b = oracle.Rng(seed_u64=7)
    for _ in range(100):
        u = a.next_u64()
        assert b.gen() == (u >> 11) * 2.0**-53


def test_host_rng_matches_oracle_stream(oracle):
    """rtpotato.rng (numpy, used to generate scenes) == the oracle's StdRng for seed_from_u64 and from_seed."""
    from rtpotato.rng import StdRng
    for seed in (0, 1, 0x5EED0001, 0xC5, 2**64 - 1):
        ref = oracle.stream_u64(seed, 300)
        r = StdRng.seed_from_u64(seed)
        got = np.array([r.next_u64() for _ in range(5)] + list(r.next_u64_array(295)), dtype=np.uint64)
        assert np.array_equal(got, ref), seed
    r = StdRng.from_seed(bytes([249] * 32))
    o = oracle.Rng(seed_bytes=bytes([249] * 32))
    assert [r.next_u64() for _ in range(70)] == [o.next_u64() for _ in range(70)]


def test_distributions(oracle):
    r = oracle.Rng(seed_u64=3)
    for _ in range(2000):
        x, y = r.unit_disk()
        assert x * x + y * y < 1.0
        bx, by, bz = r.unit_ball()
        assert (bx * bx + by * by) + bz * bz < 1.0
        sx, sy, sz = r.unit_sphere()
        assert abs((sx * sx + sy * sy) + sz * sz - 1.0) < 1e-12
    # rejection sampling consumes the documented draws: UnitDisk = 2 per attempt
    a, b = oracle.Rng(seed_u64=11), oracle.Rng(seed_u64=11)
    a.unit_disk()
    n = 0
    while True:
        x = 2.0 * b.gen() - 1.0
        y = 2.0 * b.gen() - 1.0
        n += 2
        if x * x + y * y < 1.0:
            break
    assert a.next_u64() == b.next_u64()


def test_noise_integer_wrapping(oracle):
    """randomness.rs:91-105: wrapping isize arithmetic, arithmetic right shift."""
    M = 2**64

    def ref(x, y, z, s):
        h = (0x369E6D3B899E43CF * x + 0x53F89E7FFDA3B07D * y + 0x3B13C1CA4937E629 * z + 0x577C2C6E4019D645 * s) % M
        hs = h - M if h >= 2**63 else h
        h = ((hs >> 13) % M) ^ h
        h = (h * ((h * h * 60493 + 19990303) % M) + 1376312589) % M
        return h - M if h >= 2**63 else h

    for args in [(0, 0, 0, 0), (1, -2, 3, 4), (-7, 123456789, -987654321, 2**40), (2**62, -(2**62), 5, -1)]:
        assert oracle.lib().or_noise_integer(*args) == ref(*args)
    assert oracle.lib().or_noise_real(1, 2, 3, 4) == ref(1, 2, 3, 4) / float(2**63 - 1)


def test_kernel_draw_conversion_is_exact():
    """The kernel's two-FMA forms of rand 0.8's Standard f64 (rp_kernel.hip words_f64 / words_sym) equal
    `(u >> 11) * 2^-53` and `2.0 * that - 1.0` (randomness.rs:24,42,61) bit for bit: every term is exact.
    Checked with the host libm's correctly rounded fma over random and edge-case words."""
    import ctypes
    import struct
    libm = ctypes.CDLL("libm.so.6")
    fma = libm.fma
    fma.restype = ctypes.c_double
    fma.argtypes = [ctypes.c_double] * 3
    rng = np.random.default_rng(7)
    words = [int(x) for x in rng.integers(0, 2**64, size=20000, dtype=np.uint64)]
    words += [0, 1, 2**11 - 1, 2**11, 2**32 - 1, 2**32, 2**63, 2**64 - 1, 2**64 - 2**11, 2**64 - 2**11 - 1]
    bits = lambda x: struct.pack("<d", x)
    for u in words:
        lo, hi = u & 0xFFFFFFFF, u >> 32
        ref = float(u >> 11) * (1.0 / 9007199254740992.0)
        f = fma(float(hi), 2.0**-32, float(lo >> 11) * 2.0**-53)
        sym = fma(float(hi), 2.0**-31, fma(float(lo >> 11), 2.0**-52, -1.0))
        assert bits(f) == bits(ref), u
        assert bits(sym) == bits(2.0 * ref - 1.0), u
