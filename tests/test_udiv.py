"""The unit decode's division by launch constants (raytracing-potato_amd/csrc/rp_kernel.h make_div32, used by
rp_device.h fetch_pixel): floor(n / d) = (n * m) >> s with l = ceil(log2 d), s = 31 + l, m = ceil(2^s / d), for every
numerator n < 2^31 (rp_api.cpp refuses shards of >= 2^31 units).  The header's own function (through the
librp_host.so test hook rph_make_div32, compiled from the same rp_kernel.h) is checked against Python's integer
division over edge and random cases, and against a restatement of its arithmetic; the GPU parity tests exercise the
kernel's use of the numbers."""
import ctypes
import random


def make_div32(d):
    l = 0
    while (1 << l) < d:
        l += 1
    s = 31 + l
    return ((1 << s) + d - 1) // d, s


def udiv(n, m, s):
    return ((n * m) & (2 ** 64 - 1)) >> s  # a 32 x 32 -> 64-bit product, shifted


def header_div32(d):
    from rtpotato import _ffi as F
    m, s = ctypes.c_uint32(), ctypes.c_uint32()
    F.check_host(F.host().rph_make_div32(d, ctypes.byref(m), ctypes.byref(s)))
    return m.value, s.value


def test_magic_division_is_exact_below_2_31():
    rng = random.Random(7)
    ds = list(range(1, 3000)) + [2 ** k + o for k in range(1, 32) for o in (-1, 0, 1)]
    ds += [rng.randrange(1, 2 ** 32) for _ in range(3000)]
    for d in ds:
        if not 1 <= d < 2 ** 32:
            continue
        m, s = header_div32(d)
        assert (m, s) == make_div32(d), d
        assert m < 2 ** 32 and s <= 63
        top = (2 ** 31 - 1) // d * d
        for n in [0, 1, d - 1, d, d + 1, top, top - 1, 2 ** 31 - 1] + [rng.randrange(2 ** 31) for _ in range(50)]:
            if 0 <= n < 2 ** 31:
                assert udiv(n, m, s) == n // d, (n, d)
