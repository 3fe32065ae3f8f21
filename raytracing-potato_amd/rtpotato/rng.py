"""Host-side rand 0.8 StdRng (ChaCha12) for scene generation (example_scenes.rs:98-133 more_balls, the
synthetic C5 mesh).  numpy-vectorised over blocks so that bulk draws (tens of millions) stay fast.

Stream semantics: rand_chacha 0.3 (64-bit block counter in words 12-13, zero nonce), rand_core 0.6
seed_from_u64 (PCG32 expansion) and Standard f64 = (next_u64 >> 11) * 2^-53.  The same stream is
produced on the device by rp_kernel.hip; this module is only used on the host to build scenes.
"""
from __future__ import annotations

import numpy as np

_CONST = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)
MASK64 = (1 << 64) - 1
BULK_DRAWS = 1 << 20  # draws per call from which the threaded C++ generator takes over


def _rotl(x: np.ndarray, n: int) -> np.ndarray:
    return (x << np.uint32(n)) | (x >> np.uint32(32 - n))


def chacha_blocks(key: np.ndarray, start: int, count: int, rounds: int = 12) -> np.ndarray:
    """Keystream blocks start..start+count-1 as a (count, 16) uint32 array."""
    ctr = np.arange(start, start + count, dtype=np.uint64)
    s = np.empty((16, count), dtype=np.uint32)
    s[0:4] = _CONST[:, None]
    s[4:12] = np.asarray(key, dtype=np.uint32)[:, None]
    s[12] = (ctr & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    s[13] = (ctr >> np.uint64(32)).astype(np.uint32)
    s[14] = 0
    s[15] = 0
    x = [s[i].copy() for i in range(16)]

    def qr(a, b, c, d):
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 16)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 12)
        x[a] += x[b]; x[d] ^= x[a]; x[d] = _rotl(x[d], 8)
        x[c] += x[d]; x[b] ^= x[c]; x[b] = _rotl(x[b], 7)

    with np.errstate(over="ignore"):
        for _ in range(rounds // 2):
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
        out = np.stack([x[i] + s[i] for i in range(16)], axis=1)
    return out


def pcg32_seed(state: int) -> bytes:
    """rand_core 0.6 seed_from_u64 -> 32-byte seed."""
    out = bytearray()
    state &= MASK64
    for _ in range(8):
        state = (state * 6364136223846793005 + 11634580027462260723) & MASK64
        xs = (((state >> 18) ^ state) >> 27) & 0xFFFFFFFF
        rot = state >> 59
        x = ((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF
        out += x.to_bytes(4, "little")
    return bytes(out)


class StdRng:
    """rand::rngs::StdRng with u64-granular draws (every draw in the reference is Standard f64)."""

    def __init__(self, seed: bytes):
        assert len(seed) == 32
        self.key = np.frombuffer(seed, dtype="<u4").astype(np.uint32)
        self.pos = 0  # next u64 index in the stream
        self._cache_start = 0
        self._cache = np.zeros(0, dtype=np.uint64)

    @classmethod
    def from_seed(cls, seed) -> "StdRng":
        return cls(bytes(seed))

    @classmethod
    def seed_from_u64(cls, state: int) -> "StdRng":
        return cls(pcg32_seed(state))

    def _ensure(self, n: int) -> None:
        end = self.pos + n
        if self._cache_start <= self.pos and end <= self._cache_start + len(self._cache):
            return
        first_block = self.pos // 8
        n_blocks = (end + 7) // 8 - first_block + 8
        words = chacha_blocks(self.key, first_block, n_blocks).reshape(-1)
        self._cache = words[0::2].astype(np.uint64) | (words[1::2].astype(np.uint64) << np.uint64(32))
        self._cache_start = first_block * 8

    def next_u64_array(self, n: int) -> np.ndarray:
        if n >= BULK_DRAWS:  # bulk: the host library's threaded ChaCha12 (rph_stdrng_u64), same stream
            import ctypes
            from . import _ffi as F
            out = np.empty(n, dtype=np.uint64)
            seed = np.ascontiguousarray(self.key, dtype="<u4").tobytes()
            F.check_host(F.host().rph_stdrng_u64(seed, self.pos, n, out.ctypes.data))
            self.pos += n
            return out
        self._ensure(n)
        a = self._cache[self.pos - self._cache_start: self.pos - self._cache_start + n]
        self.pos += n
        return a

    def next_u64(self) -> int:
        return int(self.next_u64_array(1)[0])

    def gen_f64_array(self, n: int) -> np.ndarray:
        return (self.next_u64_array(n) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)

    def gen(self) -> float:
        return float(self.gen_f64_array(1)[0])

    def closed_range(self, lo: float, hi: float) -> float:  # randomness.rs:12-16
        return lo + self.gen() * (hi - lo)

    def bernoulli(self, p: float) -> bool:  # randomness.rs:78-82
        return self.gen() < p
