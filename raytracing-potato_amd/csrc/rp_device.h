// rp_device.h -- device code of the gfx950 kernels (rp_kernel.hip: the persistent megakernel and the closest-hit
// query kernel): the rand 0.8 StdRng keystream, f64 vector math, the
// conservative-f32 wide-BVH traversal with exact f64 primitive tests, and the materials/textures.
//
// Arithmetic is IEEE binary64 in the reference's exact operation order (no contraction: the kernels are
// compiled with -ffp-contract=off and the pragma below), so paths -- and the RNG draws they consume --
// are the reference's.  References: render.rs:32-146, bvh.rs:93-124, hittable.rs:39-108,
// material.rs:27-179, texture.rs:21-118, randomness.rs:9-110, utility.rs:67-154.
#pragma once
#include <hip/hip_runtime.h>

#include "rp_kernel.h"

#pragma clang fp contract(off)

// Every compile-time knob below changes timing only.  Experiments that change results (timing ablations
// with wrong streams or colours) are not kept in this file, and a build asking for one is refused so a
// library that writes wrong frames can never be produced from it.
#if defined(RPK_ABLATE_RNG) || defined(RPK_ABLATE_UV) || defined(RPK_ABLATE_TEX) || defined(RPK_ABLATE_METAL) || \
    defined(RPK_BATCH_LEAF)
#error "result-changing experiment macros are not part of the product kernel"
#endif
// Timing experiments are not compile-time switches of the product sources either: the kernel below is the
// product path only (plus the RPK_DIAG instrumentation).  tools/build_variant.sh builds an experiment from a
// patched copy of these sources; the switches of earlier rounds are refused so a stale command line cannot
// silently build something else.
#if defined(RPK_NT_STORE) || defined(RPK_NT_ALL) || defined(RPK_NT_TEX) || defined(RPK_NT_OUT) ||           \
    defined(RPK_SLAB_ALIGN) || defined(RPK_SLAB_PAD) || defined(RPK_COLD_SLAB) || defined(RPK_COLD_IN_SLAB) || \
    defined(RPK_W3) || defined(RPK_W4) || defined(RPK_WAVES) || defined(RPK_TRIES_BALL) ||             \
    defined(RPK_NO_SPECULATIVE) || defined(RPK_NODE_BREAK) || defined(RPK_TRIES) || defined(RPK_RING) ||       \
    defined(RPK_RNG_BATCH) || defined(RPK_RNG_CRIT) || defined(RPK_PRIM_BREAK) || defined(RPK_PRIO_TRAV) ||    \
    defined(RPK_PRIO_SHADE) || defined(RPK_PRIO_REFILL) || defined(RPK_SORT_Q) || defined(RPK_WF_REFILL)
#error "experiment macros are not part of the product kernel (tools/build_variant.sh patches a copy instead)"
#endif

namespace rpk {

#define RPK_INLINE __device__ __forceinline__

// Diagnostic build (-DRPK_DIAG, lib/librp_diag.so only): per-wave s_memtime phase stamps and lane
// utilisation counters into KArgs::diag.  The product build compiles none of it.
#ifdef RPK_DIAG
#define DIAG(...) __VA_ARGS__
RPK_INLINE uint64_t stamp() {
#ifdef RPK_DIAG_NOSTAMP
  return 0;
#endif
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): s_memtime returns through the LGKM counter
  return t;
}
__shared__ unsigned long long g_dreg[2 * DREG_N];
// count one execution of region r by this wave and its active lanes (leader lane only; EXEC is read
// directly, no ballot)
#define DREG(r)                                                                        \
  {                                                                                    \
    const uint64_t ex_ = __builtin_amdgcn_read_exec();                                 \
    if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(ex_)) {                       \
      atomicAdd(&g_dreg[2 * (r)], 1ull);                                               \
      atomicAdd(&g_dreg[2 * (r) + 1], (unsigned long long)__popcll(ex_));             \
    }                                                                                  \
  }
// wave-cycles spent executing a code region (its lanes active, the others masked): s_memtime around it, added by
// the wave's first active lane into g_dcyc[r] (flushed to diag[DIAG_CYC + r] at the kernel's end)
__shared__ unsigned long long g_dcyc[DCYC_N];
#define DCYC_BEGIN(v) const uint64_t v = stamp();
#define DCYC_END(r, v)                                                                 \
  {                                                                                    \
    const uint64_t ex_ = __builtin_amdgcn_read_exec();                                 \
    const uint64_t d_ = stamp() - (v);                                                 \
    if ((threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(ex_)) atomicAdd(&g_dcyc[r], (unsigned long long)d_); \
  }
#else
#define DIAG(...)
#define DREG(r)
#define DCYC_BEGIN(v)
#define DCYC_END(r, v)
#endif

static constexpr int BLOCK = RENDER_BLOCK;
typedef float f2 __attribute__((ext_vector_type(2)));
RPK_INLINE f2 pk_fma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
static constexpr uint32_t STACK_SLACK = 3;  // spare LDS stack entries for the branchless push (writes reach sp+2 <= cap+2)
static constexpr double RAY_EPSILON = 1e-3;  // utility.rs:30
static constexpr double SMOL = 1e-7;         // utility.rs:31
static constexpr double PI_ = 3.14159265358979323846;
static constexpr double TAU_ = 6.28318530717958647692;
static constexpr double INF = __builtin_huge_val();

// ------------------------------------------------------------------ RNG (rand 0.8 StdRng) -------

RPK_INLINE uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define RPK_QR(a, b, c, d)              \
  a += b; d ^= a; d = rotl(d, 16);      \
  c += d; b ^= c; b = rotl(b, 12);      \
  a += b; d ^= a; d = rotl(d, 8);       \
  c += d; b ^= c; b = rotl(b, 7);

// ChaCha12 block (rand_chacha 0.3: 64-bit block counter in words 12-13, zero nonce).
RPK_INLINE void chacha12(const uint32_t k[8], uint32_t ctr, uint32_t o[16]) {
  uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
  uint32_t x4 = k[0], x5 = k[1], x6 = k[2], x7 = k[3], x8 = k[4], x9 = k[5], x10 = k[6], x11 = k[7];
  uint32_t x12 = ctr, x13 = 0, x14 = 0, x15 = 0;
#pragma unroll
  for (int r = 0; r < 6; r++) {
    RPK_QR(x0, x4, x8, x12);
    RPK_QR(x1, x5, x9, x13);
    RPK_QR(x2, x6, x10, x14);
    RPK_QR(x3, x7, x11, x15);
    RPK_QR(x0, x5, x10, x15);
    RPK_QR(x1, x6, x11, x12);
    RPK_QR(x2, x7, x8, x13);
    RPK_QR(x3, x4, x9, x14);
  }
  o[0] = x0 + 0x61707865u; o[1] = x1 + 0x3320646eu; o[2] = x2 + 0x79622d32u; o[3] = x3 + 0x6b206574u;
  o[4] = x4 + k[0]; o[5] = x5 + k[1]; o[6] = x6 + k[2]; o[7] = x7 + k[3];
  o[8] = x8 + k[4]; o[9] = x9 + k[5]; o[10] = x10 + k[6]; o[11] = x11 + k[7];
  o[12] = x12 + ctr; o[13] = x13; o[14] = x14; o[15] = x15;
}

// The same block computed by the four lanes of a DPP quad together (the coherent primary pass: four neighbouring
// samples of a pixel share a jitter block).  Lane c of the quad holds column c of the state -- words c, 4 + c, 8 + c,
// 12 + c -- so a column round is one quarter round per lane, and a diagonal round is one quarter round per lane after
// rotating rows 1, 2, 3 of the state by 1, 2, 3 lanes (quad_perm DPP moves), rotated back after it.  A quarter of a
// block's VALU per lane.  Every lane of the quad must be active and pass the same key and counter; returns the
// lane's column of the output block (words c, 4 + c, 8 + c, 12 + c).
RPK_INLINE uint32_t quad_rot(uint32_t v, int by) {  // lane c of a quad reads lane (c + by) & 3
  return by == 1 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x39, 0xF, 0xF, false)
       : by == 2 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false)
                 : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x93, 0xF, 0xF, false);
}
RPK_INLINE uint4 chacha12_quad(const uint32_t k[8], uint32_t ctr) {
  const uint32_t c = __lane_id() & 3u;
  const uint32_t a0 = c == 0 ? 0x61707865u : c == 1 ? 0x3320646eu : c == 2 ? 0x79622d32u : 0x6b206574u;
  const uint32_t b0 = c == 0 ? k[0] : c == 1 ? k[1] : c == 2 ? k[2] : k[3];
  const uint32_t c0 = c == 0 ? k[4] : c == 1 ? k[5] : c == 2 ? k[6] : k[7];
  const uint32_t d0 = c == 0 ? ctr : 0u;
  uint32_t a = a0, b = b0, x = c0, d = d0;
#pragma unroll
  for (int r = 0; r < 6; r++) {
    RPK_QR(a, b, x, d);  // column c
    b = quad_rot(b, 1);
    x = quad_rot(x, 2);
    d = quad_rot(d, 3);
    RPK_QR(a, b, x, d);  // diagonal starting at word c
    b = quad_rot(b, 3);
    x = quad_rot(x, 2);
    d = quad_rot(d, 1);
  }
  return make_uint4(a + a0, b + b0, x + c0, d + d0);
}
// Row `row` of a block held column-wise by a quad (chacha12_quad): words 4 row .. 4 row + 3.  Lane m of the quad holds
// word 4 row + m in component `row` of its column; each of the four components is read from every lane (DPP
// broadcasts within the quad) and the lane keeps its own row.
RPK_INLINE uint32_t quad_bcast(uint32_t v, int from) {  // every lane of a quad reads lane `from`
  return from == 0 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xF, 0xF, false)
       : from == 1 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xF, 0xF, false)
       : from == 2 ? (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xAA, 0xF, 0xF, false)
                   : (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xFF, 0xF, 0xF, false);
}
RPK_INLINE uint4 quad_row(uint4 col, uint32_t row) {
  uint32_t o[4];
#pragma unroll
  for (int m = 0; m < 4; m++) {
    const uint32_t r0 = quad_bcast(col.x, m), r1 = quad_bcast(col.y, m), r2 = quad_bcast(col.z, m),
                   r3 = quad_bcast(col.w, m);
    o[m] = row == 0 ? r0 : row == 1 ? r1 : row == 2 ? r2 : r3;
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}

// rand_core 0.6 seed_from_u64: PCG32 expansion of the u64 into the 8 key words.
RPK_INLINE void seed_key(uint64_t state, uint32_t key[8]) {
#pragma unroll
  for (int c = 0; c < 8; c++) {
    state = state * 6364136223846793005ull + 11634580027462260723ull;
    uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    key[c] = (xs >> rot) | (xs << ((32 - rot) & 31));
  }
}

// Main stream of one pixel.  Every draw on the path is a u64 (Standard f64), so the stream is the
// keystream read two words at a time from word `pos`: exactly rand_chacha's 4-block-buffered stream.
//
// Keystream blocks are produced ahead of use into a per-lane slab in global memory (L2/MALL resident,
// ~0.7 KB per lane): a ring of RING main-stream blocks and the two camera-jitter blocks the next
// samples need.  Production happens in ONE place per round of the render loop (rng_refill), for every
// lane that has room, so a ChaCha12 block (~600 VALU) runs with nearly all 64 lanes doing useful work;
// the draw sites only load 16-word blocks from the ring.  Generating at the draw sites instead made the
// wave pay a whole block whenever ANY lane crossed a block boundary (several per round at C3).  A draw
// that finds the ring empty still generates its block in place (rare: the refill pass keeps > RNG_CRIT
// blocks ahead of every lane).
//
// Slab layout per lane (uint4 units): [0,2) key words, [2, 2+4*RING) ring (block b in slot b % RING),
// [2+4*RING, +8) jitter blocks (block b in slot b & 1).  Per-lane cursors (LDS): end = one past the
// newest ring block; jtag[2] = block held by each jitter slot.
static constexpr uint32_t RING = 8;  // slab ring capacity; a kernel keeps RngT::ring <= RING blocks ahead
static constexpr uint32_t SLAB_KEY = 0, SLAB_RING = 2, SLAB_JIT = 2 + 4 * RING;
// The pixel sum and path throughput (6 f64 per lane, read and written at every shade) live in LDS (in the
// slab: C3 +2.6 %, C5 +4.6 %); the host then keeps ~19 traversal-stack entries in LDS and spills deeper ones to
// the lane's global run (render_blocks_per_cu picks the split; bunny: 19 of 31, rarely reached).
// (v43-v47 kept the measured unit's start time in one more uint4 of the slab: 688 B per lane, and C3 wrote 70 GB per
// frame instead of 56 -- the stamp now lives in its own lane-indexed array, KScene::unit_t0)
static constexpr uint32_t SLAB_N = SLAB_JIT + 8;
// A refill pass runs when some lane is at or below RNG_CRIT blocks ahead, or RNG_BATCH lanes have room.
static constexpr uint32_t RNG_CRIT = 2, RNG_BATCH = 48;
// Traversal wave-level exits (trav_step): leave the inner-node loop once at most KScene::leaf_break lanes of
// the wave still look for a leaf (rp_scene_options.leaf_break; C3: 0 -> 3 was -2.7 % frame time, 8 is -0.8 %
// more; C5 wants 12-16), and the leaf loop once at most PRIM_BREAK lanes still test primitives (their
// remaining run is parked as a leaf entry; C3 0 -> 12: -3.7 %, C5 -0.8 %; 6-16 within 0.5 %).
static constexpr uint32_t PRIM_BREAK = 12;

// RN = ring blocks in use (a power of two <= RING): the render kernel of the quantized-node (large-scene)
// format keeps 4, the others 8 (rp_kernel.hip RingFor).
template <uint32_t RN>
struct RngT {
  static constexpr uint32_t ring = RN;
  // a lane's slab for this ring: key, RN ring blocks, 2 jitter blocks (compact: 416 B for RN = 4)
  static constexpr uint32_t jit = SLAB_RING + 4 * RN, lane_n = jit + 8;
  static_assert(RN > RNG_CRIT && RN <= RING && (RN & (RN - 1)) == 0,
                "ring: a power of two above the critical refill level (a full ring is never refilled), <= RING");
  // a lane stride of 16 B past a 32-B boundary (688 B, v43-v47) made every 64-B block dirty three 32-B sectors: +25 %
  // memory-side writes
  static_assert(lane_n % 2 == 0, "lane slab stride must be a multiple of 32 B (keystream blocks on whole sectors)");
  uint4* slab;     // global: this lane's slab
  uint32_t pos;    // next keystream word (even)
  uint32_t* end;   // LDS cursor: one past the newest ring block
  uint32_t* jtag;  // LDS cursors: jtag[0], jtag[BLOCK]
};
template <class Rng>
RPK_INLINE void store_key(Rng& r, const uint32_t k[8]) {
  r.slab[SLAB_KEY] = make_uint4(k[0], k[1], k[2], k[3]);
  r.slab[SLAB_KEY + 1] = make_uint4(k[4], k[5], k[6], k[7]);
}
RPK_INLINE void store_block(uint4* dst, const uint32_t w[16]) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
  }
}
RPK_INLINE void load_block(const uint4* src, uint32_t w[16]) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint4 v = src[q];
    w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
  }
}
template <uint32_t RN>
RPK_INLINE uint4* ring_slot(const RngT<RN>& r, uint32_t b) { return r.slab + SLAB_RING + 4 * (b & (RN - 1u)); }
template <uint32_t RN>
RPK_INLINE uint4* jit_slot(const RngT<RN>& r, uint32_t b) { return r.slab + RngT<RN>::jit + 4 * (b & 1u); }

// The refill pass (wave-uniform call site).  `seed` is the lane's unit seed (the RNG contract's
// seed_from_u64 argument).  `s` is the lane's last sample whose jitter is consumed;
// samples s+1.. need jitter blocks (s+1)/4 and the one after.  A lane with a `fresh` unit (fetched last
// round, not started) gets its key from the unit's seed and keystream block 0 here, batched with the other
// lanes' ChaCha work -- at the fetch site the whole wave paid a ChaCha block for each fetching lane.
// Position of the n-th (0-based) set bit of m (n < popcount(m)).
RPK_INLINE uint32_t nth_set(uint64_t m, uint32_t n) {
  uint32_t pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const uint32_t c = (uint32_t)__popcll(m & ((1ull << w) - 1ull));
    if (n >= c) { n -= c; m >>= w; pos += (uint32_t)w; }
  }
  return pos;
}
static_assert(BLOCK == 64, "rng_refill: a block is one wave, so a lane's slab is the wave's lane index past the first");
template <uint32_t RN>
RPK_INLINE void rng_refill(RngT<RN>& r, bool alive, bool fresh, uint64_t seed, uint32_t s, uint32_t spp) {
  const uint32_t cur = r.pos >> 4, end = *r.end, have = end - cur;
  const uint32_t b1 = (s + 1) >> 2, b2 = b1 + 1;
  const bool j1 = alive && !fresh && 4 * b1 < spp && r.jtag[(b1 & 1u) * BLOCK] != b1;
  const bool j2 = alive && !fresh && 4 * b2 < spp && r.jtag[(b2 & 1u) * BLOCK] != b2;
  const bool crit = alive && (fresh || have <= RNG_CRIT);
  const bool room = alive && (fresh || have < RN || j1 || j2);
  if (__ballot(crit) == 0 && (uint32_t)__popcll(__ballot(room)) < RNG_BATCH) return;
  // This lane's own block (room): a fresh unit's block 0, else the next ring block or a missing jitter block.
  const bool main = fresh || crit || !(j1 || j2);  // crit: have <= RNG_CRIT < RN, so the ring has room
  const uint32_t b = fresh ? 0u : (main ? end : (j1 ? b1 : b2));
  const uint32_t end1 = !room ? end : (fresh ? 1u : (main ? end + 1u : end));  // ring end after it
  const uint32_t have1 = end1 - (fresh ? 0u : cur);
  // The lanes without a block of their own this pass (full rings, retired lanes) make ring blocks for the lanes still
  // at or below the critical level after it -- up to two each, the next blocks of their streams -- in the same ChaCha
  // pass: a fresh unit leaves the pass 3 blocks ahead instead of 1, so it does not force the next two passes, and the
  // in-place fallback (gen_block: one lane, a whole wave's ChaCha time) is rarer.  Requests are numbered lane by lane,
  // first blocks before second ones; executor x (the x-th lane without a block) takes request x.
  // (Topping up every other ring with room as well cost C3 +1.0 %, C5 +2.6 %: profiles/r4/c3_c5_refill_variants_ab.json.)
  const uint32_t want = alive && have1 <= RNG_CRIT ? min(RNG_CRIT + 1u - have1, RN - have1) : 0u;
  const uint64_t m1 = __ballot(want >= 1u), m2 = __ballot(want >= 2u), ex = __ballot(!room);
  const uint32_t lane = __lane_id();
  const uint64_t below = (1ull << lane) - 1ull;
  const uint32_t n1 = (uint32_t)__popcll(m1), nreq = n1 + (uint32_t)__popcll(m2), nex = (uint32_t)__popcll(ex);
  const uint32_t xr = (uint32_t)__popcll(ex & below);
  const bool sec = !room && xr < nreq;
  uint32_t owner = lane, j = 0u;
  if (sec) {
    if (xr < n1) owner = nth_set(m1, xr);
    else { owner = nth_set(m2, xr - n1); j = 1u; }
  }
  const uint32_t slo = __shfl((uint32_t)seed, (int)owner), shi = __shfl((uint32_t)(seed >> 32), (int)owner);
  const uint32_t oend = __shfl(end1, (int)owner);
  // this lane's requests that an executor took
  const uint32_t served = (uint32_t)(want >= 1u && (uint32_t)__popcll(m1 & below) < nex) +
                          (uint32_t)(want >= 2u && n1 + (uint32_t)__popcll(m2 & below) < nex);
  if (room || sec) {
    DREG(DREG_REFILL)
    uint32_t k[8], w[16];
    // The key is recomputed from the unit's seed (PCG32 seed_from_u64, ~100 VALU) rather than loaded from the
    // slab: a slab load that misses L2 stalls the whole pass before its ChaCha work (C3 -0.7 %, C5 -0.1 %,
    // ab48).  A fresh unit still stores it for the in-place fallback (gen_block).
    seed_key(room ? seed : ((uint64_t)shi << 32 | slo), k);
    if (fresh) {
      DREG(DREG_BEGIN_PIXEL)
      store_key(r, k);
    }
    const uint32_t bb = room ? b : oend + j;
    chacha12(k, bb, w);
    // an executor's block goes into its owner's ring (lane slabs are consecutive within the block)
    uint4* dst = room ? (main ? ring_slot(r, b) : jit_slot(r, b))
                      : r.slab + ((int)owner - (int)lane) * (int)RngT<RN>::lane_n + SLAB_RING + 4u * (bb & (RN - 1u));
    store_block(dst, w);
    if (fresh) store_block(jit_slot(r, 0), w);  // block 0 is also the jitter block of samples 0-3 (render.rs:74-82)
  }
  if (room) {
    if (fresh) {
      r.pos = 0;
      r.jtag[0] = 0;
      r.jtag[BLOCK] = 0xFFFFFFFFu;
    } else if (!main) {
      r.jtag[(b & 1u) * BLOCK] = b;
    }
  }
  if (room || served) *r.end = end1 + served;
  // An executor lane stored blocks into its owner lane's slab above, and the owner reads them through ring_u64 later:
  // a cross-lane hand-off inside one wave.  One wave's memory operations stay in order, and this wavefront-scope fence
  // states the ordering for the memory model; it compiles to no instruction (the kernel's ISA is unchanged).
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// Jitter words 4s..4s+3 of the pixel-start stream (block s/4).
// Keystream block b of the lane's key into dst, for the rare draw that finds its block not made yet.  Out
// of line: the kernel is ~50 KB of code against a 64 KB instruction cache shared by two CUs, and each
// inlined ChaCha12 is ~2.5 KB that only the fallback paths execute.
static __device__ __attribute__((noinline, unused)) void gen_block(const uint4* slab, uint32_t b, uint4* dst) {
  const uint4 a = slab[SLAB_KEY], c = slab[SLAB_KEY + 1];
  const uint32_t k[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  uint32_t w[16];
  chacha12(k, b, w);
  store_block(dst, w);
}

template <uint32_t RN>
RPK_INLINE uint4 rng_jitter(RngT<RN>& r, uint32_t s) {
  const uint32_t b = s >> 2;
  if (r.jtag[(b & 1u) * BLOCK] != b) {
    DREG(DREG_JIT_FALLBACK)
    gen_block(r.slab, b, jit_slot(r, b));
    r.jtag[(b & 1u) * BLOCK] = b;
  }
  return jit_slot(r, b)[s & 3u];
}

// rand 0.8 Standard f64: (u64 >> 11) * 2^-53 (exact conversions)
RPK_INLINE double u64_to_f64(uint64_t u) { return (double)(u >> 11) * (1.0 / 9007199254740992.0); }
// The same value from the two keystream words, as hi * 2^-32 + (lo >> 11) * 2^-53: both terms and the sum
// k * 2^-53 (k < 2^53) are exact, so the FMA returns the identical double in 2 cvt + 1 mul + 1 FMA.
RPK_INLINE double words_f64(uint32_t lo, uint32_t hi) {
  return __builtin_fma((double)hi, 0x1p-32, (double)(lo >> 11) * 0x1p-53);
}
// 2 * words_f64 - 1 (the distributions' `2.0 * r - 1.0`, randomness.rs:24,42,61): 2g = k * 2^-52 is exact and
// so is k * 2^-52 - 1 (a multiple of 2^-52 of magnitude <= 1), whatever the order -- two exact FMAs.
RPK_INLINE double words_sym(uint32_t lo, uint32_t hi) {
  return __builtin_fma((double)hi, 0x1p-31, __builtin_fma((double)(lo >> 11), 0x1p-52, -1.0));
}
// Every draw reads the ring directly: the RING blocks of a lane are one circular run of 16*RING words in
// its slab (L2-resident), so stream word a sits at ring word a % (16*RING) while its block is held
// (blocks [end - RING, end)).  A draw site makes sure every block it touches is there (ring_ensure:
// generated in place when the refill pass has not made it yet, rare) and loads its u64 words with one
// dwordx2 each.  Rejection loops (UnitBall / UnitSphere / UnitDisk) load and evaluate TRIES tries at
// once and keep the first accepted one -- the draws consumed, and so the stream, are exactly the
// sequential loop's.  A wave iterates until its slowest lane accepts: with
// acceptance p a lane needs a geometric number of tries, and the wave's maximum over its ~20 shading lanes
// is ~5 single tries for the ball (p = pi/6); each round pays one ring-load latency.  (Before, a draw
// checked its block and the wave copied a 16-word block into LDS whenever any lane crossed one.)
static constexpr uint32_t TRIES = 2;  // (1 or 3 tries: +0.6 / +0.9 %; 3 or 4 for Metal alone: +0.6 / +1.3 %)
static_assert((RING & (RING - 1)) == 0, "ring_u64 indexes the ring as 16 * ring words (a power of two)");
template <uint32_t RN>
RPK_INLINE uint2 ring_u64(const RngT<RN>& r, uint32_t a) {  // stream words a, a+1 (a even)
  return reinterpret_cast<const uint2*>(r.slab + SLAB_RING)[(a & (16u * RN - 1u)) >> 1];
}
template <uint32_t RN>
RPK_INLINE double ring_f64(const RngT<RN>& r, uint32_t a) {  // Standard f64
  const uint2 v = ring_u64(r, a);
  return words_f64(v.x, v.y);
}
template <uint32_t RN>
RPK_INLINE double ring_sym(const RngT<RN>& r, uint32_t a) {  // 2 * Standard f64 - 1
  const uint2 v = ring_u64(r, a);
  return words_sym(v.x, v.y);
}
template <uint32_t RN>
RPK_INLINE void ring_ensure(RngT<RN>& r, uint32_t last_blk) {
  while (last_blk >= *r.end) {
    DREG(DREG_RNG_FALLBACK)
    const uint32_t b = *r.end;
    gen_block(r.slab, b, ring_slot(r, b));
    *r.end = b + 1;
  }
}
// One Standard f64 draw (rand 0.8 gen::<f64>, two stream words)
template <uint32_t RN>
RPK_INLINE double gen_f64(RngT<RN>& r) {
  ring_ensure(r, r.pos >> 4);
  const double x = ring_f64(r, r.pos);
  r.pos += 2;
  return x;
}

// ------------------------------------------------------------------ math -------------------------

struct V3 { double x, y, z; };
RPK_INLINE V3 v3(double x, double y, double z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
RPK_INLINE V3 add(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RPK_INLINE V3 sub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RPK_INLINE V3 mulc(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
RPK_INLINE V3 smul(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
RPK_INLINE double dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }    // nalgebra dot
RPK_INLINE double norm2(V3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }         // norm_squared
RPK_INLINE V3 normalize(V3 a) { double n = sqrt(norm2(a)); return v3(a.x / n, a.y / n, a.z / n); }
RPK_INLINE V3 reflect(V3 i, V3 n) { return sub(i, smul(2.0 * dot(i, n), n)); }         // utility.rs:106

// Rust `as` casts saturate, NaN -> 0
RPK_INLINE uint32_t sat_u32(double x) {
  if (!(x > 0.0)) return 0u;
  if (x >= 4294967295.0) return 4294967295u;
  return (uint32_t)x;
}
RPK_INLINE int64_t sat_i64(double x) {
  if (x != x) return 0;
  if (x >= 9223372036854775807.0) return INT64_MAX;
  if (x <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)x;
}

// randomness.rs:91-105 (wrapping isize, arithmetic >> 13)
RPK_INLINE int64_t noise_integer(int64_t x, int64_t y, int64_t z, int64_t seed) {
  uint64_t h = 0x369E6D3B899E43CFull * (uint64_t)x + 0x53F89E7FFDA3B07Dull * (uint64_t)y +
               0x3B13C1CA4937E629ull * (uint64_t)z + 0x577C2C6E4019D645ull * (uint64_t)seed;
  h = (uint64_t)((int64_t)h >> 13) ^ h;
  h = h * (h * h * 60493ull + 19990303ull) + 1376312589ull;
  return (int64_t)h;
}
RPK_INLINE double noise_real(int64_t x, int64_t y, int64_t z, int64_t seed) {
  return (double)noise_integer(x, y, z, seed) / 9223372036854775807.0;
}

// ------------------------------------------------------------------ traversal --------------------

// The closest hit's primitive kind and material travel with it from the accepting test (bit 31 = triangle,
// bits 0-30 = material; scene_create caps materials below 2^31 - 1): the shading of a triangle hit then
// starts at the material and vertex loads instead of re-reading the primitive record first (one dependent
// L2 round trip less).  KM_UNKNOWN: read them from the record (the q8-node kernel, whose traversal would pay the register).
constexpr uint32_t KM_TRIANGLE = 0x80000000u, KM_UNKNOWN = 0xFFFFFFFFu;
struct HitRec {
  double t, u, v;  // u, v: barycentrics of hittable.rs:89-95 (triangles)
  int32_t prim;    // -1 = miss
  uint32_t km = KM_UNKNOWN;
};

struct TravDiag {
  uint32_t visits = 0, tests = 0, trips = 0;
};

// ---- conservative f32 box test ------------------------------------------------------------------
//
// Conservative f32 slab test.  The ray enters in f32 as o32 = fl(o_ray), inv = rcp(fl(d)) (<= 1 ulp),
// oinv = fl(o32 * inv).  Plane coordinates P are exact: f32 values rounded outward from the exact f64 boxes
// (Node4), or P = o + q s in a node frame (Node4Q: f32 o and s, 8-bit q, exact in f64).
//   Node4:  t^ = fma(P, inv, -oinv)
//   Node4Q: per node and axis A = fl(s inv), B = fma(o, inv, -oinv), and t^ = fma(q, A, B) =
//           (P inv - oinv)(1 + d3) + e,  |e| <= u (1 + u)(|q s inv| + |o inv - oinv|)
// The single-rounding form fma(P, inv, -oinv) errs by <= 5u |t| + |o_ray - o32| |inv| (1 + 6u) + u |o32 inv|
// against the exact t = (P - o_ray) / d (u = 2^-24); with every |o| and |q s| <= qbound (rp_layout.h),
// |e| <= u (1 + u) |inv| (2 qbound + |o32|) + u^2 |o32 inv|, and e = 0 when inv = +-2^64 (the clamp below)
// and o32 = 0 (A and B exact).  Call D_a the absolute terms of axis a.  Each axis's planes are moved
// outward by its own D_a, folded into the FMA's addend: near planes use nb_a = fl_down(-oinv_a - D_a), far
// planes fb_a = fl_up(-oinv_a + D_a) (Node4Q: B_near = fma(o, inv, nb_a), B_far = fma(o, inv, fb_a), whose
// roundings the frame term covers).  A box whose exact interval meets [t_min, best] at some t* > 0 then has
// every near plane <= t*(1 + 6u) (those behind the origin or below tmin32 <= t* do not raise t_near) and
// every far plane >= t*(1 - 6u), so the test
//     fma(tnear^, 1 - 2^-19, -2^-100) <= tfar^
// passes it (2^-19 = 32u).  It may pass a few more boxes, never fewer: no primitive the reference's f64 test
// reaches is culled.  The error bound is per axis: a ray nearly parallel to an axis has a huge D on that
// axis only (|inv| is huge there), which widens that slab alone -- with one scalar slack (max over the
// axes, round 1) such a ray passed every box near the plane it runs in, up to 43 k node visits on C5.
// Empty slots fail (Node4: lo = +inf, hi = -inf gives t_near = +inf; Node4Q: masked by their entry).  Slopes
// are clamped to |inv| <= 2^64 (axis-parallel rays) and frames to |o|, 255 s <= 2^56 (rp_layout.h
// COORD_MAX), so every A, B and t^ is finite; an A that underflows errs by < 2^-118, inside the 2^-100 term.
struct Ray32 {
  float ix, iy, iz;     // rcp(fl(d))
  float nbx, nby, nbz;  // near-plane addends fl_down(-oinv - D) per axis
  float fbx, fby, fbz;  // far-plane addends fl_up(-oinv + D) per axis
  float tmin;           // t_min rounded down
  uint32_t sx, sy, sz;  // per axis, by the sign of the slope: Node4 = byte offset of the near plane row
                        // (lo_* or hi_*; the far row is the other); Node4Q/Node8Q = v_perm_b32 selector picking
                        // the near plane codes out of the {hi, lo} word pair (the far codes out of {lo, hi})
  uint32_t oct;         // Node8Q: dir_octant(d), the children's rank order slot ^ oct
};

// Octant of a direction: bit a set when d_a has its sign bit set (the sign of rcp(fl(d_a)) below).  Node8Q
// visits a node's children in rank order slot ^ octant (rp_layout.h); only the order depends on it.
RPK_INLINE uint32_t dir_octant(V3 d) {
  return (uint32_t)(__double_as_longlong(d.x) < 0) | (uint32_t)(__double_as_longlong(d.y) < 0) << 1 |
         (uint32_t)(__double_as_longlong(d.z) < 0) << 2;
}

// next representable float towards +inf / -inf (finite inputs; the callers only step values that
// rounded the wrong way, which are finite)
RPK_INLINE float next_up(float f) {
  const int32_t b = __float_as_int(f);
  if (f == 0.0f) return __int_as_float(1);
  return __int_as_float(f > 0.0f ? b + 1 : b - 1);
}
RPK_INLINE float next_down(float f) { return -next_up(-f); }
RPK_INLINE float f32_down(double x) {
  const float f = (float)x;
  return (double)f > x ? next_down(f) : f;
}
RPK_INLINE float f32_up(double x) {
  const float f = (float)x;
  return (double)f < x ? next_up(f) : f;
}

template <uint32_t NF>
RPK_INLINE void setup_ray32(V3 o, V3 d, double tmin, double qbound, Ray32& r) {
  const float ox = (float)o.x, oy = (float)o.y, oz = (float)o.z;
  // |inv| clamped to 2^64: a zero direction component gives a huge finite slope instead of inf, so the
  // fma form never forms inf - inf; the slack term |o - o32| |inv| still covers an origin that rounded
  // across a slab plane, and a slab the ray never reaches still yields a huge t (a miss), as in f64.
  r.ix = fminf(fmaxf(__builtin_amdgcn_rcpf((float)d.x), -0x1p64f), 0x1p64f);
  r.iy = fminf(fmaxf(__builtin_amdgcn_rcpf((float)d.y), -0x1p64f), 0x1p64f);
  r.iz = fminf(fmaxf(__builtin_amdgcn_rcpf((float)d.z), -0x1p64f), 0x1p64f);
  const float oix = ox * r.ix, oiy = oy * r.iy, oiz = oz * r.iz;
  // |o - o32| is exact in f64 (Sterbenz); an axis with no origin rounding contributes no origin term
  const double ex = fabs(o.x - (double)ox), ey = fabs(o.y - (double)oy), ez = fabs(o.z - (double)oz);
  const double k = 1.0 + 0x1p-20, u = 0x1p-23, q2 = 2.0 * qbound;
  const auto fr = [&](float inv, float o32) {  // the Node4Q frame term e (see above)
    return (NF == rpl::NODES_F32 || (fabsf(inv) == 0x1p64f && o32 == 0.0f))
               ? 0.0
               : fabs((double)inv) * (q2 + fabs((double)o32)) * u * k;
  };
  const double Dx = ((ex == 0.0 ? 0.0 : ex * fabs((double)r.ix) * k) + fabs((double)oix) * u + fr(r.ix, ox)) * k;
  const double Dy = ((ey == 0.0 ? 0.0 : ey * fabs((double)r.iy) * k) + fabs((double)oiy) * u + fr(r.iy, oy)) * k;
  const double Dz = ((ez == 0.0 ? 0.0 : ez * fabs((double)r.iz) * k) + fabs((double)oiz) * u + fr(r.iz, oz)) * k;
  r.nbx = f32_down(-(double)oix - Dx);
  r.nby = f32_down(-(double)oiy - Dy);
  r.nbz = f32_down(-(double)oiz - Dz);
  r.fbx = f32_up(-(double)oix + Dx);
  r.fby = f32_up(-(double)oiy + Dy);
  r.fbz = f32_up(-(double)oiz + Dz);
  r.tmin = f32_down(tmin);
  r.oct = dir_octant(d);
  if (NF != rpl::NODES_F32) {
    r.sx = r.ix < 0.0f ? 0x07060504u : 0x03020100u;
    r.sy = r.iy < 0.0f ? 0x07060504u : 0x03020100u;
    r.sz = r.iz < 0.0f ? 0x07060504u : 0x03020100u;
  } else {
    // Node4: lo_x at 0, hi_x at 16, lo_y at 32, hi_y at 48, lo_z at 64, hi_z at 80
    r.sx = r.ix < 0.0f ? 16u : 0u;
    r.sy = r.iy < 0.0f ? 48u : 32u;
    r.sz = r.iz < 0.0f ? 80u : 64u;
  }
}

// Closest hit over the 4-wide BVH (the reference's Hittable::Bvh::hit, bvh.rs:121-124 / hit_node
// bvh.rs:93-119: any tree shape and visit order returns the same closest hit up to exact-t ties,
// SURVEY.md 8a A9).  Primitive tests are the reference's exact f64 ones; t_max shrinks to the closest
// hit so far and acceptance is `t <= t_max`, so an equal-t primitive tested later wins
// (hittable.rs:52,99).  Structure: "while-while" -- descend inner nodes (near child first, the others
// pushed far-to-near on the LDS stack) until this lane holds a leaf, then test the leaf's primitives;
// the wave runs the expensive f64 leaf code once for every lane that reached a leaf.
//
// The traversal state is explicit (TravState) so a lane can stop between steps and resume later: the
// render kernel steps traversal until few lanes are still traversing, shades the finished ones and
// gives them new rays, then resumes (see render_kernel).
//
// Node8Q trees (trav_step_w8) keep groups instead of entries: cur/gy = a node group {W8_GROUP | family index,
// rank bits 0-7 | imask << 8} (the children still to visit, in rank order) or a primitive group {first primitive,
// primitive bits}; leaf/py = the parked primitive group (py = 0: none, and then leaf = 0).
struct TravState {
  double best, bu, bv;
  int32_t bestp;
  uint32_t bestm;  // the closest hit's kind and material (HitRec::km)
  uint32_t cur, sp;
  uint32_t leaf;  // parked leaf entry (speculative traversal), 0 = none (entry 0 is an inner node)
  uint32_t gy, py;  // Node8Q only (0 otherwise)
};
static constexpr uint32_t W8_GROUP = 0x80000000u;  // cur: a node group (prim groups: first primitive < 2^31)

RPK_INLINE bool trav_done(const TravState& t) { return t.cur == rpl::ENTRY_EMPTY && (t.leaf | t.py) == 0u; }

// A new ray from the root; `d` orders a Node8Q root's children.
template <uint32_t NF>
RPK_INLINE void trav_init(const KScene& S, double tmax, TravState& t, V3 d) {
  t.best = tmax;
  t.bu = 0.0;
  t.bv = 0.0;
  t.bestp = -1;
  t.bestm = KM_UNKNOWN;
  t.cur = S.root;
  t.sp = 0;
  t.leaf = 0;
  t.gy = 0;
  t.py = 0;
  if constexpr (NF == rpl::NODES_W8) {
    t.cur = W8_GROUP | S.root;              // the root as a group of one: slot 0, rank 0 ^ oct
    t.gy = (1u << dir_octant(d)) | 0x100u;  // imask = slot 0
  }
}

// One exact f64 primitive test (the reference's Hittable::hit for a leaf, hittable.rs:39-101): on
// acceptance `best` shrinks to t and the hit record is taken.
RPK_INLINE void prim_test(const KScene& S, uint32_t k, V3 o, V3 d, double tmin, double& best, TravState& ts) {
  // 32-bit byte offset from the wave-uniform base (scalar-base + vector-offset loads)
  const double2* q = reinterpret_cast<const double2*>(reinterpret_cast<const char*>(S.prims) +
                                                      k * (uint32_t)sizeof(rpl::Prim));
  const double2 g01 = q[0], g23 = q[1], g45 = q[2], g67 = q[3];
  const double2 g8k = q[4];  // g[8], {kind, material}
  const uint64_t km = (uint64_t)__double_as_longlong(g8k.y);
  const uint32_t kind = (uint32_t)km, mat = (uint32_t)(km >> 32);
  if (kind == rpl::PRIM_TRIANGLE) {
    // hittable.rs:65-101, exact expression order; ba, ca were pre-subtracted (same IEEE op)
    const V3 a = v3(g01.x, g01.y, g23.x);
    const V3 ba = v3(g23.y, g45.x, g45.y);
    const V3 ca = v3(g67.x, g67.y, g8k.x);
    const V3 pa = sub(a, o);
    const double det = ba.x * ca.y * d.z + ba.y * ca.z * d.x + ba.z * ca.x * d.y
                     - ba.x * ca.z * d.y - ba.y * ca.x * d.z - ba.z * ca.y * d.x;
    if (fabs(det) < SMOL) return;
    const double inv_det = 1.0 / det;
    const double t = (pa.x * (ba.y * ca.z - ba.z * ca.y)
                    + pa.y * (ba.z * ca.x - ba.x * ca.z)
                    + pa.z * (ba.x * ca.y - ba.y * ca.x)) * inv_det;
    const double u = (pa.x * (ca.y * d.z - ca.z * d.y)
                    + pa.y * (ca.z * d.x - ca.x * d.z)
                    + pa.z * (ca.x * d.y - ca.y * d.x)) * inv_det;
    const double v = (pa.x * (ba.z * d.y - ba.y * d.z)
                    + pa.y * (ba.x * d.z - ba.z * d.x)
                    + pa.z * (ba.y * d.x - ba.x * d.y)) * inv_det;
    const double w = 1.0 - u - v;
    if (t < tmin || t > best || u < 0.0 || v < 0.0 || w < 0.0) return;
    best = t; ts.bestp = (int32_t)k; ts.bu = u; ts.bv = v; ts.bestm = KM_TRIANGLE | mat;
  } else {
    // hittable.rs:39-57
    const V3 c = v3(g01.x, g01.y, g23.x);
    const double radius = g23.y;
    const V3 tc = sub(o, c);
    const double a = norm2(d);
    const double half_b = dot(d, tc);
    const double cq = norm2(tc) - radius * radius;
    const double delta = half_b * half_b - a * cq;
    if (delta <= 0.0) return;
    const double sq = sqrt(delta);
    double t = (-half_b - sq) / a;
    if (t < tmin || t > best) {
      t = (-half_b + sq) / a;
      if (t < tmin || t > best) return;
    }
    best = t; ts.bestp = (int32_t)k; ts.bestm = mat;
  }
}

// A new ray: the always-tested primitives (KScene::n_always: boxes that dwarf the rest of the scene, kept
// out of the tree by the host builder) get their exact tests here, one wave-uniform loop over the same
// primitive for every starting lane, instead of a divergent leaf test deep in the prim loop; their hit
// also bounds the traversal from the root.  The closest hit is the tree's (any test order, up to exact-t
// ties).
template <uint32_t NF>
RPK_INLINE void trav_begin(const KScene& S, V3 o, V3 d, double tmin, double tmax, TravState& t) {
  trav_init<NF>(S, tmax, t, d);
  double best = t.best;
  for (uint32_t k = S.always_first; k < S.always_first + S.n_always; k++) prim_test(S, k, o, d, tmin, best, t);
  t.best = best;
}

// Stack entry i of a lane: in its LDS column (entry i at stk[i * stride]) or, for SPILL kernels, entries
// >= S.lds_depth in the lane's global overflow run (S.spill[spl + i - lds_depth], L2-resident) -- a deep
// tree (config C5: 43 entries) then keeps the LDS of four blocks per CU.  The two parts are typed with
// their address spaces (LDS = 3, global = 1): with generic pointers the compiler merged the LDS and the
// spill store of a push into one FLAT store through a selected pointer (and the pops into FLAT loads),
// which waits on both memory counters at every node visit.
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(1))) uint32_t glb_u32;
RPK_INLINE glb_u32* spill_ptr(const KScene& S) { return (glb_u32*)S.spill; }
template <bool SPILL>
RPK_INLINE void stk_put(const KScene& S, lds_u32* stk, uint32_t stride, uint32_t spl, uint32_t i, uint32_t v) {
  if (!SPILL || i < S.lds_depth) stk[i * stride] = v;
  else spill_ptr(S)[spl + i - S.lds_depth] = v;
}
template <bool SPILL>
RPK_INLINE uint32_t stk_get(const KScene& S, const lds_u32* stk, uint32_t stride, uint32_t spl, uint32_t i) {
  if (!SPILL || i < S.lds_depth) return stk[i * stride];
  return spill_ptr(S)[spl + i - S.lds_depth];
}

// One step: descend until a leaf is held, test the leaves.  Finished when t.cur == ENTRY_EMPTY and no leaf is
// parked (trav_done).  `spl`: the lane's first spill entry (SPILL kernels).  `work` (COUNT instantiations: the
// cost probe) accumulates the lane's traversal work in WORK_* units.
enum : uint32_t { WORK_VISIT = 2, WORK_TEST = 3, WORK_RAY = 16 };  // node visit : primitive test : shaded ray

// Node8Q step.  The lane descends while it holds a node group with children left: it takes the lowest rank
// (the nearest octant), pushes the rest of the group, and visits that child, whose hit inner children become
// the new node group and whose hit leaf children's primitives one primitive group -- parked if the lane has
// none parked (speculative traversal, as in the 4-wide step), else pushed.  Groups go on the stack as two
// words.  `w8_settle` pops until the lane holds a node group with work, a primitive group it cannot park yet
// (it waits for the leaf loop), or nothing.  The leaf loop tests one primitive per lane per iteration from the
// parked group (lowest bit first), then takes a waiting primitive group.  Same exits as trav_step.
template <bool SPILL>
RPK_INLINE void w8_settle(const KScene& S, lds_u32* stk, uint32_t stride, uint32_t spl, uint32_t& gx, uint32_t& gy,
                          uint32_t& px, uint32_t& py, uint32_t& sp) {
#pragma unroll
  for (int it = 0; it < 2; it++) {  // at most a primitive group and then anything: two pops
    if (gx & W8_GROUP) {
      if (gy & 0xFFu) return;
    } else {
      if (py) return;
      px = gx; py = gy;
    }
    if (sp == 0u) { gx = rpl::ENTRY_EMPTY; gy = 0u; return; }
    sp -= 2u;
    gx = stk_get<SPILL>(S, stk, stride, spl, sp);
    gy = stk_get<SPILL>(S, stk, stride, spl, sp + 1u);
  }
}

template <bool SPILL, bool COUNT>
RPK_INLINE void trav_step_w8(const KScene& S, lds_u32* stk, uint32_t stride, uint32_t spl, const Ray32& r, V3 o,
                             V3 d, double tmin, TravState& ts, bool& overflow, TravDiag* td, uint32_t* work) {
  uint32_t gx = ts.cur, gy = ts.gy, px = ts.leaf, py = ts.py, sp = ts.sp;
  double best = ts.best;
  float best32 = f32_up(best);
  const uint32_t cap = S.stack_depth - STACK_SLACK;  // words
  auto push = [&](uint32_t x, uint32_t y) {
    if (sp + 2u > cap) { overflow = true; return; }  // cannot happen for a stack sized from the tree depth
    stk_put<SPILL>(S, stk, stride, spl, sp, x);
    stk_put<SPILL>(S, stk, stride, spl, sp + 1u, y);
    sp += 2u;
  };
  w8_settle<SPILL>(S, stk, stride, spl, gx, gy, px, py, sp);
  // ---- inner nodes
  while ((gx & W8_GROUP) && (gy & 0xFFu) && (!COUNT || py == 0u)) {
    DIAG(if (td) td->visits++;)
    if constexpr (COUNT) *work += WORK_VISIT;
    DREG(DREG_NODE)
    const uint32_t slot = (uint32_t)__builtin_ctz(gy) ^ r.oct;
    gy &= gy - 1u;
    const uint32_t node = (gx & ~W8_GROUP) + (uint32_t)__builtin_popcount((gy >> 8) & ((1u << slot) - 1u));
    if (gy & 0xFFu) push(gx, gy);
    const char* nb = reinterpret_cast<const char*>(S.nodes);
    const uint32_t no = node << 7;
    const float4 c0 = *reinterpret_cast<const float4*>(nb + no);        // o.x o.y o.z s.x
    const uint4 c1 = *reinterpret_cast<const uint4*>(nb + (no + 16u));  // s.y s.z inner prim
    const uint4 cx = *reinterpret_cast<const uint4*>(nb + (no + 32u));  // lo_x[0-3] lo_x[4-7] hi_x[0-3] hi_x[4-7]
    const uint4 cy = *reinterpret_cast<const uint4*>(nb + (no + 48u));
    const uint4 cz = *reinterpret_cast<const uint4*>(nb + (no + 64u));
    const uint4 pa = *reinterpret_cast<const uint4*>(nb + (no + 80u));  // pmask[0-3]
    const uint4 pb = *reinterpret_cast<const uint4*>(nb + (no + 96u));  // pmask[4-7]
    const float Ax = c0.w * r.ix, Ay = __uint_as_float(c1.x) * r.iy, Az = __uint_as_float(c1.y) * r.iz;
    const float Bnx = fmaf(c0.x, r.ix, r.nbx), Bny = fmaf(c0.y, r.iy, r.nby), Bnz = fmaf(c0.z, r.iz, r.nbz);
    const float Bfx = fmaf(c0.x, r.ix, r.fbx), Bfy = fmaf(c0.y, r.iy, r.fby), Bfz = fmaf(c0.z, r.iz, r.fbz);
    const f2 ax = {Ax, Ax}, ay = {Ay, Ay}, az = {Az, Az};
    const f2 bnx = {Bnx, Bnx}, bny = {Bny, Bny}, bnz = {Bnz, Bnz}, bfx = {Bfx, Bfx}, bfy = {Bfy, Bfy}, bfz = {Bfz, Bfz};
    uint32_t hits = 0u, pm = 0u;
#define RPK_Q2(w, h) f2{(float)(((w) >> (16 * (h))) & 0xffu), (float)(((w) >> (16 * (h) + 8)) & 0xffu)}
#pragma unroll
    for (int half = 0; half < 2; half++) {  // children 4 half .. 4 half + 3
      const uint32_t lx = half ? cx.y : cx.x, hx = half ? cx.w : cx.z;
      const uint32_t ly = half ? cy.y : cy.x, hy = half ? cy.w : cy.z;
      const uint32_t lz = half ? cz.y : cz.x, hz = half ? cz.w : cz.z;
      const uint32_t qnx = __builtin_amdgcn_perm(hx, lx, r.sx), qfx = __builtin_amdgcn_perm(lx, hx, r.sx);
      const uint32_t qny = __builtin_amdgcn_perm(hy, ly, r.sy), qfy = __builtin_amdgcn_perm(ly, hy, r.sy);
      const uint32_t qnz = __builtin_amdgcn_perm(hz, lz, r.sz), qfz = __builtin_amdgcn_perm(lz, hz, r.sz);
      const uint4 pq = half ? pb : pa;
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const f2 NX = pk_fma(RPK_Q2(qnx, q), ax, bnx), FX = pk_fma(RPK_Q2(qfx, q), ax, bfx);
        const f2 NY = pk_fma(RPK_Q2(qny, q), ay, bny), FY = pk_fma(RPK_Q2(qfy, q), ay, bfy);
        const f2 NZ = pk_fma(RPK_Q2(qnz, q), az, bnz), FZ = pk_fma(RPK_Q2(qfz, q), az, bfz);
        f2 TN, TF;
#pragma unroll
        for (int e = 0; e < 2; e++) {
          TN[e] = fmaxf(fmaxf(NX[e], NY[e]), fmaxf(NZ[e], r.tmin));
          TF[e] = fminf(fminf(FX[e], FY[e]), fminf(FZ[e], best32));
        }
        const f2 lhs = pk_fma(TN, f2{1.0f - 0x1p-19f, 1.0f - 0x1p-19f}, f2{-0x1p-100f, -0x1p-100f});
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int c = 4 * half + 2 * q + e;
          const bool hit = lhs[e] <= TF[e];
          hits |= hit ? 1u << c : 0u;
          const uint32_t m = (2 * q + e) == 0 ? pq.x : (2 * q + e) == 1 ? pq.y : (2 * q + e) == 2 ? pq.z : pq.w;
          pm |= hit ? m : 0u;
        }
      }
    }
#undef RPK_Q2
    // hit inner children in rank order: bit (slot ^ oct)
    const uint32_t imask = c1.z >> 24;
    uint32_t ih = hits & imask;
    if (r.oct & 1u) ih = ((ih & 0x55u) << 1) | ((ih >> 1) & 0x55u);
    if (r.oct & 2u) ih = ((ih & 0x33u) << 2) | ((ih >> 2) & 0x33u);
    if (r.oct & 4u) ih = ((ih & 0x0Fu) << 4) | ((ih >> 4) & 0x0Fu);
    if (pm) {
      if (py == 0u) { px = c1.w; py = pm; }
      else push(c1.w, pm);
    }
    gx = W8_GROUP | (c1.z & rpl::W8_INDEX);
    gy = ih | imask << 8;
    w8_settle<SPILL>(S, stk, stride, spl, gx, gy, px, py, sp);
    if (!COUNT && (uint32_t)__popcll(__ballot(py == 0u)) <= S.leaf_break) break;
  }
  // ---- leaves: one primitive per lane per iteration from the parked group, then a waiting one
  while (py != 0u) {
    DIAG(if (td) td->tests++;)
    if constexpr (COUNT) *work += WORK_TEST;
    DREG(DREG_PRIM)
    const uint32_t k = px + (uint32_t)__builtin_ctz(py);
    py &= py - 1u;
    prim_test(S, k, o, d, tmin, best, ts);
    if (py == 0u) {
      px = 0u;
      if (!(gx & W8_GROUP)) w8_settle<SPILL>(S, stk, stride, spl, gx, gy, px, py, sp);  // park the waiting group
    }
    if (!COUNT && PRIM_BREAK > 0 && (uint32_t)__popcll(__ballot(py != 0u)) <= PRIM_BREAK) break;
  }
  ts.cur = gx;
  ts.gy = gy;
  ts.sp = sp;
  ts.best = best;
  ts.leaf = px;
  ts.py = py;
}

template <bool SPILL, uint32_t NF, bool COUNT = false>
RPK_INLINE void trav_step(const KScene& S, lds_u32* stk, uint32_t stride, uint32_t spl, const Ray32& r, V3 o, V3 d,
                          double tmin, TravState& ts, bool& overflow, TravDiag* td = nullptr,
                          uint32_t* work = nullptr) {
  if constexpr (NF == rpl::NODES_W8) {
    trav_step_w8<SPILL, COUNT>(S, stk, stride, spl, r, o, d, tmin, ts, overflow, td, work);
    return;
  }
  uint32_t cur = ts.cur, sp = ts.sp, leaf = ts.leaf;
  double best = ts.best;
  float best32 = f32_up(best);
  const uint32_t cap = S.stack_depth - STACK_SLACK;
  DCYC_BEGIN(cnode)
  // ---- inner nodes
  while (!(cur & rpl::ENTRY_LEAF)) {
    DIAG(if (td) td->visits++;)
    if constexpr (COUNT) *work += WORK_VISIT;
    DREG(DREG_NODE)
    // Near/far planes chosen per ray by the slope signs (octant), so each child costs one max3 + max for
    // t_near and one min3 + min for t_far: for a valid box the same pair of values the min/max slab form
    // picks (t^ is monotone in the plane coordinate).  Node4 picks the near/far rows by address; Node4Q
    // picks the four children's near (far) plane codes out of the {lo, hi} code words with one v_perm_b32
    // per axis and side.  32-bit byte offsets from the (wave-uniform) node base: scalar-base +
    // vector-offset addressing.
    const char* nb = reinterpret_cast<const char*>(S.nodes);
    f2 NX[2], FX[2], NY[2], FY[2], NZ[2], FZ[2];
    uint4 ch;
    if constexpr (NF == rpl::NODES_Q8) {
      const uint32_t no = cur << 6;
      const float4 c0 = *reinterpret_cast<const float4*>(nb + no);        // o.x o.y o.z s.x
      const uint4 c1 = *reinterpret_cast<const uint4*>(nb + (no + 16u));  // s.y s.z lo_x hi_x
      const uint4 c2 = *reinterpret_cast<const uint4*>(nb + (no + 32u));  // lo_y hi_y lo_z hi_z
      ch = *reinterpret_cast<const uint4*>(nb + (no + 48u));
      // per axis: A = s inv, B = fma(o, inv, -oinv); plane t^ = fma(q, A, B)
      const float Ax = c0.w * r.ix, Ay = __uint_as_float(c1.x) * r.iy, Az = __uint_as_float(c1.y) * r.iz;
      const float Bnx = fmaf(c0.x, r.ix, r.nbx), Bny = fmaf(c0.y, r.iy, r.nby), Bnz = fmaf(c0.z, r.iz, r.nbz);
      const float Bfx = fmaf(c0.x, r.ix, r.fbx), Bfy = fmaf(c0.y, r.iy, r.fby), Bfz = fmaf(c0.z, r.iz, r.fbz);
      const uint32_t qnx = __builtin_amdgcn_perm(c1.w, c1.z, r.sx), qfx = __builtin_amdgcn_perm(c1.z, c1.w, r.sx);
      const uint32_t qny = __builtin_amdgcn_perm(c2.y, c2.x, r.sy), qfy = __builtin_amdgcn_perm(c2.x, c2.y, r.sy);
      const uint32_t qnz = __builtin_amdgcn_perm(c2.w, c2.z, r.sz), qfz = __builtin_amdgcn_perm(c2.z, c2.w, r.sz);
      // children (0,1) and (2,3) as packed pairs: v_pk_fma_f32 is two fused FMAs with the same per-element
      // rounding as fmaf; byte b of a code word converts with v_cvt_f32_ubyte<b>
      const f2 ax = {Ax, Ax}, ay = {Ay, Ay}, az = {Az, Az};
      const f2 bnx = {Bnx, Bnx}, bny = {Bny, Bny}, bnz = {Bnz, Bnz}, bfx = {Bfx, Bfx}, bfy = {Bfy, Bfy}, bfz = {Bfz, Bfz};
#define RPK_Q2(w, h) f2{(float)(((w) >> (16 * (h))) & 0xffu), (float)(((w) >> (16 * (h) + 8)) & 0xffu)}
#pragma unroll
      for (int q = 0; q < 2; q++) {
        NX[q] = pk_fma(RPK_Q2(qnx, q), ax, bnx);
        FX[q] = pk_fma(RPK_Q2(qfx, q), ax, bfx);
        NY[q] = pk_fma(RPK_Q2(qny, q), ay, bny);
        FY[q] = pk_fma(RPK_Q2(qfy, q), ay, bfy);
        NZ[q] = pk_fma(RPK_Q2(qnz, q), az, bnz);
        FZ[q] = pk_fma(RPK_Q2(qfz, q), az, bfz);
      }
#undef RPK_Q2
    } else {
      const uint32_t no = cur << 7;
      const float4 nx = *reinterpret_cast<const float4*>(nb + (no + r.sx));
      const float4 fx = *reinterpret_cast<const float4*>(nb + (no + (r.sx ^ 16u)));
      const float4 ny = *reinterpret_cast<const float4*>(nb + (no + r.sy));
      const float4 fy = *reinterpret_cast<const float4*>(nb + (no + (r.sy ^ 16u)));
      const float4 nz = *reinterpret_cast<const float4*>(nb + (no + r.sz));
      const float4 fz = *reinterpret_cast<const float4*>(nb + (no + (r.sz ^ 16u)));
      ch = *reinterpret_cast<const uint4*>(nb + (no + 96u));
      const f2 ix = {r.ix, r.ix}, iy = {r.iy, r.iy}, iz = {r.iz, r.iz};
      const f2 nbx = {r.nbx, r.nbx}, nby = {r.nby, r.nby}, nbz = {r.nbz, r.nbz};
      const f2 fbx = {r.fbx, r.fbx}, fby = {r.fby, r.fby}, fbz = {r.fbz, r.fbz};
      NX[0] = pk_fma(f2{nx.x, nx.y}, ix, nbx); NX[1] = pk_fma(f2{nx.z, nx.w}, ix, nbx);
      FX[0] = pk_fma(f2{fx.x, fx.y}, ix, fbx); FX[1] = pk_fma(f2{fx.z, fx.w}, ix, fbx);
      NY[0] = pk_fma(f2{ny.x, ny.y}, iy, nby); NY[1] = pk_fma(f2{ny.z, ny.w}, iy, nby);
      FY[0] = pk_fma(f2{fy.x, fy.y}, iy, fby); FY[1] = pk_fma(f2{fy.z, fy.w}, iy, fby);
      NZ[0] = pk_fma(f2{nz.x, nz.y}, iz, nbz); NZ[1] = pk_fma(f2{nz.z, nz.w}, iz, nbz);
      FZ[0] = pk_fma(f2{fz.x, fz.y}, iz, fbz); FZ[1] = pk_fma(f2{fz.z, fz.w}, iz, fbz);
    }
    float tn[4];
    uint32_t cc[4] = {ch.x, ch.y, ch.z, ch.w};
    f2 TN[2], TF[2];
#pragma unroll
    for (int q = 0; q < 2; q++) {
#pragma unroll
      for (int e = 0; e < 2; e++) {
        TN[q][e] = fmaxf(fmaxf(NX[q][e], NY[q][e]), fmaxf(NZ[q][e], r.tmin));
        TF[q][e] = fminf(fminf(FX[q][e], FY[q][e]), fminf(FZ[q][e], best32));
      }
      // fma(tnear, 1 - 2^-19, -2^-100) <= tfar (section 4.2 of DESIGN.md): one packed FMA per pair
      const f2 lhs = pk_fma(TN[q], f2{1.0f - 0x1p-19f, 1.0f - 0x1p-19f}, f2{-0x1p-100f, -0x1p-100f});
#pragma unroll
      for (int e = 0; e < 2; e++) {
        const int c = 2 * q + e;
        const bool hit = lhs[e] <= TF[q][e] && (NF != rpl::NODES_Q8 || cc[c] != rpl::ENTRY_EMPTY);
        tn[c] = hit ? TN[q][e] : __builtin_huge_valf();
      }
    }
    // sort (tn, entry) ascending: misses (+inf) go last
#define RPK_CSWAP(a, b)                                   \
{                                                       \
  const bool sw = tn[b] < tn[a];                        \
  const float t_ = sw ? tn[b] : tn[a];                  \
  tn[b] = sw ? tn[a] : tn[b];                           \
  tn[a] = t_;                                           \
  const uint32_t c_ = sw ? cc[b] : cc[a];               \
  cc[b] = sw ? cc[a] : cc[b];                           \
  cc[a] = c_;                                           \
}
    RPK_CSWAP(0, 1) RPK_CSWAP(2, 3) RPK_CSWAP(0, 2) RPK_CSWAP(1, 3) RPK_CSWAP(1, 2)
#undef RPK_CSWAP
    // The hits are a prefix of the sorted entries (misses sort last as +inf).  Push the k = hits - 1
    // farther ones far-to-near without branches: slots sp..sp+2 are written unconditionally (the stack
    // has STACK_SLACK spare entries; slots past the new top are garbage) and sp advances by k.
    const float INFF = __builtin_huge_valf();
    const uint32_t n_hit = (uint32_t)(tn[0] != INFF) + (uint32_t)(tn[1] != INFF) + (uint32_t)(tn[2] != INFF) +
                           (uint32_t)(tn[3] != INFF);
    const uint32_t k = n_hit > 1u ? n_hit - 1u : 0u;
    const uint32_t e0 = k == 3u ? cc[3] : (k == 2u ? cc[2] : cc[1]), e1 = k == 3u ? cc[2] : cc[1];
    // Whether every lane's pushes and pops of this visit stay in the LDS part of its stack: a wave-uniform branch
    // (SPILL kernels), so the common case runs no per-lane exec-mask juggling for the spill path.
    const bool lds_only = !SPILL || __ballot(sp + 2u >= S.lds_depth) == 0;
    if (lds_only) {
      stk[sp * stride] = e0;
      stk[(sp + 1u) * stride] = e1;
      stk[(sp + 2u) * stride] = cc[1];
    } else {
      stk_put<SPILL>(S, stk, stride, spl, sp, e0);
      stk_put<SPILL>(S, stk, stride, spl, sp + 1u, e1);
      stk_put<SPILL>(S, stk, stride, spl, sp + 2u, cc[1]);
    }
    sp += k;
    if (sp > cap) {  // cannot happen for a stack sized from the tree depth; flagged, never written past
      overflow = true;
      sp = cap;
    }
    // pops below read entries < the pushes' top (sp + 2 before the push), so an LDS-only visit pops from LDS
    const auto pop = [&]() -> uint32_t {
      --sp;
      return lds_only ? stk[sp * stride] : stk_get<SPILL>(S, stk, stride, spl, sp);
    };
    // Speculative traversal (Aila & Laine 2009): a lane that reaches a leaf parks it and keeps
    // descending, so lanes do not idle in this loop until every lane of the wave holds a leaf.  (Not in the
    // cost probe, COUNT: there a lane's node visits and primitive tests must not depend on its wave-mates, so
    // every rank of a balanced multi-GPU frame computes the same costs -- include/rp.h RP_SHARD_BALANCED.)
    if (lds_only) {
      // the next entry without a branch: the two entries under the top are read at once (indices clamped into the
      // column; an entry below the stack's bottom is read but never taken), then the pop for a visit that hit no
      // child and the pop behind a parked leaf are selects
      const uint32_t t1 = stk[min(sp - 1u, sp) * stride], t2 = stk[min(sp - 2u, sp) * stride];
      uint32_t npop = (!n_hit && sp) ? 1u : 0u;
      uint32_t c = n_hit ? cc[0] : (sp ? t1 : rpl::ENTRY_EMPTY);
      if constexpr (!COUNT) {
        const bool park = (c & rpl::ENTRY_LEAF) && c != rpl::ENTRY_EMPTY && leaf == 0u;
        const uint32_t left = sp - npop;
        leaf = park ? c : leaf;
        const uint32_t c2 = left ? (npop ? t2 : t1) : rpl::ENTRY_EMPTY;
        npop += (park && left) ? 1u : 0u;
        c = park ? c2 : c;
      }
      cur = c;
      sp -= npop;
    } else {
      if (n_hit) cur = cc[0];
      else cur = sp ? pop() : rpl::ENTRY_EMPTY;
      if constexpr (!COUNT) {
        if ((cur & rpl::ENTRY_LEAF) && cur != rpl::ENTRY_EMPTY && leaf == 0u) {
          leaf = cur;
          cur = sp ? pop() : rpl::ENTRY_EMPTY;
        }
      }
    }
    if constexpr (!COUNT) {
      // ... and once at most S.leaf_break lanes still look for one, the wave moves on to the leaves: the
      // last few descents ran with most of the wave idle (those lanes resume their descent next step)
      if ((uint32_t)__popcll(__ballot(leaf == 0u)) <= S.leaf_break) break;
    }
  }
  DCYC_END(DCYC_NODE_LOOP, cnode)
  DCYC_BEGIN(cprim)
  // the pops from here on only shrink sp: when no lane's stack reaches into its spill run, they all read LDS (a
  // wave-uniform branch, as in the node loop)
  const bool lds_pop = !SPILL || __ballot(sp > S.lds_depth) == 0;
  const auto pop = [&]() -> uint32_t {
    --sp;
    return lds_pop ? stk[sp * stride] : stk_get<SPILL>(S, stk, stride, spl, sp);
  };
  if (leaf == 0u && cur != rpl::ENTRY_EMPTY && (cur & rpl::ENTRY_LEAF)) {
    leaf = cur;
    cur = sp ? pop() : rpl::ENTRY_EMPTY;
  }
  // ---- leaves: the reference's exact f64 primitive tests, the parked leaf first, then the current
  // entry while it is a leaf as well.  One primitive per lane per iteration across those leaves, so
  // lanes with different leaf sizes advance together instead of the wave running every leaf's count.
  uint32_t k = leaf & rpl::LEAF_FIRST_MASK;
  uint32_t kend = k + ((leaf >> rpl::LEAF_SHIFT) & 7u) + 1u;
  while (leaf != 0u) {
    DIAG(if (td) td->tests++;)
    if constexpr (COUNT) *work += WORK_TEST;
    DREG(DREG_PRIM)
    prim_test(S, k, o, d, tmin, best, ts);
    if (++k == kend) {
      if (cur != rpl::ENTRY_EMPTY && (cur & rpl::ENTRY_LEAF)) {
        leaf = cur;
        cur = sp ? pop() : rpl::ENTRY_EMPTY;
        k = leaf & rpl::LEAF_FIRST_MASK;
        kend = k + ((leaf >> rpl::LEAF_SHIFT) & 7u) + 1u;
      } else {
        leaf = 0u;
      }
    }
    if (!COUNT && PRIM_BREAK > 0 && (uint32_t)__popcll(__ballot(leaf != 0u)) <= PRIM_BREAK) {
      // park the rest of the current run [k, kend) as a leaf entry; the next step tests it first
      if (leaf != 0u) leaf = rpl::ENTRY_LEAF | ((kend - k - 1u) << rpl::LEAF_SHIFT) | k;
      break;
    }
  }
  DCYC_END(DCYC_PRIM_LOOP, cprim)
  ts.cur = cur;
  ts.sp = sp;
  ts.best = best;
  ts.leaf = leaf;
}

template <uint32_t NF>
RPK_INLINE void traverse(const KScene& S, lds_u32* stk, uint32_t stride, V3 o, V3 d, double tmin, double tmax,
                         HitRec& hr, bool& overflow, TravDiag* td = nullptr) {
  Ray32 r;
  setup_ray32<NF>(o, d, tmin, S.qbound, r);
  TravState t;
  trav_begin<NF>(S, o, d, tmin, tmax, t);
  while (!trav_done(t)) trav_step<false, NF>(S, stk, stride, 0u, r, o, d, tmin, t, overflow, td);
  hr.t = t.best;
  hr.u = t.bu;
  hr.v = t.bv;
  hr.prim = t.bestp;
  hr.km = t.bestm;
}

// Hit record of the closest primitive (hittable.rs:59-62, 103-107).
struct Surf {
  V3 p, n;
  double u, v;
  uint32_t material;
};

// uv is computed only when the hit material reads it (rpl::Material::needs_uv): same values, and the
// f64 atan2/asin of a sphere hit are skipped for untextured spheres (the ground).
RPK_INLINE bool surface(const KScene& S, const HitRec& hr, V3 o, V3 d, Surf& s, bool force_uv = false) {
  const rpl::Prim* p = S.prims + hr.prim;
  s.p = add(o, smul(hr.t, d));  // Ray::at (utility.rs:67)
  const bool known = hr.km != KM_UNKNOWN;
  s.material = known ? hr.km & ~KM_TRIANGLE : p->material;
  s.u = 0.0;
  s.v = 0.0;
  const bool need_uv = force_uv || S.mats[s.material].needs_uv != 0;
  if (known ? (hr.km & KM_TRIANGLE) != 0 : p->kind == rpl::PRIM_TRIANGLE) {
    const double u = hr.u, v = hr.v, w = 1.0 - u - v;
    const rpl::PrimRef& pr = S.prim_refs[hr.prim];
    const uint32_t i0 = pr.v[0], i1 = pr.v[1], i2 = pr.v[2];
    const V3 n0 = v3(S.vnrm[3 * i0], S.vnrm[3 * i0 + 1], S.vnrm[3 * i0 + 2]);
    const V3 n1 = v3(S.vnrm[3 * i1], S.vnrm[3 * i1 + 1], S.vnrm[3 * i1 + 2]);
    const V3 n2 = v3(S.vnrm[3 * i2], S.vnrm[3 * i2 + 1], S.vnrm[3 * i2 + 2]);
    s.n = add(add(smul(w, n0), smul(u, n1)), smul(v, n2));
    if (need_uv) {
      s.u = (w * S.vuv[2 * i0] + u * S.vuv[2 * i1]) + v * S.vuv[2 * i2];
      s.v = (w * S.vuv[2 * i0 + 1] + u * S.vuv[2 * i1 + 1]) + v * S.vuv[2 * i2 + 1];
    }
  } else {
    const V3 c = v3(p->g[0], p->g[1], p->g[2]);
    s.n = normalize(sub(s.p, c));
    return need_uv;  // the caller computes the sphere uv (shared site)
  }
  return false;
}

// ------------------------------------------------------------------ shading ----------------------

// x / 255.0 for a byte x, correctly rounded without a division: q0 = x * fl(1/255) is off by at most
// one ulp and one FMA residual step corrects it (exhaustively checked for all 256 x, tests/test_host.py).
RPK_INLINE double u8_unit(uint32_t x) {
  const double xd = (double)x, R = 1.0 / 255.0;
  const double q0 = xd * R;
  return __builtin_fma(__builtin_fma(-q0, 255.0, xd), R, q0);
}

// texture.rs:51-60: walk Checker indirections down to the texture that produces the value
// (validate() guarantees the walk terminates).
RPK_INLINE uint32_t tex_resolve(const KScene& S, uint32_t tid, const Surf& h) {
  while (S.texs[tid].kind == 4) {
    const rpl::Texture& t = S.texs[tid];
    const double s = floor(h.p.x) + floor(h.p.y) + floor(h.p.z);
    tid = fmod(s, 2.0) == 0.0 ? t.even : t.odd;
  }
  return tid;
}

// One RGBA8 texel (a non-temporal load, keeping the sky's random bounce lookups out of L2, cost +5 %)
RPK_INLINE uint32_t texel(const KScene& S, uint64_t i) { return S.texels[i]; }

// texture.rs:40-49 Image: clamp, then saturating `as u32` -> texel index
RPK_INLINE uint64_t image_texel(const rpl::Texture& t, const Surf& h) {
  const double w = (double)t.width, hh = (double)t.height;
  double x = h.u * w, y = h.v * hh;
  if (x < 0.0) x = 0.0;
  if (x > w - 1.0) x = w - 1.0;
  if (y < 0.0) y = 0.0;
  if (y > hh - 1.0) y = hh - 1.0;
  return t.texel_offset + (uint64_t)sat_u32(x) + (uint64_t)sat_u32(y) * t.width;
}

// texture.rs:21-118 value of a resolved (non-Checker) texture; `px` is the Image texel, fetched by the
// caller ahead of use so its latency overlaps other shading work.
RPK_INLINE V3 tex_value(const KScene& S, uint32_t tid, const Surf& h, uint32_t px) {
  const rpl::Texture& t = S.texs[tid];
  switch (t.kind) {
    case 1:  // DebugUVs
      return v3(h.u, h.v, 0.0);
    case 2:  // Solid
      return v3(t.color[0], t.color[1], t.color[2]);
    case 3:  // Image
      return v3(u8_unit(px & 0xffu), u8_unit((px >> 8) & 0xffu), u8_unit((px >> 16) & 0xffu));
      case 5: {  // Noise (texture.rs:62-68)
        double x = noise_real(sat_i64(floor(h.p.x)), sat_i64(floor(h.p.y)), sat_i64(floor(h.p.z)), t.seed);
        x = 0.5 * x + 0.5;
        return v3(x, x, x);
      }
      case 6: {  // Perlin (texture.rs:83-118)
        const V3 p = h.p;
        const V3 fp = v3(floor(p.x), floor(p.y), floor(p.z));
        const int64_t fx = sat_i64(fp.x), fy = sat_i64(fp.y), fz = sat_i64(fp.z);
        const int64_t cx = (int64_t)((uint64_t)fx + 1), cy = (int64_t)((uint64_t)fy + 1),
                      cz = (int64_t)((uint64_t)fz + 1);
        const int64_t s1 = (int64_t)((uint64_t)t.seed + 1), s2 = (int64_t)((uint64_t)t.seed + 2),
                      s3 = (int64_t)((uint64_t)t.seed + 3);
        double k[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const int64_t X = (q & 1) ? cx : fx, Y = (q & 2) ? cy : fy, Z = (q & 4) ? cz : fz;
          const V3 g = v3(noise_real(X, Y, Z, s1), noise_real(X, Y, Z, s2), noise_real(X, Y, Z, s3));
          k[q] = dot(sub(p, v3((double)X, (double)Y, (double)Z)), g);
        }
        V3 tt = sub(p, fp);
        tt.x = (tt.x * (tt.x * 6.0 - 15.0) + 10.0) * tt.x * tt.x * tt.x;
        tt.y = (tt.y * (tt.y * 6.0 - 15.0) + 10.0) * tt.y * tt.y * tt.y;
        tt.z = (tt.z * (tt.z * 6.0 - 15.0) + 10.0) * tt.z * tt.z * tt.z;
        const double k12 = (k[1] - k[0]) * tt.x + k[0], k34 = (k[3] - k[2]) * tt.x + k[2];
        const double k56 = (k[5] - k[4]) * tt.x + k[4], k78 = (k[7] - k[6]) * tt.x + k[6];
        const double k1234 = (k34 - k12) * tt.y + k12, k5678 = (k78 - k56) * tt.y + k56;
        const double kk = (k5678 - k1234) * tt.z + k1234;
        const double x = 0.5 * kk + 0.5;
        return v3(x, x, x);
      }
      default:  // Missing
      return v3(0.0, 0.0, 0.0);
  }
}

RPK_INLINE V3 tex_sample(const KScene& S, uint32_t tid, const Surf& h) {
  tid = tex_resolve(S, tid, h);
  const rpl::Texture& t = S.texs[tid];
  const uint32_t px = t.kind == 3 ? texel(S, image_texel(t, h)) : 0u;
  return tex_value(S, tid, h, px);
}

// material.rs:49-60 Emit::evaluate (SkySphere's texture value sampled by the caller)
RPK_INLINE V3 emit_eval(uint32_t kind, V3 color, V3 tex, V3 d, const Surf& h) {
  switch (kind) {
    case 1: return h.n;                                  // DebugNormals
    case 2: return color;                                // Color
    case 3: {                                            // SkyGradient
      const double t = 0.5 * (d.y / sqrt(norm2(d)) + 1.0);
      return add(smul(1.0 - t, v3(1.0, 1.0, 1.0)), smul(t, v3(0.5, 0.7, 1.0)));
    }
    case 4: return tex;                                  // SkySphere
    default: return v3(0.0, 0.0, 0.0);                   // None
  }
}

// material.rs:74-81 Absorb::evaluate (AlbedoMap's texture value sampled by the caller)
RPK_INLINE V3 absorb_eval(const rpl::Material& m, V3 tex) {
  switch (m.absorb_kind) {
    case 1: return v3(1.0, 1.0, 1.0);
    case 2: return v3(m.absorb_color[0], m.absorb_color[1], m.absorb_color[2]);
    case 3: return tex;
    default: return v3(0.0, 0.0, 0.0);
  }
}

// material.rs:27-34, 115-179 Scatter::evaluate.  Returns true and the new direction when scattered.
template <class R>
RPK_INLINE bool scatter_eval(const rpl::Material& m, V3 d, const Surf& h, R& rng, V3& nd) {
  switch (m.scatter_kind) {
    case 1: {  // Lambert (material.rs:115-130)
      DREG(DREG_LAMBERT)
      if (dot(h.n, d) > 0.0) return false;
      double x = 0.0, y = 0.0, s = 0.0;
      // UnitSphere (randomness.rs:58-73): tries of 2 draws, TRIES per round (see ring_ensure)
      for (uint32_t a = rng.pos;; a += 4u * TRIES) {
        DREG(DREG_LOOP_LAMBERT)
        ring_ensure(rng, (a + 4u * TRIES - 1u) >> 4);
        double tx[TRIES], ty[TRIES];
#pragma unroll
        for (int j = 0; j < TRIES; j++) {
          tx[j] = ring_sym(rng, a + 4u * j);
          ty[j] = ring_sym(rng, a + 4u * j + 2u);
        }
        bool done = false;
#pragma unroll
        for (int j = TRIES - 1; j >= 0; j--) {  // the first accepted try wins
          const double qx = tx[j], qy = ty[j], qs = qx * qx + qy * qy;
          if (qs < 1.0) { x = qx; y = qy; s = qs; rng.pos = a + 4u * (j + 1); done = true; }
        }
        if (done) break;
      }
      const double q = 2.0 * sqrt(1.0 - s);
      nd = normalize(add(h.n, v3(x * q, y * q, 1.0 - 2.0 * s)));
      return true;
    }
    case 2: {  // Metal (material.rs:132-152)
      DREG(DREG_METAL)
      if (dot(h.n, d) > 0.0) return false;
      double x = 0.0, y = 0.0, z = 0.0;
      // UnitBall (randomness.rs:39-53): tries of 3 draws, TRIES per round (see ring_ensure)
      for (uint32_t a = rng.pos;; a += 6u * TRIES) {
        DREG(DREG_LOOP_METAL)
        ring_ensure(rng, (a + 6u * TRIES - 1u) >> 4);
        double tx[TRIES], ty[TRIES], tz[TRIES];
#pragma unroll
        for (int j = 0; j < TRIES; j++) {
          tx[j] = ring_sym(rng, a + 6u * j);
          ty[j] = ring_sym(rng, a + 6u * j + 2u);
          tz[j] = ring_sym(rng, a + 6u * j + 4u);
        }
        bool done = false;
#pragma unroll
        for (int j = TRIES - 1; j >= 0; j--) {  // the first accepted try wins
          const double qx = tx[j], qy = ty[j], qz = tz[j];
          if ((qx * qx + qy * qy) + qz * qz < 1.0) { x = qx; y = qy; z = qz; rng.pos = a + 6u * (j + 1); done = true; }
        }
        if (done) break;
      }
      const V3 r = normalize(add(reflect(d, h.n), smul(m.scatter_param, v3(x, y, z))));
      if (dot(h.n, r) < 0.0) return false;
      nd = r;
      return true;
    }
    case 3: {  // Dielectric (material.rs:154-179)
      DREG(DREG_DIELEC)
      double eta;
      V3 n;
      if (dot(h.n, d) > 0.0) { eta = m.scatter_param; n = v3(-h.n.x, -h.n.y, -h.n.z); }
      else { eta = 1.0 / m.scatter_param; n = h.n; }
      double r0 = (1.0 - eta) / (1.0 + eta);
      r0 = r0 * r0;                                  // powi(2)
      const double x = 1.0 + dot(n, d);
      const double x2 = x * x;
      const double reflectance = r0 + (1.0 - r0) * (x * (x2 * x2));  // powi(5), LLVM binary expansion
      if (gen_f64(rng) < reflectance) {              // Bernoulli (randomness.rs:78-82)
        nd = reflect(d, n);
      } else {
        const double cos_theta = dot(n, d);          // refract (utility.rs:111-119)
        const double k = 1.0 - eta * eta * (1.0 - cos_theta * cos_theta);
        if (k < 0.0) nd = reflect(d, n);
        else nd = sub(smul(eta, d), smul(eta * cos_theta + sqrt(k), n));
      }
      return true;
    }
    default:
      return false;
  }
}

// Shading of one finished ray: the step of the reference's trace_path after the closest-hit query
// (render.rs:104-118 / 133-145, material.rs:104-110): the hit's surface record or the miss's
// Hit::at_infinity, textures, Scatter (the only RNG consumer), Absorb, Emit; T (*) emit goes into the sum
// (forward accumulation: main.rs:80 adds the sample's total, the association differs in the last ulp only).
// Returns true when the material scattered: (o, d) become the hit point and the new direction and T is
// multiplied by the absorption.  Hits and misses share one spherical-uv site and one texture site, so a
// wave with both pays for each f64 atan2/asin and texture walk once.
template <class R, class D, class U>
RPK_INLINE bool shade_ray(const KScene& S, const HitRec& hr, V3& o, V3& d, R& rng, D& T_x, D& T_y, D& T_z, D& sum_x,
                          D& sum_y, D& sum_z, bool first, U& hits) {
  const bool hit = hr.prim >= 0;
  Surf h;
  const rpl::Material* m = nullptr;
  bool sph_uv;
  if (hit) {
    DREG(DREG_SURF)
    DCYC_BEGIN(c0)
    sph_uv = surface(S, hr, o, d, h);
    m = &S.mats[h.material];
    DCYC_END(DCYC_SURF, c0)
  } else {
    DREG(DREG_MISS)
    // background.evaluate(ray, Hit::at_infinity(dir)) (render.rs:118,144; utility.rs:93-100)
    h.p = d;
    h.n = d;
    h.u = 0.0;
    h.v = 0.0;
    h.material = 0;
    sph_uv = S.background.needs_uv != 0;
  }
  if (sph_uv) {  // hittable.rs:59-62 for a sphere hit, utility.rs:96-97 for a miss
    DREG(DREG_SPHUV)
    DCYC_BEGIN(c1)
    const V3 q = hit ? h.n : d;
    h.u = 0.5 - atan2(q.z, q.x) / TAU_;
    h.v = asin(q.y) / PI_ + 0.5;
    DCYC_END(DCYC_SPHUV, c1)
  }
  // Textures: each lane reads at most one here -- the absorb map of a hit or the sky sphere of a miss
  // (or of an emissive hit); its Checker walk and Image texel load are issued BEFORE the scatter so
  // the load latency overlaps it.  A hit reading both takes the second in a rare extra pass.
  const uint32_t emit_kind = hit ? m->emit_kind : S.background.kind;
  const uint32_t emit_tex = hit ? m->emit_tex : S.background.tex;
  const bool ta = hit && m->absorb_kind == 3, te = emit_kind == 4;
  const bool t1 = ta || te;
  uint32_t tid1 = 0, px1 = 0;
  // a miss under an Image sky sphere: size and offset are kernel arguments (scalar registers), so the
  // texel load waits on no texture-table load
  const bool sky_img = !hit && S.background.img_w != 0;
  DCYC_BEGIN(c2)
  if (t1) {
    if (sky_img) {
      rpl::Texture t;
      t.width = S.background.img_w;
      t.height = S.background.img_h;
      t.texel_offset = S.background.img_off;
      tid1 = S.background.tex;
      px1 = texel(S, image_texel(t, h));
    } else {
      tid1 = tex_resolve(S, ta ? m->absorb_tex : emit_tex, h);
      const rpl::Texture& t = S.texs[tid1];
      if (t.kind == 3) px1 = texel(S, image_texel(t, h));
    }
  }
  DCYC_END(DCYC_TEXISSUE, c2)
  // scatter (the only RNG consumer; material.rs order scatter, absorb, emit -- the textures draw none)
  V3 nd = v3(0.0, 0.0, 0.0);
  bool scattered = false;
  if (hit) {
    DCYC_BEGIN(c3)
    scattered = scatter_eval(*m, d, h, rng, nd);
    DCYC_END(DCYC_SCATTER, c3)
  }
  V3 tex_ab = v3(0.0, 0.0, 0.0), tex_em = v3(0.0, 0.0, 0.0);
  DCYC_BEGIN(c4)
  if (t1) {
    DREG(DREG_TEX)
    const V3 tv = sky_img ? v3(u8_unit(px1 & 0xffu), u8_unit((px1 >> 8) & 0xffu), u8_unit((px1 >> 16) & 0xffu))
                          : tex_value(S, tid1, h, px1);
    if (ta) tex_ab = tv;
    else tex_em = tv;
  }
  if (ta && te) tex_em = tex_sample(S, emit_tex, h);
  DCYC_END(DCYC_TEXVAL, c4)
  DCYC_BEGIN(c5)
  const double* ecol = hit ? m->emit_color : S.background.color;
  const V3 em = emit_eval(emit_kind, v3(ecol[0], ecol[1], ecol[2]), tex_em, d, h);
  // emit + absorb (*) trace_path_continue (render.rs:108-115, 135-142), accumulated forward: each
  // bounce's T (*) emit goes straight into the pixel sum (main.rs:80 adds the sample's total; the
  // association differs in the last ulp only)
  sum_x = sum_x + T_x * em.x;
  sum_y = sum_y + T_y * em.y;
  sum_z = sum_z + T_z * em.z;
  if (hit && first) hits++;
  if (scattered) {
    const V3 ab = absorb_eval(*m, tex_ab);
    T_x = T_x * ab.x;
    T_y = T_y * ab.y;
    T_z = T_z * ab.z;
    o = h.p;
    d = nd;
  }
  DCYC_END(DCYC_EMIT, c5)
  return scattered;
}

// ------------------------------------------------------------------ render kernel ----------------

RPK_INLINE V3 matvec(const double* m, V3 v) {  // nalgebra Matrix3 * Vector3 (column axpy)
  return v3((v.x * m[0] + v.y * m[3]) + v.z * m[6], (v.x * m[1] + v.y * m[4]) + v.z * m[7],
            (v.x * m[2] + v.y * m[5]) + v.z * m[8]);
}

// All launch arguments in one kernarg struct.  The persistent loop re-reads the fields it needs through
// a laundered pointer to the kernarg segment (scalar loads, served by the constant cache) instead of
// keeping ~70 uniform values live in SGPRs for the whole kernel: that SGPR pressure otherwise spills
// into VGPR lanes and halves the wave occupancy of this register-bound kernel.
struct KArgs {
  KScene S;
  KParams P;
  double* out;
  float* out_fg;
  unsigned long long* ctr;
  unsigned int* queue;       // the unit queue's next index (workspace-owned, zeroed before the launch)
  unsigned long long* diag;  // RPK_DIAG builds only (DIAG_N counters)
};
typedef const __attribute__((address_space(4))) KArgs* KArgsPtr;

RPK_INLINE KScene load_scene(KArgsPtr A) {
  KScene S;
  S.nodes = A->S.nodes;
  S.prims = A->S.prims;
  S.prim_refs = A->S.prim_refs;
  S.vnrm = A->S.vnrm;
  S.vuv = A->S.vuv;
  S.mats = A->S.mats;
  S.texs = A->S.texs;
  S.texels = A->S.texels;
  S.background.kind = A->S.background.kind;
  S.background.tex = A->S.background.tex;
  S.background.needs_uv = A->S.background.needs_uv;
  S.background.img_w = A->S.background.img_w;
  S.background.img_h = A->S.background.img_h;
  S.background.img_off = A->S.background.img_off;
  S.background.color[0] = A->S.background.color[0];
  S.background.color[1] = A->S.background.color[1];
  S.background.color[2] = A->S.background.color[2];
  S.root = A->S.root;
  S.always_first = A->S.always_first;
  S.n_always = A->S.n_always;
  S.qbound = A->S.qbound;
  S.node_format = A->S.node_format;
  S.leaf_break = A->S.leaf_break;
  S.stack_depth = A->S.stack_depth;
  S.lds_depth = A->S.lds_depth;
  S.spill = A->S.spill;
  S.rng_slab = A->S.rng_slab;
  S.unit_t0 = A->S.unit_t0;
  return S;
}

RPK_INLINE KArgsPtr kargs() {
  KArgsPtr p = (KArgsPtr)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}

// Pull the next unit (pixel, sample batch) of the shard from the unit queues.  Queue order: shard tiles
// (in cost or Z-order when tile_order is set), inside a tile the pixels row-major, each pixel's batches
// consecutive; slots of edge tiles outside the frame are skipped.  Returns false when every queue is drained.
RPK_INLINE uint32_t udiv(uint32_t n, uint32_t m, uint32_t s) { return (uint32_t)(((uint64_t)n * m) >> s); }  // rp_kernel.h make_div32
#define RPK_UDIV(n, dv) udiv((n), A->P.dv.m, A->P.dv.s)

template <bool PROBE>
RPK_INLINE bool fetch_pixel(uint32_t& slot, uint32_t& pi, uint32_t& pj, uint32_t& batch) {
  KArgsPtr A = kargs();
  unsigned int* queue = A->queue;
  const uint32_t tw = A->P.tw, th = A->P.th;
  if (PROBE && A->P.probe_n) {  // cost probe: an n x n lattice per tile (cell centres), clamped into the frame
    slot = atomicAdd(queue, 1u);
    if ((uint64_t)slot >= A->P.n_queue) return false;
    batch = 0;
    const uint32_t n = A->P.probe_n;
    const uint32_t k = slot / A->P.probe_px, sub = slot % A->P.probe_px;
    const uint32_t dk = A->P.shard + k * A->P.nshards, t = A->P.tile_map ? A->P.tile_map[dk] : dk;
    const uint32_t tx = t % A->P.tiles_x, ty = t / A->P.tiles_x;
    pi = min(tx * tw + min((sub % n) * tw / n + tw / (2u * n), tw - 1u), A->P.W - 1u);
    pj = min(ty * th + min((sub / n) * th / n + th / (2u * n), th - 1u), A->P.H - 1u);
    return true;
  }
  const uint32_t tile_px = tw * th, tile_units = tile_px * A->P.nbatch;
  if (!PROBE && A->P.unit_order) {
    // the learned per-unit order (rp_sched.hip): queue g serves the chunks g, g + G, ... of C consecutive positions,
    // position p holds unit unit_order[p] = slot * nbatch + batch -- with several frames per launch, position p is frame
    // p mod n_frames of unit unit_order[p / n_frames] (a unit's frames consecutive); the same drained-queue walk as the
    // tile queues below
    const uint32_t G = max(A->P.queue_groups, 1u), C = A->P.order_chunk, GC = G * C;
    const uint32_t home = G > 1 ? blockIdx.x % G : 0u;
    const uint32_t Q = (uint32_t)A->P.n_queue;
    for (uint32_t tries = 0;;) {
      uint32_t g = home + tries;
      if (g >= G) g -= G;
      g = __builtin_amdgcn_readfirstlane(g);
      const uint32_t rest = Q % GC, nq = (Q / GC) * C + min(rest - min(rest, g * C), C);
      const uint32_t q = atomicAdd(A->queue + g * QUEUE_STRIDE, 1u);
      const bool drained = q >= nq;
      if (__ballot(drained) != 0) {
        ++tries;
        if (drained) {
          if (tries >= G) return false;
          continue;
        }
      }
      const uint32_t i = RPK_UDIV(q, dv_ochunk);
      uint32_t pos = i * GC + g * C + (q - i * C), f = 0;
      if (A->P.n_frames > 1) {
        const uint32_t r = RPK_UDIV(pos, dv_frames);
        f = pos - r * A->P.n_frames;
        pos = r;
      }
      const uint32_t u = A->P.unit_order[pos];
      const uint32_t sl = RPK_UDIV(u, dv_nbatch);
      batch = u - sl * A->P.nbatch + f * A->P.nbatch;  // (the unit carries its global batch)
      slot = sl;
      const uint32_t k = RPK_UDIV(sl, dv_tile_px), local = sl - k * tile_px;
      const uint32_t dk = A->P.shard + k * A->P.nshards, t = A->P.tile_map ? A->P.tile_map[dk] : dk;
      const uint32_t ty = RPK_UDIV(t, dv_tiles_x), tx = t - ty * A->P.tiles_x;
      const uint32_t lj = RPK_UDIV(local, dv_tw), li = local - lj * tw;
      pi = tx * tw + li;
      pj = ty * th + lj;
      if (pi < A->P.W && pj < A->P.H) return true;
    }
  }
  // Per-XCD queues (rp.h RP_QUEUES_*): blocks blockIdx mod G share an XCD; their queue g serves the tiles
  // k = g, g + G, ... of the order (or the g-th run of it), and once it is drained they take units from the
  // next queues in turn.  Every fetch starts at the home queue: a drained queue costs one failed increment.
  // The queue a wave increments is wave-uniform (`tries` moves for the whole wave once any lane finds the
  // queue drained -- then it is drained for every lane), so the compiler folds the lanes' atomicAdd into one
  // wave atomic (ballot + mbcnt); a per-lane atomic on one word cost C3 +35 %.
  // several frames per launch: n_frames x n_shard_tiles virtual tiles (rp_kernel.h KParams::n_frames)
  const uint32_t G = max(A->P.queue_groups, 1u), K = A->P.n_shard_tiles * (PROBE ? 1u : A->P.n_frames);
  const uint32_t home = G > 1 ? blockIdx.x % G : 0u;
  for (uint32_t tries = 0;;) {
    uint32_t g = home + tries;
    if (g >= G) g -= G;
    g = __builtin_amdgcn_readfirstlane(g);
    // queue g serves the chunks g, g + G, ... of C consecutive tiles of the order: tile k of its i-th unit
    // run is (i / C) * G * C + g * C + i % C
    const uint32_t C = A->P.queue_chunk, GC = G * C;
    const uint32_t rest = K % GC, nk = (K / GC) * C + min(rest - min(rest, g * C), C);
    const uint32_t q = atomicAdd(queue + g * QUEUE_STRIDE, 1u);
    const bool drained = (uint64_t)q >= (uint64_t)nk * tile_units;
    if (__ballot(drained) != 0) {
      ++tries;
      if (drained) {
        if (tries >= G) return false;  // every queue drained
        continue;
      }
    }
    // (PROBE launches decode with plain divisions: one small launch)
    uint32_t i = PROBE ? q / tile_units : RPK_UDIV(q, dv_units);
    uint32_t rem = q - i * tile_units;
    if (!PROBE && A->P.frames_inter == 2u) {
      // RP_FRAME_ORDER_PIXEL: the n_frames consecutive virtual tiles of a queue's sequence (one shard tile of every
      // frame) as one run of units with a unit's frames consecutive -- a wave holds ~64 / n_frames pixels x their frames
      const uint32_t grp = RPK_UDIV(i, dv_frames);
      const uint32_t o = (i - grp * A->P.n_frames) * tile_units + rem;
      const uint32_t u = RPK_UDIV(o, dv_frames);
      i = grp * A->P.n_frames + (o - u * A->P.n_frames);
      rem = u;
    }
    const uint32_t ic = PROBE ? i / C : RPK_UDIV(i, dv_chunk);
    uint32_t k = ic * GC + g * C + (i - ic * C);
    // a tile's units pixel-major, a pixel's batches consecutive: a wave fetches 64 / nbatch pixels with all
    // their batches, whose camera rays traverse nearly the same nodes (C3 -0.9 %, C5 -0.9 % against
    // batch-major, ab32)
    const uint32_t local = PROBE ? rem / A->P.nbatch : RPK_UDIV(rem, dv_nbatch);
    batch = rem - local * A->P.nbatch;
    if (!PROBE && A->P.n_frames > 1) {  // virtual tile -> frame f, its tile k; the unit carries its global batch
      uint32_t f;
      if (A->P.frames_inter) {
        const uint32_t r = RPK_UDIV(k, dv_frames);
        f = k - r * A->P.n_frames;
        k = r;
      } else {
        f = RPK_UDIV(k, dv_tiles);
        k -= f * A->P.n_shard_tiles;
      }
      batch += f * A->P.nbatch;
    }
    if (!PROBE && A->P.tile_order) k = A->P.tile_order[k];  // the queue hands out shard tiles in cost order
    slot = k * tile_px + local;                     // output slot: shard tile order (rp_shard_unpack)
    const uint32_t dk = A->P.shard + k * A->P.nshards, t = A->P.tile_map ? A->P.tile_map[dk] : dk;
    const uint32_t ty = PROBE ? t / A->P.tiles_x : RPK_UDIV(t, dv_tiles_x), tx = t - ty * A->P.tiles_x;
    const uint32_t lj = PROBE ? local / tw : RPK_UDIV(local, dv_tw), li = local - lj * tw;
    pi = tx * tw + li;
    pj = ty * th + lj;
    if (pi < A->P.W && pj < A->P.H) return true;
  }
}

// RNG contract (include/rp.h): batch b of pixel (i, j) is its own StdRng stream,
// seed_from_u64(seed + b * W * H + j * W + i); batch 0 is the per-pixel stream of the original contract.
RPK_INLINE uint64_t unit_seed(KArgsPtr A, uint32_t pi, uint32_t pj, uint32_t batch) {
  return A->P.seed + (uint64_t)batch * A->P.W * A->P.H + (uint64_t)pj * A->P.W + pi;
}
// The frame of a unit's (global) batch and its batch within the frame (several frames per launch: KParams::n_frames).
RPK_INLINE uint32_t unit_frame(KArgsPtr A, uint32_t batch) { return A->P.n_frames > 1 ? RPK_UDIV(batch, dv_nbatch) : 0u; }
// Samples in this unit's batch.
RPK_INLINE uint32_t unit_spp(KArgsPtr A, uint32_t batch) {
  const uint32_t b = batch - unit_frame(A, batch) * A->P.nbatch;
  return min(A->P.spp_batch, A->P.spp - b * A->P.spp_batch);
}

// Camera::shoot (render.rs:32-52) from the jittered frame coordinates (ju, jv) and the UnitDisk sample (dx, dy): one
// definition for the path loop (start_sample) and the coherent primary pass, which passes (0, 0) -- with lens_radius 0
// the disk is multiplied by 0 and only the signs of zeros could differ (the direction never: -focal - 0 and
// x - (+-0) for x != 0 are exact, and x = (2 ju - 1) ... is +0 when 2 ju - 1 = 0).
RPK_INLINE void camera_dir(KArgsPtr A, double ju, double jv, double dx, double dy, V3& o, V3& d) {
  // tan(fov/2) is computed on the host (render.rs:33 is a per-camera constant; same libm as the reference)
  const double lens = A->P.lens, tanf = A->P.tan_fov, focal = A->P.focal, aspect = A->P.aspect;
  const V3 lo = v3(lens * dx, lens * dy, 0.0);
  const V3 dl = normalize(sub(v3((2.0 * ju - 1.0) * tanf * focal * aspect, (2.0 * jv - 1.0) * tanf * focal, -focal), lo));
  double m[9];
#pragma unroll
  for (int q = 0; q < 9; q++) m[q] = A->P.orient[q];
  d = matvec(m, dl);
  o = add(matvec(m, lo), v3(A->P.pos[0], A->P.pos[1], A->P.pos[2]));
}

// One camera sample (main.rs:75-76): make_uv_jitter draws 2s, 2s+1 of a CLONE of the pixel-start
// stream (render.rs:74-82) = keystream words 4s..4s+3 = block s/4 at offset 4(s%4); Camera::shoot
// (render.rs:32-52) then draws its UnitDisk from the main stream (even when lens_radius == 0).
template <class R>
RPK_INLINE void start_sample(R& rng, uint32_t s, uint32_t pi, uint32_t pj, V3& o, V3& d) {
  DREG(DREG_START_SAMPLE)
  KArgsPtr A = kargs();
  const uint4 jw = rng_jitter(rng, s);
  const uint32_t w0 = jw.x, w1 = jw.y, w2 = jw.z, w3 = jw.w;
  const double ju = ((double)pi + words_f64(w0, w1)) / (double)A->P.W;
  const double jv = ((double)pj + words_f64(w2, w3)) / (double)A->P.H;
  double dx = 0.0, dy = 0.0;
  // UnitDisk (randomness.rs:21-34): tries of 2 draws, TRIES per round (see ring_ensure)
  for (uint32_t a = rng.pos;; a += 4u * TRIES) {
    ring_ensure(rng, (a + 4u * TRIES - 1u) >> 4);
    double tx[TRIES], ty[TRIES];
#pragma unroll
    for (int j = 0; j < TRIES; j++) {
      tx[j] = ring_sym(rng, a + 4u * j);
      ty[j] = ring_sym(rng, a + 4u * j + 2u);
    }
    bool done = false;
#pragma unroll
    for (int j = TRIES - 1; j >= 0; j--) {  // the first accepted try wins
      const double qx = tx[j], qy = ty[j];
      if (qx * qx + qy * qy < 1.0) { dx = qx; dy = qy; rng.pos = a + 4u * (j + 1); done = true; }
    }
    if (done) break;
  }
  camera_dir(kargs(), ju, jv, dx, dy, o, d);
}

}  // namespace rpk
