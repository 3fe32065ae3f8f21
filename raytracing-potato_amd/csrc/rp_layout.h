// rp_layout.h -- device-resident scene layout shared by the host builder (rp_bvh.cpp) and the HIP
// kernels (rp_kernel.hip).  Plain structs, no HIP types, so the builder can be unit-tested on the CPU.
//
// Layout rationale (DESIGN.md "Data layout in HBM"): traversal is one ray per lane, so neighbouring
// lanes read unrelated nodes; what matters is that one lane's node fetch is a few wide (16 B) loads
// from one 128 B (or 64 B) record.  Each wide node stores all four children's boxes (the parent tests them
// with one fetch), and primitives are stored contiguously in leaf
// order with the triangle operands pre-subtracted exactly as hittable.rs:71-72 computes them.
#pragma once
#include <math.h>
#include <stdint.h>

namespace rpl {

// Two 4-wide node formats, chosen per scene (rp_scene_options.node_format; rp_api.cpp picks by size):
//
// Node4 (128 B, cache-resident trees): the four child boxes per axis (SoA within the record: 6 float4
// loads + the children) in f32, rounded OUTWARD from the exact f64 boxes.
//
// Node4Q (64 B, large trees): the child boxes quantized to 8 bits per plane in a per-node frame (per axis an
// f32 origin o and step s: plane(q) = o + q * s, exact in f64, q = 0..255), rounded outward from the exact
// f64 boxes.  16 B chunks: {o.x, o.y, o.z, s.x} {s.y, s.z, lo_x, hi_x} {lo_y, hi_y, lo_z, hi_z} {child[4]}.
// Four loads per visit instead of seven; the dequantization (v_perm + v_cvt_f32_ubyte per plane, the same
// one FMA) costs ALU.  Measured: C5 (10 M triangles, SAH tree) -4.4 % frame time,
// C3 (bunny, L2-resident) +0.7 %.
//
// Both are tested with a conservative slab test (rp_device.h trav_step) so no primitive the exact f64
// test would accept is ever culled.  Child entries:
//   inner node : node index (bit 31 clear)
//   leaf       : ENTRY_LEAF | (count - 1) << LEAF_SHIFT | first primitive   (count 1..8)
//   empty slot : ENTRY_EMPTY (Node4: lo = +inf, hi = -inf; Node4Q: plane bytes meaningless, masked by the entry)
struct alignas(16) Node4 {
  float lo_x[4], hi_x[4];
  float lo_y[4], hi_y[4];
  float lo_z[4], hi_z[4];
  uint32_t child[4];
  uint32_t pad[4];
};
static_assert(sizeof(Node4) == 128, "Node4 must be 128 B");

struct alignas(16) Node4Q {
  float o[3];  // frame origin per axis
  float s[3];  // frame step per axis
  uint8_t lo_x[4], hi_x[4];
  uint8_t lo_y[4], hi_y[4];
  uint8_t lo_z[4], hi_z[4];
  uint32_t child[4];
};
static_assert(sizeof(Node4Q) == 64, "Node4Q must be 64 B");

// Node8Q (128 B, one cache line; host SAH trees): eight children quantized like Node4Q.  Slot s (0..7) holds a
// child lying towards (s&1 ? +x : -x, s&2 ? +y : -y, s&4 ? +z : -z) of the node's centre, so a ray visits its
// children in the order of rank = slot ^ octant (octant bit a set when the ray's slope on axis a is negative):
// approximately near-first without sorting.  Inner children are consecutive records from `inner` in slot order
// (child at slot s = (inner & W8_INDEX) + popcount(imask & ((1 << s) - 1)), imask = inner >> 24); the primitives
// of the leaf children are one run from `prim`, pmask[s] the bits of slot s's leaf in that run (<= 32 bits: at
// most 8 leaves of <= 4 primitives).  16 B chunks: {o.x, o.y, o.z, s.x} {s.y, s.z, inner, prim}
// {lo_x, hi_x} {lo_y, hi_y} {lo_z, hi_z} {pmask[0..3]} {pmask[4..7]} {pad}: seven loads per visit.
struct alignas(16) Node8Q {
  float o[3];
  float s[3];
  uint32_t inner;
  uint32_t prim;
  uint8_t lo_x[8], hi_x[8];
  uint8_t lo_y[8], hi_y[8];
  uint8_t lo_z[8], hi_z[8];
  uint32_t pmask[8];
  uint32_t pad[4];
};
static_assert(sizeof(Node8Q) == 128, "Node8Q must be 128 B");
constexpr uint32_t W8_INDEX = 0x00FFFFFFu;  // Node8Q.inner: family index bits (imask above)
constexpr uint32_t W8_MAX_NODES = 1u << 24;
constexpr uint32_t W8_MAX_LEAF = 4;

enum : uint32_t { NODES_F32 = 1, NODES_Q8 = 2, NODES_W8 = 3 };  // = RP_NODES_F32 / _Q8 / _W8 (include/rp.h)

#if defined(__HIPCC__)
#define RPL_HD __host__ __device__
#else
#define RPL_HD
#endif

// f64 -> f32 rounded towards -inf / +inf; Node4 child boxes rounded outward
RPL_HD inline float f32_rd(double x) {
  float f = (float)x;
  if ((double)f > x) f = nextafterf(f, -__builtin_huge_valf());
  return f;
}
RPL_HD inline float f32_ru(double x) {
  float f = (float)x;
  if ((double)f < x) f = nextafterf(f, __builtin_huge_valf());
  return f;
}
RPL_HD inline void f32_child(Node4& n, int c, const double lo[3], const double hi[3]) {
  n.lo_x[c] = f32_rd(lo[0]); n.hi_x[c] = f32_ru(hi[0]);
  n.lo_y[c] = f32_rd(lo[1]); n.hi_y[c] = f32_ru(hi[1]);
  n.lo_z[c] = f32_rd(lo[2]); n.hi_z[c] = f32_ru(hi[2]);
}
RPL_HD inline void f32_empty(Node4& n, int c) {
  n.lo_x[c] = n.lo_y[c] = n.lo_z[c] = __builtin_huge_valf();
  n.hi_x[c] = n.hi_y[c] = n.hi_z[c] = -__builtin_huge_valf();
}

// Node frames.  qframe(lo, hi) picks the frame of a node box [lo, hi] along one axis (finite, lo <= hi):
//   o <= lo and o + 255 s >= hi;
//   o is a multiple of 2^(E_s - 8) (E_s = floor(log2 s)) or, far from 0, of its own ulp (>= 2^(E_s - 8)),
//   and |o| < 2^(E_s + 29), so o + q s is a multiple of 2^(E_s - 23) below 2^(E_s + 30): exact in f64;
//   s >= (hi - lo) (1 + 2^-7) / 255 leaves room for o's rounding below lo;  s >= 2^-60.
// plane_q(o, s, q) is that exact value; q_down / q_up the conservative quantization of a child's bounds.
RPL_HD inline double plane_q(float o, float s, uint32_t q) { return (double)o + (double)q * (double)s; }
RPL_HD inline void qframe(double lo, double hi, float& o, float& s) {
  const float o0 = f32_rd(lo);
  double need = fmax((hi - lo) * (1.0 + 0x1p-7), hi - (double)o0) / 255.0 * (1.0 + 0x1p-40);
  need = fmax(fmax(need, fabs((double)o0) * 0x1p-28), 0x1p-60);
  s = f32_ru(need);
  int e = 0;
  (void)frexp((double)s, &e);  // s = m 2^e, m in [0.5, 1): E_s = e - 1
  if (fabs(lo) < ldexp(1.0, e + 15)) {
    const double g = ldexp(1.0, e - 9);
    o = (float)(floor(lo / g) * g);
  } else {
    o = o0;
  }
  while (plane_q(o, s, 255u) < hi) s = nextafterf(s, __builtin_huge_valf());  // not expected to run
}
RPL_HD inline uint32_t q_down(double x, float o, float s) {  // largest q with plane(q) <= x (0 if none)
  double f = floor((x - (double)o) / (double)s);
  uint32_t q = f <= 0.0 ? 0u : (f >= 255.0 ? 255u : (uint32_t)f);
  while (q > 0u && plane_q(o, s, q) > x) q--;
  while (q < 255u && plane_q(o, s, q + 1u) <= x) q++;
  return q;
}
RPL_HD inline uint32_t q_up(double x, float o, float s) {  // smallest q with plane(q) >= x (255 if none)
  double c = ceil((x - (double)o) / (double)s);
  uint32_t q = c <= 0.0 ? 0u : (c >= 255.0 ? 255u : (uint32_t)c);
  while (q < 255u && plane_q(o, s, q) < x) q++;
  while (q > 0u && plane_q(o, s, q - 1u) >= x) q--;
  return q;
}
// Frames are built from the primitive boxes of the tree, so every |o| and 255 s stays below
// qbound(amax) (amax = the largest |coordinate| of those boxes): the traversal's slack uses it
// (rp_device.h setup_ray32).  Coordinates beyond 2^54 are refused (rp_bvh.cpp build).
RPL_HD inline double qbound(double amax) { return 4.0 * amax + 0x1p-50; }
constexpr double COORD_MAX = 0x1p54;

// Quantize child c of node n (Node4Q or Node8Q) from its exact f64 box (lo[3], hi[3]); a non-finite bound (NaN geometry: never
// hit) takes the whole frame.
template <class N>
RPL_HD inline void quantize_child(N& n, int c, const double lo[3], const double hi[3]) {
  uint8_t* L[3] = {n.lo_x, n.lo_y, n.lo_z};
  uint8_t* H[3] = {n.hi_x, n.hi_y, n.hi_z};
  for (int a = 0; a < 3; a++) {
    const bool ok = lo[a] == lo[a] && hi[a] == hi[a];
    L[a][c] = ok ? (uint8_t)q_down(lo[a], n.o[a], n.s[a]) : (uint8_t)0;
    H[a][c] = ok ? (uint8_t)q_up(hi[a], n.o[a], n.s[a]) : (uint8_t)255;
  }
}
template <class N>
RPL_HD inline void empty_child(N& n, int c) {
  n.lo_x[c] = n.lo_y[c] = n.lo_z[c] = 255;
  n.hi_x[c] = n.hi_y[c] = n.hi_z[c] = 0;
}

constexpr uint32_t ENTRY_LEAF = 0x80000000u;
constexpr uint32_t ENTRY_EMPTY = 0xFFFFFFFFu;
constexpr uint32_t LEAF_SHIFT = 28;
constexpr uint32_t LEAF_FIRST_MASK = (1u << LEAF_SHIFT) - 1u;
constexpr uint32_t LEAF_MAX = 8;
constexpr uint32_t MAX_PRIMS = LEAF_FIRST_MASK - LEAF_MAX;  // keeps every leaf entry distinct from EMPTY

enum : uint32_t { PRIM_SPHERE = 0, PRIM_TRIANGLE = 1 };

// Primitive in leaf order: 80 B, everything the intersection test reads (five 16 B loads per lane).
//   triangle: g = {a.xyz, (a-b).xyz, (a-c).xyz}
//   sphere:   g = {center.xyz, radius, 0...}
// Adding data here costs more than it saves: each extra 16 B is one more divergent load per test (a
// variant carrying the determinant's products, 176 B, ran 10% slower although it saved 12 f64 ops).
struct alignas(16) Prim {
  double g[9];
  uint32_t kind;
  uint32_t material;
};
static_assert(sizeof(Prim) == 80, "Prim must be 80 B");

// Per primitive, read only for the closest hit: global vertex ids (normals/uvs) and the source hittable.
struct alignas(16) PrimRef {
  uint32_t v[3];
  uint32_t src;  // index of the source hittable (diagnostics / tie analysis)
};
static_assert(sizeof(PrimRef) == 16, "PrimRef must be 16 B");

// Material: rp_material flattened (material.rs:87-91).
struct alignas(16) Material {
  uint32_t scatter_kind, absorb_kind, emit_kind, absorb_tex;
  uint32_t emit_tex, needs_uv, pad1, pad2;  // needs_uv: a texture this material samples reads hit.uv
  double scatter_param;
  double absorb_color[3];
  double emit_color[3];
  double pad3;
};
static_assert(sizeof(Material) == 96, "Material must be 96 B");

// Texture (texture.rs:10-18); Image texels live in one RGBA8 pool.
struct alignas(16) Texture {
  uint32_t kind, odd, even, width;
  uint32_t height, pad0;
  int64_t seed;
  uint64_t texel_offset;  // in texels (uint32) into the pool
  double color[3];
  double pad1;
};
static_assert(sizeof(Texture) == 72 || sizeof(Texture) == 80, "Texture size");

struct Emit {
  uint32_t kind, tex;  // tex only read for SkySphere
  uint32_t needs_uv, img_off;
  uint32_t img_w, img_h;  // SkySphere over an Image (background): its size (img_w = 0 otherwise)
  double color[3];
};

}  // namespace rpl
