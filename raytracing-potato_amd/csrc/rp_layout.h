// rp_layout.h -- device-resident scene layout shared by the host builder (rp_bvh.cpp) and the HIP
// kernels (rp_kernel.hip).  Plain structs, no HIP types, so the builder can be unit-tested on the CPU.
//
// Layout rationale (DESIGN.md "Data layout in HBM"): traversal is one ray per lane, so neighbouring
// lanes read unrelated nodes; what matters is that one lane's node fetch is a few wide (16 B) loads
// from one 128 B record.  Each wide node stores all four children's boxes (the parent tests them with
// one fetch), grouped per axis (SoA within the record), and primitives are stored contiguously in leaf
// order with the triangle operands pre-subtracted exactly as hittable.rs:71-72 computes them.
#pragma once
#include <stdint.h>

namespace rpl {

// 4-wide BVH node: 128 B, one cache line pair-aligned record per lane fetch.  The four child boxes
// are stored per axis (SoA within the record: 6 x float4 loads) in f32, rounded OUTWARD from the exact
// f64 boxes, and tested with a conservative slab test (rp_kernel.hip) so no primitive the exact f64
// test would accept is ever culled.  Child entries:
//   inner node : node index (bit 31 clear)
//   leaf       : ENTRY_LEAF | (count - 1) << LEAF_SHIFT | first primitive   (count 1..8)
//   empty slot : ENTRY_EMPTY
struct alignas(16) Node4 {
  float lo_x[4], hi_x[4];
  float lo_y[4], hi_y[4];
  float lo_z[4], hi_z[4];
  uint32_t child[4];
  uint32_t pad[4];
};
static_assert(sizeof(Node4) == 128, "Node4 must be 128 B");

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
