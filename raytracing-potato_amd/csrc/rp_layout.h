// rp_layout.h -- device-resident scene layout shared by the host builder (rp_bvh.cpp) and the HIP
// kernels (rp_kernel.hip).  Plain structs, no HIP types, so the builder can be unit-tested on the CPU.
//
// Layout rationale (DESIGN.md "Data layout in HBM"): traversal is one ray per lane, so neighbouring
// lanes read unrelated nodes; what matters is that one lane's node fetch is a few wide (16 B) loads
// from as few 128 B lines as possible.  Each BVH2 node therefore stores BOTH children's boxes
// (the parent tests the pair with one fetch) with the six slabs of the two children grouped per axis
// (SoA within the record), and primitives are stored contiguously in leaf order with the triangle
// operands pre-subtracted exactly as hittable.rs:71-72 computes them (a, a-b, a-c).
#pragma once
#include <stdint.h>

namespace rpl {

// Binary BVH node: 128 B, 16-B aligned.  Child c of the node:
//   count[c] > 0  -> leaf, primitives [child[c], child[c] + count[c]) of the prim array
//   count[c] == 0 -> inner node index child[c] (>= 0), or empty slot when child[c] < 0
struct alignas(16) Node2 {
  double lo_x[2], hi_x[2];
  double lo_y[2], hi_y[2];
  double lo_z[2], hi_z[2];
  int32_t child[2];
  uint32_t count[2];
  uint32_t pad[4];
};
static_assert(sizeof(Node2) == 128, "Node2 must be 128 B");

enum : uint32_t { PRIM_SPHERE = 0, PRIM_TRIANGLE = 1 };

// Primitive in leaf order: 96 B.
//   triangle: g = {a.xyz, (a-b).xyz, (a-c).xyz}, v = global vertex ids (normals/uvs for shading)
//   sphere:   g = {center.xyz, radius, 0...}
struct alignas(16) Prim {
  double g[9];
  uint32_t kind;
  uint32_t material;
  uint32_t v[3];
  uint32_t src;  // index of the source hittable (diagnostics / tie analysis)
};
static_assert(sizeof(Prim) == 96, "Prim must be 96 B");

// Material: rp_material flattened (material.rs:87-91).
struct alignas(16) Material {
  uint32_t scatter_kind, absorb_kind, emit_kind, absorb_tex;
  uint32_t emit_tex, pad0, pad1, pad2;
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
  uint32_t kind, tex;
  double color[3];
};

}  // namespace rpl
