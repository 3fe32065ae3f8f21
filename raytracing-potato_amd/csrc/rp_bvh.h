// rp_bvh.h -- host-side scene validation, SAH BVH build and packing into the device layout.
//
// Replaces Bvh::new / make_bvh / split (bvh.rs:36-91).  The reference's median split with one
// primitive per leaf is not reproduced: the closest hit does not depend on tree shape or visit order
// except for exact-t ties, so the build is free to use a binned-SAH tree with
// small leaves, which roughly halves node visits on the bunny (the r = 1000 ground sphere ends up as
// a leaf next to the root instead of inflating every ancestor box).
#pragma once
#include <stdint.h>

#include <memory>
#include <string>
#include <vector>

#include "../../include/rp.h"
#include "rp_layout.h"

namespace rpb {

enum : uint32_t { COLLAPSE_GREEDY = 0, COLLAPSE_SAH = 1 };

struct BuildOptions {
  uint32_t max_leaf = 4;        // primitives per leaf at most (<= rpl::LEAF_MAX)
  uint32_t bins = 32;           // SAH bins per axis
  double cost_traverse = 0.7;   // relative cost of one node (two child boxes); C3 sweep 0.35-1.5: 0.7 best (-1..2 %)
  double cost_intersect = 1.0;  // relative cost of one primitive test
  bool tables_only = false;     // shading tables only (nodes/prims left empty: the device builder makes them)
  bool vertex_tables = true;    // vnrm / vuv (false: the caller uploads the meshes' normals and uvs itself)
  // Primitives kept out of the tree and tested first for every ray: among the always_max largest boxes
  // (surface area), those at least always_ratio times the area of the box of everything else (config C3's
  // ground sphere, r = 1000 under a bunny of size ~0.2).  always_max = 0 disables.
  uint32_t always_max = 4;
  double always_ratio = 4.0;
  uint32_t node_format = rpl::NODES_F32;  // rpl::NODES_F32 (Node4), _Q8 (Node4Q), _W8 (Node8Q) or 0 (auto_node_format)
  uint32_t collapse = COLLAPSE_SAH;  // 4-wide collapse: COLLAPSE_GREEDY (largest-area child first) or _SAH (rp_bvh.cpp)
  uint32_t threads = 0;                   // host build threads (0 = the machine's, at most 16); same tree for any
};

struct PackedScene {
  uint32_t node_format = rpl::NODES_F32;  // resolved (never 0 after a tree build)
  std::vector<rpl::Node4> nodes;      // NODES_F32: nodes[root] is the root (always an inner record)
  std::vector<rpl::Node4Q> qnodes;    // NODES_Q8: the same tree in the quantized format
  std::vector<rpl::Node8Q> wnodes;    // NODES_W8: the 8-wide quantized tree (its own leaf order)
  std::vector<rpl::Prim> prims;       // leaf order
  std::vector<rpl::PrimRef> prim_refs;  // leaf order: vertex ids, source hittable
  std::vector<double> vnrm;           // 3 per global vertex (mesh vertices concatenated)
  std::vector<double> vuv;            // 2 per global vertex
  std::vector<rpl::Material> materials;
  std::vector<rpl::Texture> textures;
  std::vector<uint32_t> texels;       // RGBA8 pool
  rpl::Emit background{};
  uint32_t root = 0;
  uint32_t max_depth = 0;             // deepest wide node (root = 0)
  uint32_t always_first = 0, n_always = 0;  // prims[always_first, +n_always): outside the tree, tested first
  uint64_t n_leaves = 0;
  double qbound = 0.0;  // rp_layout.h qbound: >= |o| and 255 s of every node frame (NODES_Q8, NODES_W8)
  size_t n_nodes() const {
    return node_format == rpl::NODES_W8 ? wnodes.size() : node_format == rpl::NODES_Q8 ? qnodes.size() : nodes.size();
  }
};

// The node format of RP_NODES_AUTO for the host SAH tree: the 64 B quantized node once the 128 B tree
// outgrows the caches (~2^21 hittables: ~1 M wide nodes, 130 MB of f32 nodes next to 170 MB of primitives
// against the 256 MB Infinity Cache), unless a coordinate exceeds the frames' range (rp_layout.h
// COORD_MAX).  Measured: C5, 10 M triangles, -6 % frame time; C3 (4 971 hittables) +0.4 %.
// The device LBVH keeps f32 (its tree has 3x fewer nodes: q8 +1.5 % on C5).  `amax`: the largest
// |coordinate| of the primitive boxes.
constexpr uint32_t Q8_MIN_PRIMS = 1u << 21;
inline uint32_t auto_node_format(uint32_t n_hittables, double amax) {
  return n_hittables >= Q8_MIN_PRIMS && amax <= rpl::COORD_MAX ? rpl::NODES_Q8 : rpl::NODES_F32;
}

// Checks every index the reference would bounds-check (or loop on).  Returns RP_OK or RP_EINVAL.
int validate(const rp_scene_desc* d, std::string& err);

// Builds the acceleration structure and the packed scene.  Assumes validate() passed.
int build(const rp_scene_desc* d, const BuildOptions& opt, PackedScene& out, std::string& err);

// Primitive records in hittable order (Prim, PrimRef with src = hittable id), their exact f64 boxes
// (hittable.rs:124-147; lo xyz, hi xyz) and the bounds of the box centroids: the device builder's input.
// A heap array without value-initialisation (PrimInput: 1.4 GB for 10 M triangles, filled in parallel)
template <class T>
struct RawArray {
  std::unique_ptr<T[]> p;
  size_t n = 0;
  void resize(size_t k) { p.reset(new T[k]); n = k; }
  size_t size() const { return n; }
  T* data() { return p.get(); }
  const T* data() const { return p.get(); }
  T& operator[](size_t i) { return p[i]; }
  const T& operator[](size_t i) const { return p[i]; }
};
struct PrimInput {
  RawArray<rpl::Prim> prims;
  RawArray<rpl::PrimRef> refs;
  RawArray<double> boxes;  // 6 per primitive
  double cmin[3], cmax[3];
  double amax;                // largest |coordinate| of the boxes (NaN ignored)
};
int prim_input(const rp_scene_desc* d, PrimInput& out, std::string& err);

// Structural self-check of a packed tree: every primitive referenced exactly once, every child box
// contains its subtree's primitive boxes, no cycles.  Returns RP_OK or RP_EINTERNAL (message in err).
int check(const PackedScene& s, std::string& err);

}  // namespace rpb

namespace rpg {

// A tree built on the device (rp_bvh_gpu.hip): device buffers in the rp_layout.h format, owned by the caller.
struct GpuTree {
  void* d_nodes = nullptr;  // rpl::Node4 or rpl::Node4Q by node_format; n_nodes used (capacity: one per primitive)
  uint32_t node_format = rpl::NODES_F32;
  rpl::Prim* d_prims = nullptr;   // leaf order
  rpl::PrimRef* d_prim_refs = nullptr;
  uint64_t n_nodes = 0, n_leaves = 0;
  uint32_t max_depth = 0;
  double qbound = 0.0;
};

// Device builds on the current device (>= 2 primitives), then the wide collapse: GPU_LBVH = Karras 2012 (Morton
// bits split), GPU_PLOC = Meister & Bittner 2018 (agglomerative, SAH quality).
enum { GPU_LBVH = 0, GPU_PLOC = 1 };
// cost_traverse: the SAH node cost relative to a primitive test (PLOC's leaf decisions; rp_scene_options).
// align: PLOC's depth-first node families start at multiples of this many nodes (pad slots zero; RP_LAYOUT_DFS_LINE).
int build_gpu(const rpb::PrimInput& in, uint32_t max_leaf, uint32_t node_format, uint32_t algo, double cost_traverse,
              uint32_t align, GpuTree& out, std::string& err);

}  // namespace rpg
