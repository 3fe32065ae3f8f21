// rp_bvh_gpu.hip -- acceleration-structure build on the device, for scenes whose
// host binned-SAH build (rp_bvh.cpp) would dominate setup (config C5: 10 M triangles).
//
// Replaces Bvh::new / make_bvh / split (bvh.rs:36-91) like the host builder does: the tree shape is not
// part of the contract, only the packed layout of rp_layout.h, which is identical, so
// the render and intersect kernels run unchanged.  Pipeline (Karras 2012 LBVH, then a wide collapse):
//   1. 30-bit Morton code of each primitive's box centroid, key = code << 32 | primitive (unique keys);
//   2. device radix sort of the keys (hipCUB);
//   3. one thread per inner node finds its key range and split (the binary radix tree of Karras 2012);
//   4. bottom-up f64 boxes: each leaf walks to the root, the second arrival at a node unions its
//      children's boxes (the exact min/max of AABB::union, utility.rs:130-135);
//   5. collapse into 4-wide nodes, one launch per level: a wide node takes its binary node's children
//      and opens the inner child of largest surface area until it has four (the host collapser's rule);
//      a subtree of <= max_leaf primitives -- a contiguous run of the sorted order -- becomes a leaf;
//   6. primitive records permuted into leaf (= sorted) order; child boxes rounded outward to f32.
#include <hip/hip_runtime.h>

#include <type_traits>
#include <hipcub/hipcub.hpp>

#include <string>
#include <vector>

#include "rp_bvh.h"

namespace rpg {

namespace {

constexpr uint32_t BIN_LEAF = 0x80000000u;  // binary child reference: leaf (sorted position) vs inner node

struct Box6 {
  double lo[3], hi[3];
};

__device__ __forceinline__ uint32_t expand_bits10(uint32_t v) {  // 10 bits -> every third bit of 30
  v = (v * 0x00010001u) & 0xFF0000FFu;
  v = (v * 0x00000101u) & 0x0F00F00Fu;
  v = (v * 0x00000011u) & 0xC30C30C3u;
  v = (v * 0x00000005u) & 0x49249249u;
  return v;
}

__global__ void morton_kernel(uint32_t n, const Box6* __restrict__ boxes, double3 cmin, double3 scale,
                              uint64_t* __restrict__ keys) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Box6 b = boxes[i];
  const double c[3] = {0.5 * (b.lo[0] + b.hi[0]), 0.5 * (b.lo[1] + b.hi[1]), 0.5 * (b.lo[2] + b.hi[2])};
  const double m[3] = {cmin.x, cmin.y, cmin.z}, s[3] = {scale.x, scale.y, scale.z};
  uint32_t code = 0;
  for (int k = 0; k < 3; k++) {
    double q = (c[k] - m[k]) * s[k];
    q = !(q >= 0.0) ? 0.0 : (q > 1023.0 ? 1023.0 : q);  // a NaN centroid (NaN geometry) sorts as 0
    code |= expand_bits10((uint32_t)q) << (2 - k);
  }
  keys[i] = ((uint64_t)code << 32) | i;
}

__device__ __forceinline__ uint64_t expand_bits21(uint64_t v) {  // 21 bits -> every third bit of 63
  v &= 0x1FFFFFull;
  v = (v | v << 32) & 0x1F00000000FFFFull;
  v = (v | v << 16) & 0x1F0000FF0000FFull;
  v = (v | v << 8) & 0x100F00F00F00F00Full;
  v = (v | v << 4) & 0x10C30C30C30C30C3ull;
  v = (v | v << 2) & 0x1249249249249249ull;
  return v;
}

// PLOC's order: 63-bit Morton codes (21 bits per axis; 10 M triangles share 30-bit codes ~10 to a cell), sorted
// with the primitive index as the value
__global__ void morton63_kernel(uint32_t n, const Box6* __restrict__ boxes, double3 cmin, double3 scale,
                                uint64_t* __restrict__ keys, uint32_t* __restrict__ idx) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Box6 b = boxes[i];
  const double c[3] = {0.5 * (b.lo[0] + b.hi[0]), 0.5 * (b.lo[1] + b.hi[1]), 0.5 * (b.lo[2] + b.hi[2])};
  const double m[3] = {cmin.x, cmin.y, cmin.z}, s[3] = {scale.x, scale.y, scale.z};
  uint64_t code = 0;
  for (int k = 0; k < 3; k++) {
    double q = (c[k] - m[k]) * s[k] * 2048.0;  // scale maps the centroid range to [0, 1024]
    q = !(q >= 0.0) ? 0.0 : (q > 2097151.0 ? 2097151.0 : q);  // NaN centroid -> 0
    code |= expand_bits21((uint64_t)q) << (2 - k);
  }
  keys[i] = code;
  idx[i] = i;
}

__device__ __forceinline__ int delta(const uint64_t* keys, uint32_t n, int i, int j) {
  if (j < 0 || j >= (int)n) return -1;
  return __clzll(keys[i] ^ keys[j]);  // keys are unique: < 64
}

// Karras 2012, Fig. 4: inner node i of n - 1.  Children are inner nodes or leaves (sorted positions).
__global__ void radix_tree_kernel(uint32_t n, const uint64_t* __restrict__ keys, uint32_t* __restrict__ left,
                                  uint32_t* __restrict__ right, uint32_t* __restrict__ parent_inner,
                                  uint32_t* __restrict__ parent_leaf, uint32_t* __restrict__ first,
                                  uint32_t* __restrict__ last) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int)n - 1) return;
  const int d = delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1) >= 0 ? 1 : -1;
  const int dmin = delta(keys, n, i, i - d);
  int lmax = 2;
  while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
  int l = 0;
  for (int t = lmax / 2; t >= 1; t /= 2)
    if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
  const int j = i + l * d;
  const int dnode = delta(keys, n, i, j);
  int s = 0;
  for (int div = 2;; div *= 2) {
    const int t = (l + div - 1) / div;
    if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    if (t <= 1) break;
  }
  const int g = i + s * d + (d < 0 ? -1 : 0);
  const int lo = i < j ? i : j, hi = i < j ? j : i;
  first[i] = (uint32_t)lo;
  last[i] = (uint32_t)hi;
  if (lo == g) {
    left[i] = BIN_LEAF | (uint32_t)g;
    parent_leaf[g] = (uint32_t)i;
  } else {
    left[i] = (uint32_t)g;
    parent_inner[g] = (uint32_t)i;
  }
  if (hi == g + 1) {
    right[i] = BIN_LEAF | (uint32_t)(g + 1);
    parent_leaf[g + 1] = (uint32_t)i;
  } else {
    right[i] = (uint32_t)(g + 1);
    parent_inner[g + 1] = (uint32_t)i;
  }
}

__device__ __forceinline__ double load_coherent(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ Box6 child_box(uint32_t c, const Box6* leaf_boxes, const uint32_t* order,
                                         const Box6* node_boxes) {
  Box6 b;
  if (c & BIN_LEAF) {
    b = leaf_boxes[order[c & ~BIN_LEAF]];  // written before the build: plain loads
  } else {
    const double* p = node_boxes[c].lo;  // written by another thread of this launch
    for (int k = 0; k < 3; k++) {
      b.lo[k] = load_coherent(p + k);
      b.hi[k] = load_coherent(p + 3 + k);
    }
  }
  return b;
}

// Bottom-up boxes: the second thread to reach an inner node computes it (the first stops there).
__global__ void boxes_kernel(uint32_t n, const Box6* __restrict__ leaf_boxes, const uint32_t* __restrict__ order,
                             const uint32_t* __restrict__ left, const uint32_t* __restrict__ right,
                             const uint32_t* __restrict__ parent_inner, const uint32_t* __restrict__ parent_leaf,
                             Box6* node_boxes, uint32_t* visits) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  uint32_t p = parent_leaf[k];
  for (;;) {
    __threadfence();
    if (atomicAdd(&visits[p], 1u) == 0u) return;
    __threadfence();
    const Box6 a = child_box(left[p], leaf_boxes, order, node_boxes);
    const Box6 b = child_box(right[p], leaf_boxes, order, node_boxes);
    Box6 u;
    for (int c = 0; c < 3; c++) {
      u.lo[c] = fmin(a.lo[c], b.lo[c]);
      u.hi[c] = fmax(a.hi[c], b.hi[c]);
    }
    double* q = node_boxes[p].lo;
    for (int c = 0; c < 3; c++) {
      __hip_atomic_store(q + c, u.lo[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(q + 3 + c, u.hi[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (p == 0) return;
    p = parent_inner[p];
  }
}

__device__ __forceinline__ double area(const Box6& b) {  // rp_bvh.cpp Box::area
  const double dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
  if (!(dx >= 0) || !(dy >= 0) || !(dz >= 0)) return 0.0;
  return 2.0 * (dx * dy + dy * dz + dz * dx);
}

struct Frontier {
  uint32_t bin;   // binary inner node
  uint32_t wide;  // its wide node
};

__device__ __forceinline__ uint32_t bin_count(uint32_t c, const uint32_t* first, const uint32_t* last) {
  return (c & BIN_LEAF) ? 1u : last[c] - first[c] + 1u;
}

// One level of the collapse: every frontier entry fills its wide node and appends its inner wide
// children to the next frontier.
template <uint32_t NF>
__global__ void collapse_kernel(const Frontier* __restrict__ cur, uint32_t n_cur, Frontier* __restrict__ next,
                                uint32_t* __restrict__ counters /* [0] wide nodes, [1] next frontier, [2] leaves */,
                                uint32_t max_leaf, const Box6* __restrict__ leaf_boxes,
                                const uint32_t* __restrict__ order, const uint32_t* __restrict__ left,
                                const uint32_t* __restrict__ right, const uint32_t* __restrict__ first,
                                const uint32_t* __restrict__ last, const Box6* __restrict__ node_boxes,
                                void* __restrict__ nodes) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_cur) return;
  const Frontier f = cur[t];
  uint32_t kids[4] = {left[f.bin], right[f.bin], 0u, 0u};
  uint32_t nk = 2;
  while (nk < 4) {
    int best = -1;
    double best_area = -1.0;
    for (uint32_t k = 0; k < nk; k++) {
      const uint32_t c = kids[k];
      if ((c & BIN_LEAF) || bin_count(c, first, last) <= max_leaf) continue;  // leaves are not opened
      const double a = area(node_boxes[c]);
      if (a > best_area) {
        best_area = a;
        best = (int)k;
      }
    }
    if (best < 0) break;
    const uint32_t open = kids[best];
    kids[best] = left[open];
    kids[nk++] = right[open];
  }
  Box6 kb[4];
  Box6 nb;
  for (int a = 0; a < 3; a++) {
    nb.lo[a] = __builtin_huge_val();
    nb.hi[a] = -__builtin_huge_val();
  }
  for (uint32_t k = 0; k < nk; k++) {
    const uint32_t c = kids[k];
    kb[k] = (c & BIN_LEAF) ? leaf_boxes[order[c & ~BIN_LEAF]] : node_boxes[c];
    for (int a = 0; a < 3; a++) {
      nb.lo[a] = fmin(nb.lo[a], kb[k].lo[a]);
      nb.hi[a] = fmax(nb.hi[a], kb[k].hi[a]);
    }
  }
  // child boxes in the node format: f32 rounded outward, or quantized in the node's frame (rp_layout.h
  // qframe; rp_bvh.cpp node_frame / Collapser)
  typedef typename std::conditional<NF == rpl::NODES_Q8, rpl::Node4Q, rpl::Node4>::type NodeT;
  NodeT nd;
  if constexpr (NF == rpl::NODES_Q8) {
    for (int a = 0; a < 3; a++) {
      const bool ok = isfinite(nb.lo[a]) && isfinite(nb.hi[a]) && nb.lo[a] <= nb.hi[a];
      rpl::qframe(ok ? nb.lo[a] : 0.0, ok ? nb.hi[a] : 0.0, nd.o[a], nd.s[a]);
    }
  } else {
    for (int k = 0; k < 4; k++) nd.pad[k] = 0;
  }
  // the inner children's wide nodes are allocated as one consecutive family (rp_bvh.cpp Collapser)
  uint32_t n_inner = 0;
  for (uint32_t k = 0; k < nk; k++) n_inner += bin_count(kids[k], first, last) > max_leaf;
  uint32_t fam = n_inner ? atomicAdd(&counters[0], n_inner) : 0u;
  for (uint32_t k = 0; k < 4; k++) {
    if (k >= nk) {
      if constexpr (NF == rpl::NODES_Q8) rpl::empty_child(nd, (int)k);
      else rpl::f32_empty(nd, (int)k);
      nd.child[k] = rpl::ENTRY_EMPTY;
      continue;
    }
    const uint32_t c = kids[k];
    if constexpr (NF == rpl::NODES_Q8) rpl::quantize_child(nd, (int)k, kb[k].lo, kb[k].hi);
    else rpl::f32_child(nd, (int)k, kb[k].lo, kb[k].hi);
    const uint32_t cnt = bin_count(c, first, last);
    if (cnt <= max_leaf) {
      const uint32_t lo = (c & BIN_LEAF) ? (c & ~BIN_LEAF) : first[c];
      nd.child[k] = rpl::ENTRY_LEAF | ((cnt - 1u) << rpl::LEAF_SHIFT) | lo;
      atomicAdd(&counters[2], 1u);
    } else {
      const uint32_t w = fam++;
      nd.child[k] = w;
      next[atomicAdd(&counters[1], 1u)] = Frontier{c, w};
    }
  }
  reinterpret_cast<NodeT*>(nodes)[f.wide] = nd;
}

__global__ void permute_kernel(uint32_t n, const uint32_t* __restrict__ order, const rpl::Prim* __restrict__ prims_in,
                               const rpl::PrimRef* __restrict__ refs_in, rpl::Prim* __restrict__ prims,
                               rpl::PrimRef* __restrict__ refs) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint32_t i = order[k];
  prims[k] = prims_in[i];
  refs[k] = refs_in[i];
}

__global__ void order_kernel(uint32_t n, const uint64_t* __restrict__ keys, uint32_t* __restrict__ order) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) order[k] = (uint32_t)keys[k];
}

unsigned grid(uint64_t n, unsigned block) { return (unsigned)((n + block - 1) / block); }

// ---------------------------------------------------------------------------------------------------------------
// Depth-first layout of a collapsed wide tree.  The level-by-level collapse numbers wide nodes by atomic family
// allocation, one level after another in no particular order, so a node and its children sit far apart; the host
// builder numbers them depth-first (a node's inner children as one consecutive family, each child's own subtree --
// its family first -- right behind the family, in child order), so a descent walks forward through memory.  The
// relayout: per level (the collapse's frontiers, recorded), bottom-up the number of wide nodes below each node, then
// top-down each node's new index and the start of its family, then every record copied to its new index with its
// inner child indices renamed.  Leaf entries and the primitive order are unchanged.  `align` (nodes): every family
// starts at a multiple of it -- 2 puts a 64-B quantized node's family on 128-B cache lines (RP_LAYOUT_DFS_LINE; the
// pad slots are zero and never referenced), 1 packs the families.
template <uint32_t NF>
__device__ __forceinline__ const uint32_t* node_children(const void* nodes, uint32_t i) {
  typedef typename std::conditional<NF == rpl::NODES_Q8, rpl::Node4Q, rpl::Node4>::type NodeT;
  return reinterpret_cast<const NodeT*>(nodes)[i].child;
}

__global__ void record_level_kernel(const uint32_t* __restrict__ wide_of, uint32_t stride_words, uint32_t n,
                                    uint32_t* __restrict__ ids) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) ids[i] = wide_of[(uint64_t)i * stride_words];
}

template <uint32_t NF>
__global__ void subtree_count_kernel(const uint32_t* __restrict__ ids, uint32_t n, const void* __restrict__ nodes,
                                     uint32_t align, uint32_t* __restrict__ below) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t u = ids[i];
  const uint32_t* ch = node_children<NF>(nodes, u);
  uint32_t f = 0, m = 0;
  for (int k = 0; k < 4; k++)
    if (!(ch[k] & rpl::ENTRY_LEAF)) {
      m++;
      f += below[ch[k]];
    }
  below[u] = f + (m + align - 1) / align * align;  // the family (padded) and the children's own subtrees
}

template <uint32_t NF>
__global__ void dfs_index_kernel(const uint32_t* __restrict__ ids, uint32_t n, const void* __restrict__ nodes,
                                 const uint32_t* __restrict__ below, uint32_t align, uint32_t* __restrict__ newid,
                                 uint32_t* __restrict__ fam) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t u = ids[i];
  const uint32_t* ch = node_children<NF>(nodes, u);
  uint32_t m = 0;
  for (int k = 0; k < 4; k++) m += !(ch[k] & rpl::ENTRY_LEAF);
  uint32_t slot = fam[u], next = fam[u] + (m + align - 1) / align * align;
  for (int k = 0; k < 4; k++) {
    const uint32_t c = ch[k];
    if (c & rpl::ENTRY_LEAF) continue;
    newid[c] = slot++;
    fam[c] = next;
    next += below[c];
  }
}

template <uint32_t NF>
__global__ void relayout_kernel(uint32_t n, const void* __restrict__ nodes, const uint32_t* __restrict__ newid,
                                void* __restrict__ out) {
  typedef typename std::conditional<NF == rpl::NODES_Q8, rpl::Node4Q, rpl::Node4>::type NodeT;
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= n) return;
  NodeT nd = reinterpret_cast<const NodeT*>(nodes)[u];
  for (int k = 0; k < 4; k++)
    if (!(nd.child[k] & rpl::ENTRY_LEAF)) nd.child[k] = newid[nd.child[k]];
  reinterpret_cast<NodeT*>(out)[newid[u]] = nd;
}

// Renumber the n_nodes wide nodes of `nodes` depth-first (see above); `level_ids` holds each collapse level's wide
// node ids (level k at level_off[k] .. level_off[k + 1]).  Replaces *nodes (the old buffer is freed).
int dfs_relayout(void** nodes, uint32_t node_format, uint64_t* n_nodes_io, const uint32_t* level_ids,
                 const std::vector<uint32_t>& level_off, uint32_t align, std::string& err) {
  const uint64_t n_nodes = *n_nodes_io;
  const size_t nb = node_format == rpl::NODES_Q8 ? sizeof(rpl::Node4Q) : sizeof(rpl::Node4);
  uint32_t *below = nullptr, *newid = nullptr, *fam = nullptr;
  void* out = nullptr;
  hipError_t e = hipMalloc((void**)&below, sizeof(uint32_t) * n_nodes);
  if (e == hipSuccess) e = hipMalloc((void**)&newid, sizeof(uint32_t) * n_nodes);
  if (e == hipSuccess) e = hipMalloc((void**)&fam, sizeof(uint32_t) * n_nodes);
  const unsigned B = 256;
  const uint32_t L = (uint32_t)level_off.size() - 1;
  for (uint32_t k = L; k-- > 0 && e == hipSuccess;) {
    const uint32_t n = level_off[k + 1] - level_off[k];
    if (node_format == rpl::NODES_Q8)
      hipLaunchKernelGGL(subtree_count_kernel<rpl::NODES_Q8>, dim3(grid(n, B)), dim3(B), 0, nullptr, level_ids + level_off[k],
                         n, *nodes, align, below);
    else
      hipLaunchKernelGGL(subtree_count_kernel<rpl::NODES_F32>, dim3(grid(n, B)), dim3(B), 0, nullptr, level_ids + level_off[k],
                         n, *nodes, align, below);
    e = hipGetLastError();
  }
  const uint32_t root_new = 0, root_fam = align;  // the root, padded to the alignment, then its family
  uint32_t root = 0, below_root = 0;
  if (e == hipSuccess) e = hipMemcpy(&root, level_ids, sizeof root, hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(&below_root, below + root, sizeof below_root, hipMemcpyDeviceToHost);
  const uint64_t total = (uint64_t)root_fam + below_root;  // == n_nodes when align == 1
  if (e == hipSuccess) e = hipMalloc(&out, nb * total);
  if (e == hipSuccess && total != n_nodes) e = hipMemset(out, 0, nb * total);
  if (e == hipSuccess) e = hipMemcpy(newid + root, &root_new, sizeof root_new, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(fam + root, &root_fam, sizeof root_fam, hipMemcpyHostToDevice);
  for (uint32_t k = 0; k < L && e == hipSuccess; k++) {
    const uint32_t n = level_off[k + 1] - level_off[k];
    if (node_format == rpl::NODES_Q8)
      hipLaunchKernelGGL(dfs_index_kernel<rpl::NODES_Q8>, dim3(grid(n, B)), dim3(B), 0, nullptr, level_ids + level_off[k], n,
                         *nodes, below, align, newid, fam);
    else
      hipLaunchKernelGGL(dfs_index_kernel<rpl::NODES_F32>, dim3(grid(n, B)), dim3(B), 0, nullptr, level_ids + level_off[k], n,
                         *nodes, below, align, newid, fam);
    e = hipGetLastError();
  }
  if (e == hipSuccess) {
    if (node_format == rpl::NODES_Q8)
      hipLaunchKernelGGL(relayout_kernel<rpl::NODES_Q8>, dim3(grid(n_nodes, B)), dim3(B), 0, nullptr, (uint32_t)n_nodes, *nodes,
                         newid, out);
    else
      hipLaunchKernelGGL(relayout_kernel<rpl::NODES_F32>, dim3(grid(n_nodes, B)), dim3(B), 0, nullptr, (uint32_t)n_nodes, *nodes,
                         newid, out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipDeviceSynchronize();
  for (void* p : {(void*)below, (void*)newid, (void*)fam}) if (p) (void)hipFree(p);
  if (e != hipSuccess) {
    if (out) (void)hipFree(out);
    err = std::string("depth-first relayout: ") + hipGetErrorString(e);
    return RP_EHIP;
  }
  (void)hipFree(*nodes);
  *nodes = out;
  *n_nodes_io = total;
  return RP_OK;
}

// ---------------------------------------------------------------------------------------------------------------
// PLOC (Meister & Bittner 2018, "Parallel Locally-Ordered Clustering for Bounding Volume Hierarchy Construction"):
// the primitives in Morton order are the initial clusters; every round, each cluster finds its nearest neighbour
// within PLOC_R positions of the (Morton-ordered) cluster array under the SAH distance -- the surface area of the
// union of the two boxes -- and mutual nearest neighbours merge into a new binary node (at the lower position;
// the higher one is removed and the array compacted, order kept).  Agglomerative like a sweep-SAH build, so the
// tree is of SAH quality where the LBVH above splits by Morton bits.  Deterministic: distances tie-break on the
// pair's positions, merges take node ids from a prefix sum.
// Search radius: measured on C5's 10 M random triangles (32-spp frame over the q8 tree; host SAH tree 229.5 ms):
// r = 1: 234.1, 2: 233.2, 3: 232.8, 4: 235.4, 6: 240.9, 8: 258.7, 16: 255.3, 32: 300.8, 64: 312.1 ms.  (The paper's
// r = 16 merges more distant Morton neighbours early, which here makes deeper, costlier trees.)
constexpr int PLOC_R = 3;
constexpr int PLOC_B = 256;

struct PNode {
  uint32_t left, right, size, leaf;  // children (BIN_LEAF | primitive, or a node id); primitives below; 1 = the
                                     // subtree becomes one leaf of the wide tree (the SAH decision, ploc_apply)
};

__device__ __forceinline__ Box6 box_union(const Box6& a, const Box6& b) {
  Box6 u;
  for (int c = 0; c < 3; c++) {
    u.lo[c] = fmin(a.lo[c], b.lo[c]);
    u.hi[c] = fmax(a.hi[c], b.hi[c]);
  }
  return u;
}

__global__ void ploc_init_kernel(uint32_t n, const uint32_t* __restrict__ order, const Box6* __restrict__ boxes,
                                 uint32_t* __restrict__ ref, Box6* __restrict__ cbox, uint32_t* __restrict__ csize,
                                 double* __restrict__ ccost) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t p = order[i];
  ref[i] = BIN_LEAF | p;
  cbox[i] = boxes[p];
  csize[i] = 1u;
  ccost[i] = 1.0;  // one primitive test
}

// nearest neighbour of every cluster within PLOC_R positions: the boxes of the block's window in LDS
__global__ void __launch_bounds__(PLOC_B) ploc_nn_kernel(uint32_t m, const Box6* __restrict__ cbox, uint32_t* __restrict__ nn) {
  __shared__ Box6 win[PLOC_B + 2 * PLOC_R];
  const int base = (int)(blockIdx.x * PLOC_B) - PLOC_R;
  for (int t = threadIdx.x; t < PLOC_B + 2 * PLOC_R; t += PLOC_B) {
    const int g = base + t;
    if (g >= 0 && g < (int)m) win[t] = cbox[g];
  }
  __syncthreads();
  const int i = (int)(blockIdx.x * PLOC_B + threadIdx.x);
  if (i >= (int)m) return;
  const Box6 a = win[threadIdx.x + PLOC_R];
  double best = __builtin_huge_val();
  int bj = -1;
  const int lo = max(0, i - PLOC_R), hi = min((int)m - 1, i + PLOC_R);
  for (int j = lo; j <= hi; j++) {
    if (j == i) continue;
    double d = area(box_union(a, win[j - base]));
    if (d != d) d = __builtin_huge_val();
    // strict order on (distance, lower position, higher position): the global minimum pair is mutual, so every
    // round merges at least one pair; candidates are scanned in increasing j, so `<` keeps the smaller j on ties.
    // A NaN distance (NaN geometry: fmin/fmax keep a NaN when both operands are NaN) ranks as +inf, and a cluster
    // with no finite candidate takes its first one (if no pair is finite, clusters 0 and 1 pair up, so the round
    // still merges) -- never the -1 that ploc_flags_kernel would index with.
    if (d < best || bj < 0) {
      best = d;
      bj = j;
    }
  }
  nn[i] = (uint32_t)bj;
}

// flags: keep[i] (the cluster survives at its position: not merged, or the lower of a mutual pair) and merge[i]
__global__ void ploc_flags_kernel(uint32_t m, const uint32_t* __restrict__ nn, uint32_t* __restrict__ keep,
                                  uint32_t* __restrict__ merge) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const uint32_t j = nn[i];
  const bool mutual = j < m && nn[j] == i;
  keep[i] = (!mutual || i < j) ? 1u : 0u;
  merge[i] = (mutual && i < j) ? 1u : 0u;
}

__global__ void ploc_apply_kernel(uint32_t m, const uint32_t* __restrict__ nn, const uint32_t* __restrict__ keep,
                                  const uint32_t* __restrict__ kpos, const uint32_t* __restrict__ merge,
                                  const uint32_t* __restrict__ mrank, uint32_t node_base, const uint32_t* __restrict__ ref,
                                  const Box6* __restrict__ cbox, const uint32_t* __restrict__ csize,
                                  const double* __restrict__ ccost, uint32_t* __restrict__ ref2, Box6* __restrict__ cbox2,
                                  uint32_t* __restrict__ csize2, double* __restrict__ ccost2, PNode* __restrict__ nodes,
                                  Box6* __restrict__ nbox, uint32_t max_leaf, double cost_traverse) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m || !keep[i]) return;
  const uint32_t o = kpos[i];
  if (merge[i]) {
    const uint32_t j = nn[i], id = node_base + mrank[i];
    const Box6 u = box_union(cbox[i], cbox[j]);
    const uint32_t sz = csize[i] + csize[j];
    // SAH, bottom-up (the expected primitive-test cost of a ray entering the box, node visits at cost_traverse):
    // a subtree of <= max_leaf primitives becomes one leaf when testing them all is cheaper than splitting
    const double au = area(u);
    const double split = cost_traverse + (au > 0.0 ? (area(cbox[i]) * ccost[i] + area(cbox[j]) * ccost[j]) / au
                                                    : 0.5 * (ccost[i] + ccost[j]));
    const bool leaf = sz <= max_leaf && (double)sz <= split;
    PNode nd;
    nd.left = ref[i];
    nd.right = ref[j];
    nd.size = sz;
    nd.leaf = leaf ? 1u : 0u;
    nodes[id] = nd;
    nbox[id] = u;
    ref2[o] = id;
    cbox2[o] = u;
    csize2[o] = sz;
    ccost2[o] = leaf ? (double)sz : split;
  } else {
    ref2[o] = ref[i];
    cbox2[o] = cbox[i];
    csize2[o] = csize[i];
    ccost2[o] = ccost[i];
  }
}

struct PFront {
  uint32_t bin, wide, poff;  // binary node, its wide node, the first primitive slot of its subtree
};

__device__ __forceinline__ uint32_t psize(uint32_t c, const PNode* nodes) { return (c & BIN_LEAF) ? 1u : nodes[c].size; }
__device__ __forceinline__ bool pleaf(uint32_t c, const PNode* nodes) { return (c & BIN_LEAF) || nodes[c].leaf; }

// One level of the collapse of the PLOC tree (collapse_kernel's rule: open the inner child of largest area until four
// children); primitives are laid out depth-first as the frontier descends: each child subtree takes the next run of
// primitive slots, and a leaf child (<= max_leaf primitives) writes its primitives' ids into perm there.
template <uint32_t NF>
__global__ void ploc_collapse_kernel(const PFront* __restrict__ cur, uint32_t n_cur, PFront* __restrict__ next,
                                     uint32_t* __restrict__ counters /* [0] wide nodes, [1] next frontier, [2] leaves */,
                                     uint32_t max_leaf, const Box6* __restrict__ prim_boxes,
                                     const PNode* __restrict__ bnodes, const Box6* __restrict__ nbox,
                                     uint32_t* __restrict__ perm, void* __restrict__ nodes) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_cur) return;
  const PFront f = cur[t];
  uint32_t kids[4] = {bnodes[f.bin].left, bnodes[f.bin].right, 0u, 0u};
  uint32_t nk = 2;
  while (nk < 4) {
    int best = -1;
    double best_area = -1.0;
    for (uint32_t k = 0; k < nk; k++) {
      const uint32_t c = kids[k];
      if (pleaf(c, bnodes)) continue;
      const double a = area(nbox[c]);
      if (a > best_area) {
        best_area = a;
        best = (int)k;
      }
    }
    if (best < 0) break;
    const uint32_t open = kids[best];
    kids[best] = bnodes[open].left;
    kids[nk++] = bnodes[open].right;
  }
  Box6 kb[4];
  Box6 nb;
  for (int a = 0; a < 3; a++) {
    nb.lo[a] = __builtin_huge_val();
    nb.hi[a] = -__builtin_huge_val();
  }
  for (uint32_t k = 0; k < nk; k++) {
    const uint32_t c = kids[k];
    kb[k] = (c & BIN_LEAF) ? prim_boxes[c & ~BIN_LEAF] : nbox[c];
    nb = box_union(nb, kb[k]);
  }
  typedef typename std::conditional<NF == rpl::NODES_Q8, rpl::Node4Q, rpl::Node4>::type NodeT;
  NodeT nd;
  if constexpr (NF == rpl::NODES_Q8) {
    for (int a = 0; a < 3; a++) {
      const bool ok = isfinite(nb.lo[a]) && isfinite(nb.hi[a]) && nb.lo[a] <= nb.hi[a];
      rpl::qframe(ok ? nb.lo[a] : 0.0, ok ? nb.hi[a] : 0.0, nd.o[a], nd.s[a]);
    }
  } else {
    for (int k = 0; k < 4; k++) nd.pad[k] = 0;
  }
  uint32_t n_inner = 0;
  for (uint32_t k = 0; k < nk; k++) n_inner += !pleaf(kids[k], bnodes);
  uint32_t fam = n_inner ? atomicAdd(&counters[0], n_inner) : 0u;
  uint32_t off = f.poff;
  for (uint32_t k = 0; k < 4; k++) {
    if (k >= nk) {
      if constexpr (NF == rpl::NODES_Q8) rpl::empty_child(nd, (int)k);
      else rpl::f32_empty(nd, (int)k);
      nd.child[k] = rpl::ENTRY_EMPTY;
      continue;
    }
    const uint32_t c = kids[k];
    if constexpr (NF == rpl::NODES_Q8) rpl::quantize_child(nd, (int)k, kb[k].lo, kb[k].hi);
    else rpl::f32_child(nd, (int)k, kb[k].lo, kb[k].hi);
    const uint32_t cnt = psize(c, bnodes);
    if (pleaf(c, bnodes)) {
      nd.child[k] = rpl::ENTRY_LEAF | ((cnt - 1u) << rpl::LEAF_SHIFT) | off;
      // the subtree's primitives (<= max_leaf <= 8: a binary subtree of <= 7 inner nodes) into perm[off ...]
      uint32_t stk[8], sp = 0, w = off;
      stk[sp++] = c;
      while (sp) {
        const uint32_t x = stk[--sp];
        if (x & BIN_LEAF) {
          perm[w++] = x & ~BIN_LEAF;
        } else {
          stk[sp++] = bnodes[x].right;
          stk[sp++] = bnodes[x].left;
        }
      }
      atomicAdd(&counters[2], 1u);
    } else {
      const uint32_t wn = fam++;
      nd.child[k] = wn;
      next[atomicAdd(&counters[1], 1u)] = PFront{c, wn, off};
    }
    off += cnt;
  }
  reinterpret_cast<NodeT*>(nodes)[f.wide] = nd;
}

}  // namespace

namespace {

// PLOC build (see the kernels above) from the Morton-sorted keys, then the depth-first collapse; fills out.d_nodes
// and out.d_prims / d_prim_refs (permuted).  Device buffers: boxes / prims_in / refs_in in hittable order.
int build_ploc(uint32_t n, const uint32_t* d_order, const Box6* d_boxes, const rpl::Prim* d_prims_in,
               const rpl::PrimRef* d_refs_in, uint32_t max_leaf, double cost_traverse, uint32_t node_format, uint32_t align,
               GpuTree& out, std::string& err) {
  std::vector<void*> tmp;
  hipError_t e = hipSuccess;
  auto alloc = [&](void** p, size_t bytes) {
    if (e != hipSuccess) return;
    e = hipMalloc(p, bytes);
    if (e == hipSuccess) tmp.push_back(*p);
    else *p = nullptr;
  };
  uint32_t *ref[2] = {nullptr, nullptr}, *csz[2] = {nullptr, nullptr};
  Box6* cbox[2] = {nullptr, nullptr};
  double* ccost[2] = {nullptr, nullptr};
  uint32_t *d_nn = nullptr, *d_keep = nullptr, *d_kpos = nullptr, *d_merge = nullptr, *d_mrank = nullptr;
  uint32_t *d_perm = nullptr, *d_ctr = nullptr;
  PNode* d_bn = nullptr;
  Box6* d_nbox = nullptr;
  PFront *d_fa = nullptr, *d_fb = nullptr;
  for (int b = 0; b < 2; b++) {
    alloc((void**)&ref[b], sizeof(uint32_t) * n);
    alloc((void**)&csz[b], sizeof(uint32_t) * n);
    alloc((void**)&cbox[b], sizeof(Box6) * n);
    alloc((void**)&ccost[b], sizeof(double) * n);
  }
  alloc((void**)&d_nn, sizeof(uint32_t) * n);
  alloc((void**)&d_keep, sizeof(uint32_t) * n);
  alloc((void**)&d_kpos, sizeof(uint32_t) * n);
  alloc((void**)&d_merge, sizeof(uint32_t) * n);
  alloc((void**)&d_mrank, sizeof(uint32_t) * n);
  alloc((void**)&d_perm, sizeof(uint32_t) * n);
  alloc((void**)&d_ctr, sizeof(uint32_t) * 4);
  alloc((void**)&d_bn, sizeof(PNode) * n);
  alloc((void**)&d_nbox, sizeof(Box6) * n);
  alloc((void**)&d_fa, sizeof(PFront) * n);
  alloc((void**)&d_fb, sizeof(PFront) * n);
  size_t scan_bytes = 0;
  void* d_scan = nullptr;
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, d_keep, d_kpos, (int)n);
  alloc(&d_scan, scan_bytes);
  auto done = [&](int code, const std::string& msg) {
    for (void* p : tmp) (void)hipFree(p);
    if (code != RP_OK) err = msg;
    return code;
  };
  if (e != hipSuccess) return done(RP_ENOMEM, std::string("hipMalloc (PLOC build): ") + hipGetErrorString(e));
#define RPG_CHECK2(what)                                                                         \
  do {                                                                                           \
    if (e == hipSuccess) e = hipGetLastError();                                                  \
    if (e != hipSuccess) return done(RP_EHIP, std::string(what) + ": " + hipGetErrorString(e));  \
  } while (0)
  const unsigned B = 256;
  hipLaunchKernelGGL(ploc_init_kernel, dim3(grid(n, B)), dim3(B), 0, nullptr, n, d_order, d_boxes, ref[0], cbox[0],
                     csz[0], ccost[0]);
  RPG_CHECK2("PLOC init");
  uint32_t m = n, node_base = 0;
  int cb = 0;
  while (m > 1) {
    hipLaunchKernelGGL(ploc_nn_kernel, dim3(grid(m, PLOC_B)), dim3(PLOC_B), 0, nullptr, m, cbox[cb], d_nn);
    hipLaunchKernelGGL(ploc_flags_kernel, dim3(grid(m, B)), dim3(B), 0, nullptr, m, d_nn, d_keep, d_merge);
    RPG_CHECK2("PLOC neighbours");
    e = hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_keep, d_kpos, (int)m);
    if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(d_scan, scan_bytes, d_merge, d_mrank, (int)m);
    uint32_t last[4];
    if (e == hipSuccess) e = hipMemcpy(&last[0], d_kpos + (m - 1), 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(&last[1], d_keep + (m - 1), 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(&last[2], d_mrank + (m - 1), 4, hipMemcpyDeviceToHost);
    if (e == hipSuccess) e = hipMemcpy(&last[3], d_merge + (m - 1), 4, hipMemcpyDeviceToHost);
    RPG_CHECK2("PLOC scan");
    const uint32_t m2 = last[0] + last[1], merges = last[2] + last[3];
    if (merges == 0 || m2 != m - merges) return done(RP_EINTERNAL, "PLOC build: no progress");
    hipLaunchKernelGGL(ploc_apply_kernel, dim3(grid(m, B)), dim3(B), 0, nullptr, m, d_nn, d_keep, d_kpos, d_merge, d_mrank,
                       node_base, ref[cb], cbox[cb], csz[cb], ccost[cb], ref[1 - cb], cbox[1 - cb], csz[1 - cb],
                       ccost[1 - cb], d_bn, d_nbox, max_leaf, cost_traverse);
    RPG_CHECK2("PLOC merge");
    node_base += merges;
    m = m2;
    cb = 1 - cb;
  }
  if (node_base != n - 1) return done(RP_EINTERNAL, "PLOC build: node count");
  uint32_t* d_levels = nullptr;  // every collapse level's wide node ids (the depth-first relayout)
  alloc((void**)&d_levels, sizeof(uint32_t) * n);
  if (e != hipSuccess) return done(RP_ENOMEM, std::string("hipMalloc (PLOC build): ") + hipGetErrorString(e));
  std::vector<uint32_t> level_off{0};
  // collapse from the root (the last node made) into wide node 0, primitives from slot 0
  const PFront root{n - 2, 0u, 0u};
  const uint32_t ctr0[4] = {1u, 0u, 0u, 0u};
  e = hipMemcpy(d_fa, &root, sizeof root, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_ctr, ctr0, sizeof ctr0, hipMemcpyHostToDevice);
  RPG_CHECK2("PLOC collapse setup");
  uint32_t n_cur = 1, depth = 0;
  for (;;) {
    e = hipMemset(d_ctr + 1, 0, sizeof(uint32_t));
    RPG_CHECK2("PLOC collapse");
    hipLaunchKernelGGL(record_level_kernel, dim3(grid(n_cur, B)), dim3(B), 0, nullptr, &d_fa->wide,
                       (uint32_t)(sizeof(PFront) / 4), n_cur, d_levels + level_off.back());
    level_off.push_back(level_off.back() + n_cur);
    if (node_format == rpl::NODES_Q8)
      hipLaunchKernelGGL(ploc_collapse_kernel<rpl::NODES_Q8>, dim3(grid(n_cur, B)), dim3(B), 0, nullptr, d_fa, n_cur, d_fb,
                         d_ctr, max_leaf, d_boxes, d_bn, d_nbox, d_perm, out.d_nodes);
    else
      hipLaunchKernelGGL(ploc_collapse_kernel<rpl::NODES_F32>, dim3(grid(n_cur, B)), dim3(B), 0, nullptr, d_fa, n_cur, d_fb,
                         d_ctr, max_leaf, d_boxes, d_bn, d_nbox, d_perm, out.d_nodes);
    RPG_CHECK2("PLOC collapse");
    uint32_t ctr[4];
    e = hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost);
    RPG_CHECK2("PLOC collapse");
    if (ctr[0] > n) return done(RP_EINTERNAL, "PLOC build: wide node overflow");
    if (ctr[1] == 0) {
      out.n_nodes = ctr[0];
      out.n_leaves = ctr[2];
      break;
    }
    depth++;
    n_cur = ctr[1];
    std::swap(d_fa, d_fb);
  }
  out.max_depth = depth;
  {
    std::string rerr;
    const int rc = dfs_relayout(&out.d_nodes, node_format, &out.n_nodes, d_levels, level_off, align, rerr);
    if (rc) return done(rc, rerr);
  }
  hipLaunchKernelGGL(permute_kernel, dim3(grid(n, B)), dim3(B), 0, nullptr, n, d_perm, d_prims_in, d_refs_in, out.d_prims,
                     out.d_prim_refs);
  RPG_CHECK2("PLOC permute");
  e = hipDeviceSynchronize();
  RPG_CHECK2("PLOC build");
#undef RPG_CHECK2
  return done(RP_OK, "");
}

}  // namespace

// Temporaries are freed on every path; on success the caller owns out.d_nodes / d_prims / d_prim_refs.
int build_gpu(const rpb::PrimInput& in, uint32_t max_leaf, uint32_t node_format, uint32_t algo, double cost_traverse,
              uint32_t align, GpuTree& out, std::string& err) {
  out = GpuTree{};
  const uint32_t n = (uint32_t)in.prims.size();
  if (n < 2) {
    err = "device BVH build needs at least 2 primitives";
    return RP_EINVAL;
  }
  if (node_format != rpl::NODES_F32 && node_format != rpl::NODES_Q8) {
    err = "unknown node format";
    return RP_EINVAL;
  }
  if (node_format == rpl::NODES_Q8 && !(in.amax <= rpl::COORD_MAX)) {
    err = "primitive coordinates beyond +-2^54 (or infinite) are not supported by the quantized nodes";
    return RP_EINVAL;
  }
  if (max_leaf < 1 || max_leaf > rpl::LEAF_MAX) {
    err = "max_leaf out of range";
    return RP_EINVAL;
  }
  std::vector<void*> tmp;
  hipError_t e = hipSuccess;
  auto alloc = [&](void** p, size_t bytes) {
    if (e != hipSuccess) return;
    e = hipMalloc(p, bytes);
    if (e == hipSuccess) tmp.push_back(*p);
    else *p = nullptr;
  };
  Box6* d_boxes = nullptr;
  rpl::Prim* d_prims_in = nullptr;
  rpl::PrimRef* d_refs_in = nullptr;
  uint64_t *d_keys = nullptr, *d_keys_sorted = nullptr;
  uint32_t *d_order = nullptr, *d_left = nullptr, *d_right = nullptr, *d_pin = nullptr, *d_pleaf = nullptr;
  uint32_t *d_first = nullptr, *d_last = nullptr, *d_visits = nullptr, *d_ctr = nullptr;
  Box6* d_nboxes = nullptr;
  Frontier *d_fa = nullptr, *d_fb = nullptr;
  alloc((void**)&d_boxes, sizeof(Box6) * n);
  alloc((void**)&d_prims_in, sizeof(rpl::Prim) * n);
  alloc((void**)&d_refs_in, sizeof(rpl::PrimRef) * n);
  alloc((void**)&d_keys, sizeof(uint64_t) * n);
  alloc((void**)&d_keys_sorted, sizeof(uint64_t) * n);
  alloc((void**)&d_order, sizeof(uint32_t) * n);
  alloc((void**)&d_left, sizeof(uint32_t) * n);
  alloc((void**)&d_right, sizeof(uint32_t) * n);
  alloc((void**)&d_pin, sizeof(uint32_t) * n);
  alloc((void**)&d_pleaf, sizeof(uint32_t) * n);
  alloc((void**)&d_first, sizeof(uint32_t) * n);
  alloc((void**)&d_last, sizeof(uint32_t) * n);
  alloc((void**)&d_visits, sizeof(uint32_t) * n);
  alloc((void**)&d_ctr, sizeof(uint32_t) * 4);
  alloc((void**)&d_nboxes, sizeof(Box6) * n);
  alloc((void**)&d_fa, sizeof(Frontier) * n);
  alloc((void**)&d_fb, sizeof(Frontier) * n);
  // outputs: at most n - 1 wide nodes (each inner wide node has >= 2 children)
  const size_t node_bytes = node_format == rpl::NODES_Q8 ? sizeof(rpl::Node4Q) : sizeof(rpl::Node4);
  if (e == hipSuccess) e = hipMalloc(&out.d_nodes, node_bytes * n);
  if (e == hipSuccess) e = hipMalloc((void**)&out.d_prims, sizeof(rpl::Prim) * n);
  if (e == hipSuccess) e = hipMalloc((void**)&out.d_prim_refs, sizeof(rpl::PrimRef) * n);
  void* d_sort_tmp = nullptr;
  size_t sort_bytes = 0;
  auto cleanup = [&](int code, const std::string& msg) {
    for (void* p : tmp) (void)hipFree(p);
    if (d_sort_tmp) (void)hipFree(d_sort_tmp);
    if (code != RP_OK) {
      if (out.d_nodes) (void)hipFree(out.d_nodes);
      if (out.d_prims) (void)hipFree(out.d_prims);
      if (out.d_prim_refs) (void)hipFree(out.d_prim_refs);
      out = GpuTree{};
      err = msg;
    }
    return code;
  };
  if (e != hipSuccess) return cleanup(RP_ENOMEM, std::string("hipMalloc (device BVH build): ") + hipGetErrorString(e));
#define RPG_CHECK(what)                                                                              \
  do {                                                                                               \
    e = hipGetLastError();                                                                           \
    if (e != hipSuccess) return cleanup(RP_EHIP, std::string(what) + ": " + hipGetErrorString(e));   \
  } while (0)
  e = hipMemcpy(d_boxes, in.boxes.data(), sizeof(Box6) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_prims_in, in.prims.data(), sizeof(rpl::Prim) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_refs_in, in.refs.data(), sizeof(rpl::PrimRef) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemset(d_visits, 0, sizeof(uint32_t) * n);
  if (e == hipSuccess) e = hipMemset(d_ctr, 0, sizeof(uint32_t) * 4);
  if (e != hipSuccess) return cleanup(RP_EHIP, std::string("upload (device BVH build): ") + hipGetErrorString(e));

  const unsigned B = 256;
  double3 cmin = make_double3(in.cmin[0], in.cmin[1], in.cmin[2]);
  double sc[3];
  for (int k = 0; k < 3; k++) {
    const double ext = in.cmax[k] - in.cmin[k];
    sc[k] = ext > 0.0 ? 1024.0 / ext : 0.0;
  }
  if (algo == GPU_PLOC) {
    hipLaunchKernelGGL(morton63_kernel, dim3(grid(n, B)), dim3(B), 0, nullptr, n, d_boxes, cmin,
                       make_double3(sc[0], sc[1], sc[2]), d_keys, d_left);
    RPG_CHECK("morton");
    e = hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, d_keys, d_keys_sorted, d_left, d_order, (int)n, 0, 63);
    if (e == hipSuccess) e = hipMalloc(&d_sort_tmp, sort_bytes);
    if (e == hipSuccess)
      e = hipcub::DeviceRadixSort::SortPairs(d_sort_tmp, sort_bytes, d_keys, d_keys_sorted, d_left, d_order, (int)n, 0, 63);
    if (e != hipSuccess) return cleanup(RP_EHIP, std::string("radix sort: ") + hipGetErrorString(e));
    out.node_format = node_format;
    out.qbound = rpl::qbound(in.amax);
    std::string perr;
    const int rc = build_ploc(n, d_order, d_boxes, d_prims_in, d_refs_in, max_leaf, cost_traverse, node_format,
                                std::max(1u, align), out, perr);
    return cleanup(rc, perr);
  }
  hipLaunchKernelGGL(morton_kernel, dim3(grid(n, B)), dim3(B), 0, nullptr, n, d_boxes, cmin,
                     make_double3(sc[0], sc[1], sc[2]), d_keys);
  RPG_CHECK("morton");
  e = hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, d_keys, d_keys_sorted, (int)n, 0, 62);
  if (e == hipSuccess) e = hipMalloc(&d_sort_tmp, sort_bytes);
  if (e == hipSuccess) e = hipcub::DeviceRadixSort::SortKeys(d_sort_tmp, sort_bytes, d_keys, d_keys_sorted, (int)n, 0, 62);
  if (e != hipSuccess) return cleanup(RP_EHIP, std::string("radix sort: ") + hipGetErrorString(e));
  hipLaunchKernelGGL(order_kernel, dim3(grid(n, B)), dim3(B), 0, nullptr, n, d_keys_sorted, d_order);
  RPG_CHECK("order");
  hipLaunchKernelGGL(radix_tree_kernel, dim3(grid(n - 1, B)), dim3(B), 0, nullptr, n, d_keys_sorted, d_left, d_right,
                     d_pin, d_pleaf, d_first, d_last);
  RPG_CHECK("radix tree");
  hipLaunchKernelGGL(boxes_kernel, dim3(grid(n, B)), dim3(B), 0, nullptr, n, d_boxes, d_order, d_left, d_right,
                     d_pin, d_pleaf, d_nboxes, d_visits);
  RPG_CHECK("boxes");
  // collapse, level by level from the root (binary inner node 0 -> wide node 0)
  const Frontier root{0u, 0u};
  const uint32_t one = 1u;
  e = hipMemcpy(d_fa, &root, sizeof root, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_ctr, &one, sizeof one, hipMemcpyHostToDevice);  // wide node 0 taken
  if (e != hipSuccess) return cleanup(RP_EHIP, std::string("collapse setup: ") + hipGetErrorString(e));
  uint32_t n_cur = 1, depth = 0;
  for (;;) {
    e = hipMemset(d_ctr + 1, 0, sizeof(uint32_t));
    if (e != hipSuccess) return cleanup(RP_EHIP, std::string("collapse: ") + hipGetErrorString(e));
    if (node_format == rpl::NODES_Q8)
      hipLaunchKernelGGL(collapse_kernel<rpl::NODES_Q8>, dim3(grid(n_cur, B)), dim3(B), 0, nullptr, d_fa, n_cur, d_fb,
                         d_ctr, max_leaf, d_boxes, d_order, d_left, d_right, d_first, d_last, d_nboxes, out.d_nodes);
    else
      hipLaunchKernelGGL(collapse_kernel<rpl::NODES_F32>, dim3(grid(n_cur, B)), dim3(B), 0, nullptr, d_fa, n_cur, d_fb,
                         d_ctr, max_leaf, d_boxes, d_order, d_left, d_right, d_first, d_last, d_nboxes, out.d_nodes);
    RPG_CHECK("collapse");
    uint32_t ctr[4];
    e = hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return cleanup(RP_EHIP, std::string("collapse: ") + hipGetErrorString(e));
    if (ctr[0] > n) return cleanup(RP_EINTERNAL, "device BVH build: wide node overflow");
    if (ctr[1] == 0) {
      out.n_nodes = ctr[0];
      out.n_leaves = ctr[2];
      break;
    }
    depth++;
    n_cur = ctr[1];
    std::swap(d_fa, d_fb);
  }
  out.max_depth = depth;
  out.node_format = node_format;
  out.qbound = rpl::qbound(in.amax);
  hipLaunchKernelGGL(permute_kernel, dim3(grid(n, B)), dim3(B), 0, nullptr, n, d_order, d_prims_in, d_refs_in,
                     out.d_prims, out.d_prim_refs);
  RPG_CHECK("permute");
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return cleanup(RP_EHIP, std::string("device BVH build: ") + hipGetErrorString(e));
#undef RPG_CHECK
  return cleanup(RP_OK, "");
}

}  // namespace rpg
