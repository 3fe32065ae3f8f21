// rp_api.cpp -- implementation of the C-ABI in include/rp.h (librp.so).
//
// Host side of the drop-in: validates the reference-shaped scene (rp_scene_desc mirrors hittable.rs,
// mesh.rs, material.rs, texture.rs), builds the acceleration structure (rp_bvh.cpp), copies it to HBM
// once, and launches the persistent render kernel (rp_kernel.hip) per frame / shard.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rp.h"
#include "rp_bvh.h"
#include "rp_kernel.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define RP_HIP(call)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess) return fail(RP_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <class T>
int upload(const std::vector<T>& v, T** out) {
  size_t bytes = sizeof(T) * (v.empty() ? 1 : v.size());
  hipError_t e = hipMalloc(reinterpret_cast<void**>(out), bytes);
  if (e != hipSuccess) return fail(RP_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  if (!v.empty()) {
    e = hipMemcpy(*out, v.data(), sizeof(T) * v.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) return fail(RP_EHIP, std::string("hipMemcpy: ") + hipGetErrorString(e));
  }
  return RP_OK;
}

}  // namespace

// Per-frame device state of a render (include/rp.h rp_workspace): frames with different workspaces may
// run concurrently on different streams.
struct rp_workspace {
  rp_scene* scene = nullptr;
  uint64_t* d_ctr = nullptr;         // default counter block (CTR_N x u64)
  uint64_t* d_probe_ctr = nullptr;   // counter block of the probe launch
  uint32_t* d_tile_cost = nullptr;   // cost probe output, 2 x rpk::TILE_SORT_MAX entries
  uint32_t* d_tile_order = nullptr;  // cost-ordered shard tiles, rpk::TILE_SORT_MAX entries
  uint32_t* d_slab = nullptr;        // keystream cache, one slab per resident render lane
  uint32_t* d_spill = nullptr;       // traversal-stack overflow entries of every resident lane (deep trees)
  double* d_partial = nullptr;       // per-batch sample sums of multi-batch frames (grown on demand)
  uint32_t* d_partial_hits = nullptr;
  uint64_t partial_units = 0;        // capacity of d_partial / d_partial_hits in units
};

struct rp_scene {
  int device = 0;
  rpk::KScene ks{};
  rpl::Node4* d_nodes = nullptr;
  rpl::Prim* d_prims = nullptr;
  rpl::PrimRef* d_prim_refs = nullptr;
  double* d_vnrm = nullptr;
  double* d_vuv = nullptr;
  rpl::Material* d_mats = nullptr;
  rpl::Texture* d_texs = nullptr;
  uint32_t* d_texels = nullptr;
  uint64_t* d_diag = nullptr;  // diagnostic counters (rpk::DIAG_N)
  rp_workspace ws0;            // the scene's own workspace (rp_render, rp_render_device)
  int n_workspaces = 0;        // live workspaces from rp_workspace_create
  uint64_t n_nodes = 0, n_leaves = 0, n_prims = 0, device_bytes = 0;
  uint32_t max_depth = 0;
  int num_cu = 0;
  int blocks_per_cu = 0;
};

namespace {

void ws_release(rp_workspace* w) {
  for (void* p : {(void*)w->d_ctr, (void*)w->d_probe_ctr, (void*)w->d_tile_cost, (void*)w->d_tile_order,
                  (void*)w->d_slab, (void*)w->d_spill, (void*)w->d_partial, (void*)w->d_partial_hits})
    if (p) (void)hipFree(p);
  *w = rp_workspace{};
}

// Allocate a workspace for scene s (current device = the scene's): counters, probe/sort buffers and a
// keystream slab for every lane the render grid can hold resident.
int ws_alloc(rp_scene* s, rp_workspace* w) {
  *w = rp_workspace{};
  w->scene = s;
  const uint64_t lanes = (uint64_t)s->num_cu * (uint64_t)s->blocks_per_cu * rpk::RENDER_BLOCK;
  if (hipMalloc(reinterpret_cast<void**>(&w->d_ctr), sizeof(uint64_t) * rpk::CTR_N) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&w->d_probe_ctr), sizeof(uint64_t) * rpk::CTR_N) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&w->d_tile_cost), sizeof(uint32_t) * 2 * rpk::TILE_SORT_MAX) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&w->d_tile_order), sizeof(uint32_t) * rpk::TILE_SORT_MAX) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&w->d_slab), lanes * rpk::rng_slab_bytes_per_lane()) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&w->d_spill),
                lanes * sizeof(uint32_t) * std::max<uint64_t>(1, s->ks.stack_depth - s->ks.lds_depth)) != hipSuccess) {
    ws_release(w);
    return fail(RP_ENOMEM, "hipMalloc render workspace");
  }
  return RP_OK;
}

struct Tiling {
  uint32_t tw, th, shards, shard, tiles_x, tiles_y, n_tiles, n_shard_tiles;
  uint64_t n_slots;
};

int make_tiling(const rp_render_params* p, Tiling& t) {
  if (!p) return fail(RP_EINVAL, "params is NULL");
  if (p->width == 0 || p->height == 0) return fail(RP_EINVAL, "width and height must be >= 1");
  if (p->width > 65535 || p->height > 65535) return fail(RP_EINVAL, "width and height must be <= 65535");
  t.tw = p->tile_w ? p->tile_w : 32;
  t.th = p->tile_h ? p->tile_h : 32;
  t.shards = p->num_shards ? p->num_shards : 1;
  t.shard = p->shard;
  if (t.shard >= t.shards) return fail(RP_EINVAL, "shard must be < num_shards");
  t.tiles_x = (p->width + t.tw - 1) / t.tw;
  t.tiles_y = (p->height + t.th - 1) / t.th;
  t.n_tiles = t.tiles_x * t.tiles_y;
  t.n_shard_tiles = t.n_tiles > t.shard ? (t.n_tiles - t.shard + t.shards - 1) / t.shards : 0;
  t.n_slots = (uint64_t)t.n_shard_tiles * t.tw * t.th;
  if (t.n_slots >= 0xffffffffull) return fail(RP_EINVAL, "shard too large (>= 2^32 pixel slots)");
  return RP_OK;
}

// Lanes of a wave keep stepping traversal while at least this many are still traversing; below it,
// the finished lanes shade and take new rays (1 = wait for every lane, 64 = shade eagerly).
// Override with RP_TRAV_THRESHOLD for tuning.
uint32_t trav_threshold() {
  static const uint32_t v = [] {
    const char* e = std::getenv("RP_TRAV_THRESHOLD");
    long x = e ? std::strtol(e, nullptr, 10) : 24;
    return (uint32_t)(x < 1 ? 1 : (x > 64 ? 64 : x));
  }();
  return v;
}

// Acceleration-structure builder: the host binned SAH (rp_bvh.cpp, the better tree) unless the scene is
// large enough for its single-threaded build to dominate setup, then the device LBVH (rp_bvh_gpu.hip).
// RP_BVH_BUILDER=host|gpu forces one (read per scene).
enum : uint32_t { GPU_BUILD_MIN_PRIMS = 1u << 20 };
bool use_gpu_builder(uint32_t n_hittables) {
  if (n_hittables < 2) return false;
  if (const char* e = std::getenv("RP_BVH_BUILDER")) {
    if (std::strcmp(e, "gpu") == 0) return true;
    if (std::strcmp(e, "host") == 0) return false;
  }
  return n_hittables >= GPU_BUILD_MIN_PRIMS;
}

// Cost-ordered tile scheduling (rp_kernel.h); RP_TILE_ORDER=0 restores plain shard order (for A/B timing).
bool tile_order_enabled() {
  static const bool v = [] {
    const char* e = std::getenv("RP_TILE_ORDER");
    return !(e && std::strtol(e, nullptr, 10) == 0);
  }();
  return v;
}

// to_srgb_u8's byte for one channel (utility.rs:212-216), in the host libm: the reference's arithmetic
// (Rust's f64::powf is the platform pow).  Same expression as rph_to_srgb_u8 (rp_host.cpp).
uint32_t srgb_byte(double x) {
  if (x < 0.0) x = 0.0;
  if (x > 1.0) x = 1.0;
  const double y = 255.0 * std::pow(x, 1.0 / 2.2);
  return !(y > 0.0) ? 0u : (y >= 255.0 ? 255u : (uint32_t)y);
}

// thr[k] = the smallest double x in [0, 1] with srgb_byte(x) >= k (bisection over the bit patterns of
// non-negative doubles, which order like their values); computed once.
const rpk::SrgbTable& srgb_table() {
  static const rpk::SrgbTable tab = [] {
    rpk::SrgbTable t{};
    t.thr[0] = -HUGE_VAL;
    for (uint32_t k = 1; k < 256; k++) {
      uint64_t lo = 0, hi = 0x3FF0000000000000ull;  // srgb_byte(0) = 0 < k <= 255 = srgb_byte(1)
      while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        double x;
        std::memcpy(&x, &mid, sizeof x);
        if (srgb_byte(x) >= k) hi = mid;
        else lo = mid;
      }
      std::memcpy(&t.thr[k], &hi, sizeof hi);
    }
    return t;
  }();
  return tab;
}

}  // namespace

extern "C" {

int rp_srgb_thresholds(double* out) {
  if (!out) return fail(RP_EINVAL, "out is NULL");
  std::memcpy(out, srgb_table().thr, sizeof(double) * 256);
  return RP_OK;
}

int rp_shard_to_bgra8(rp_scene* s, const rp_render_params* p, const double* d_shard_rgb, uint8_t* d_shard_bgra,
                      void* stream) {
  if (!s || !d_shard_rgb || !d_shard_bgra) return fail(RP_EINVAL, "scene and buffers must be non-NULL");
  if (reinterpret_cast<uintptr_t>(d_shard_bgra) % 4 != 0) return fail(RP_EINVAL, "d_shard_bgra must be 4-byte aligned");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  DeviceGuard g(s->device);
  int e = rpk::launch_srgb_bgra(srgb_table(), d_shard_rgb, t.n_slots, d_shard_bgra, stream);
  if (e != 0) return fail(RP_EHIP, std::string("output stage launch: ") + hipGetErrorString((hipError_t)e));
  return RP_OK;
}

int rp_abi_version(void) { return RP_ABI_VERSION; }

const char* rp_last_error(void) { return g_err.c_str(); }

int rp_device_count(int* count) {
  if (!count) return fail(RP_EINVAL, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(RP_ENODEV, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = n;
  return RP_OK;
}

void rp_scene_destroy(rp_scene* s) {
  if (!s) return;
  DeviceGuard g(s->device);
  ws_release(&s->ws0);
  for (void* p : {(void*)s->d_nodes, (void*)s->d_prims, (void*)s->d_prim_refs, (void*)s->d_vnrm, (void*)s->d_vuv, (void*)s->d_mats,
                  (void*)s->d_texs, (void*)s->d_texels, (void*)s->d_diag})
    if (p) (void)hipFree(p);
  delete s;
}

int rp_scene_create(const rp_scene_desc* desc, int device, rp_scene** out) {
  if (!out) return fail(RP_EINVAL, "out is NULL");
  *out = nullptr;
  std::string err;
  int rc = rpb::validate(desc, err);
  if (rc != RP_OK) return fail(rc, err);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RP_ENODEV, "no HIP device");
  if (device < 0 || device >= ndev) return fail(RP_EINVAL, "device index out of range");
  hipDeviceProp_t prop;
  RP_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(RP_ENODEV, std::string("librp.so is built for gfx950, device is ") + prop.gcnArchName);

  rpb::PackedScene ps;
  rpb::BuildOptions opt;
  const bool gpu_build = use_gpu_builder(desc->n_hittables);
  opt.tables_only = gpu_build;
  // tuning knobs for experiments (the defaults are the measured best): leaf size and SAH cost ratio
  if (const char* e = std::getenv("RP_BVH_MAX_LEAF")) opt.max_leaf = (uint32_t)std::strtoul(e, nullptr, 10);
  if (const char* e = std::getenv("RP_BVH_COST_TRAVERSE")) opt.cost_traverse = std::strtod(e, nullptr);
  if (const char* e = std::getenv("RP_ALWAYS_MAX")) opt.always_max = (uint32_t)std::strtoul(e, nullptr, 10);
  rc = rpb::build(desc, opt, ps, err);
  if (rc != RP_OK) return fail(rc, err);

  DeviceGuard g(device);
  rp_scene* s = new rp_scene();
  s->device = device;
  s->num_cu = prop.multiProcessorCount;
  auto bail = [&](int code) { rp_scene_destroy(s); return code; };
  uint64_t n_tree_nodes = ps.nodes.size(), n_tree_prims = ps.prims.size();
  if (gpu_build) {
    rpb::PrimInput pin;
    if ((rc = rpb::prim_input(desc, pin, err))) return bail(fail(rc, err));
    rpg::GpuTree gt;
    if ((rc = rpg::build_gpu(pin, opt.max_leaf, gt, err))) return bail(fail(rc, err));
    s->d_nodes = gt.d_nodes;
    s->d_prims = gt.d_prims;
    s->d_prim_refs = gt.d_prim_refs;
    ps.root = 0;
    ps.max_depth = gt.max_depth;
    ps.n_leaves = gt.n_leaves;
    n_tree_nodes = gt.n_nodes;
    n_tree_prims = pin.prims.size();
    if (const char* e = std::getenv("RP_BVH_CHECK"); e && std::strcmp(e, "1") == 0) {
      // test hook: the structural self-check of the host builder on the device-built tree
      rpb::PackedScene chk;
      chk.nodes.resize(n_tree_nodes);
      chk.prims.resize(n_tree_prims);
      chk.prim_refs.resize(n_tree_prims);
      RP_HIP(hipMemcpy(chk.nodes.data(), s->d_nodes, sizeof(rpl::Node4) * n_tree_nodes, hipMemcpyDeviceToHost));
      RP_HIP(hipMemcpy(chk.prims.data(), s->d_prims, sizeof(rpl::Prim) * n_tree_prims, hipMemcpyDeviceToHost));
      RP_HIP(hipMemcpy(chk.prim_refs.data(), s->d_prim_refs, sizeof(rpl::PrimRef) * n_tree_prims, hipMemcpyDeviceToHost));
      chk.root = 0;
      chk.max_depth = gt.max_depth;
      chk.n_leaves = gt.n_leaves;
      if ((rc = rpb::check(chk, err))) return bail(fail(rc, "device BVH self-check: " + err));
    }
  } else if ((rc = upload(ps.nodes, &s->d_nodes)) || (rc = upload(ps.prims, &s->d_prims)) ||
             (rc = upload(ps.prim_refs, &s->d_prim_refs))) {
    return bail(rc);
  }
  if ((rc = upload(ps.vnrm, &s->d_vnrm)) || (rc = upload(ps.vuv, &s->d_vuv)) ||
      (rc = upload(ps.materials, &s->d_mats)) || (rc = upload(ps.textures, &s->d_texs)) ||
      (rc = upload(ps.texels, &s->d_texels)))
    return bail(rc);
  if (hipMalloc(reinterpret_cast<void**>(&s->d_diag), sizeof(uint64_t) * rpk::DIAG_N) != hipSuccess ||
      hipMemset(s->d_diag, 0, sizeof(uint64_t) * rpk::DIAG_N) != hipSuccess)
    return bail(fail(RP_ENOMEM, "hipMalloc workspace"));
  s->ks.diag = s->d_diag;
  s->ks.nodes = s->d_nodes;
  s->ks.prims = s->d_prims;
  s->ks.prim_refs = s->d_prim_refs;
  s->ks.vnrm = s->d_vnrm;
  s->ks.vuv = s->d_vuv;
  s->ks.mats = s->d_mats;
  s->ks.texs = s->d_texs;
  s->ks.texels = s->d_texels;
  s->ks.background = ps.background;
  s->ks.root = ps.root;
  s->ks.always_first = ps.always_first;  // 0 / 0 for a device-built tree
  s->ks.n_always = ps.n_always;
  // a wide node pushes at most 3 entries (its non-nearest hits) per level below the root; +3 spare
  // entries for the kernel's branchless push (rp_kernel.hip STACK_SLACK)
  s->ks.stack_depth = 3 * ps.max_depth + 4 + 3;
  // floor of 17 entries: the spill split below never keeps fewer in LDS (RP_LDS_DEPTH tests force 17)
  if (s->ks.stack_depth < 17) s->ks.stack_depth = 17;
  s->n_nodes = n_tree_nodes;
  s->n_leaves = ps.n_leaves;
  s->n_prims = desc->n_hittables;
  s->max_depth = ps.max_depth;
  s->device_bytes = sizeof(rpl::Node4) * n_tree_nodes + (sizeof(rpl::Prim) + sizeof(rpl::PrimRef)) * n_tree_prims +
                    sizeof(double) * (ps.vnrm.size() + ps.vuv.size()) + sizeof(rpl::Material) * ps.materials.size() +
                    sizeof(rpl::Texture) * ps.textures.size() + sizeof(uint32_t) * ps.texels.size();
  // LDS holds the whole stack unless that costs resident blocks: then the deepest entries spill to a
  // per-lane global run (rp_kernel.hip stk_put/stk_get) and LDS keeps the largest depth that still fits
  // the occupancy of a shallow stack (C5's 43-entry stack: 3 -> 4 blocks per CU).  RP_LDS_DEPTH forces a
  // depth (>= 17) for tests and tuning.
  s->ks.lds_depth = s->ks.stack_depth;
  int bpc = 0;
  if (rpk::render_blocks_per_cu(s->ks.stack_depth, false, &bpc) != 0 || bpc < 1) bpc = 1;
  int bpc_spill = 0;
  if (rpk::render_blocks_per_cu(17, true, &bpc_spill) == 0 && bpc_spill > bpc) {
    uint32_t L = s->ks.stack_depth - 1;
    int b = 0;
    while (L > 17 && (rpk::render_blocks_per_cu(L, true, &b) != 0 || b < bpc_spill)) L--;
    s->ks.lds_depth = L;
    bpc = bpc_spill;
  }
  if (const char* e = std::getenv("RP_LDS_DEPTH")) {
    const uint32_t L = (uint32_t)std::strtoul(e, nullptr, 10);
    if (L >= 17 && L < s->ks.stack_depth) {
      s->ks.lds_depth = L;
      if (rpk::render_blocks_per_cu(L, true, &bpc) != 0 || bpc < 1) bpc = 1;
    }
  }
  s->blocks_per_cu = bpc;
  if ((rc = ws_alloc(s, &s->ws0))) return bail(rc);
  *out = s;
  return RP_OK;
}

int rp_scene_info(const rp_scene* s, uint64_t* n_nodes, uint64_t* n_leaves, uint32_t* max_depth, uint64_t* n_prims,
                  uint64_t* device_bytes) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  if (n_nodes) *n_nodes = s->n_nodes;
  if (n_leaves) *n_leaves = s->n_leaves;
  if (max_depth) *max_depth = s->max_depth;
  if (n_prims) *n_prims = s->n_prims;
  if (device_bytes) *device_bytes = s->device_bytes;
  return RP_OK;
}

int rp_shard_pixel_count(const rp_render_params* p, uint64_t* count) {
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (!count) return fail(RP_EINVAL, "count is NULL");
  *count = t.n_slots;
  return RP_OK;
}

int rp_shard_unpack(const rp_render_params* p, const double* shard_buf, uint32_t channels, double* frame) {
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (!shard_buf || !frame || channels == 0) return fail(RP_EINVAL, "NULL buffer or zero channels");
  const uint64_t tile_px = (uint64_t)t.tw * t.th;
  for (uint32_t k = 0; k < t.n_shard_tiles; k++) {
    uint32_t tile = t.shard + k * t.shards;
    uint32_t ox = (tile % t.tiles_x) * t.tw, oy = (tile / t.tiles_x) * t.th;
    for (uint32_t lj = 0; lj < t.th; lj++) {
      uint32_t j = oy + lj;
      if (j >= p->height) break;
      for (uint32_t li = 0; li < t.tw; li++) {
        uint32_t i = ox + li;
        if (i >= p->width) break;
        const double* src = shard_buf + (k * tile_px + (uint64_t)lj * t.tw + li) * channels;
        double* dst = frame + ((uint64_t)j * p->width + i) * channels;
        for (uint32_t c = 0; c < channels; c++) dst[c] = src[c];
      }
    }
  }
  return RP_OK;
}

int rp_workspace_create(rp_scene* s, rp_workspace** out) {
  if (!out) return fail(RP_EINVAL, "out is NULL");
  *out = nullptr;
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  DeviceGuard g(s->device);
  rp_workspace* w = new rp_workspace();
  int rc = ws_alloc(s, w);
  if (rc) {
    delete w;
    return rc;
  }
  s->n_workspaces++;
  *out = w;
  return RP_OK;
}

void rp_workspace_destroy(rp_workspace* w) {
  if (!w || !w->scene) return;
  rp_scene* s = w->scene;
  DeviceGuard g(s->device);
  ws_release(w);
  s->n_workspaces--;
  delete w;
}

int rp_render_device(rp_scene* s, const rp_camera* cam, const rp_render_params* p, double* d_rgb, float* d_fg,
                     uint64_t* d_counters, void* stream) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  return rp_render_device_ws(s, &s->ws0, cam, p, d_rgb, d_fg, d_counters, stream);
}

int rp_render_device_ws(rp_scene* s, rp_workspace* w, const rp_camera* cam, const rp_render_params* p, double* d_rgb,
                        float* d_fg, uint64_t* d_counters, void* stream) {
  if (!s || !cam || !d_rgb) return fail(RP_EINVAL, "scene, camera and output must be non-NULL");
  if (!w || w->scene != s) return fail(RP_EINVAL, "workspace is NULL or belongs to another scene");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (p->max_bounce < 1) return fail(RP_EINVAL, "max_bounce must be >= 1 (render.rs:97 assert!(depth >= 1))");
  DeviceGuard g(s->device);
  uint64_t* ctr = d_counters ? d_counters : w->d_ctr;
  hipStream_t st = (hipStream_t)stream;
  RP_HIP(hipMemsetAsync(ctr, 0, sizeof(uint64_t) * rpk::CTR_N, st));
  if (t.n_slots == 0) return RP_OK;
  if (p->spp == 0) {
    // main.rs:86-87 with num_samples = 0: (0,0,0) / 0 and 0 / 0 are NaN; all-ones bits are a NaN.
    RP_HIP(hipMemsetAsync(d_rgb, 0xff, sizeof(double) * 3 * t.n_slots, st));
    if (d_fg) RP_HIP(hipMemsetAsync(d_fg, 0xff, sizeof(float) * t.n_slots, st));
    return RP_OK;
  }
  rpk::KParams kp{};
  std::memcpy(kp.orient, cam->orientation, sizeof kp.orient);
  std::memcpy(kp.pos, cam->position, sizeof kp.pos);
  kp.aspect = cam->aspect_ratio;
  kp.tan_fov = std::tan(0.5 * cam->fov);  // render.rs:33, hoisted: a per-camera constant
  kp.focal = cam->focal_dist;
  kp.lens = cam->lens_radius;
  kp.seed = p->seed;
  kp.W = p->width;
  kp.H = p->height;
  kp.spp = p->spp;
  kp.max_bounce = p->max_bounce;
  kp.tw = t.tw;
  kp.th = t.th;
  kp.shard = t.shard;
  kp.nshards = t.shards;
  kp.tiles_x = t.tiles_x;
  kp.n_shard_tiles = t.n_shard_tiles;
  kp.n_slots = t.n_slots;
  kp.trav_threshold = trav_threshold();
  // RP_SPP_BATCH overrides the contract's batch size for timing studies only (it changes every
  // multi-batch image: never set it for parity runs)
  kp.spp_batch = rpk::SPP_BATCH;
  if (const char* e = std::getenv("RP_SPP_BATCH")) kp.spp_batch = std::max(1u, (uint32_t)std::strtoul(e, nullptr, 10));
  kp.nbatch = (p->spp + kp.spp_batch - 1) / kp.spp_batch;
  kp.n_queue = t.n_slots * kp.nbatch;
  if (kp.n_queue >= 0xffffffffull) return fail(RP_EINVAL, "shard too large (>= 2^32 pixel-batch units)");
  if (kp.nbatch > 1) {
    if (kp.n_queue > w->partial_units) {  // workspace-owned, grown on the first call that needs it
      if (w->d_partial) (void)hipFree(w->d_partial);
      if (w->d_partial_hits) (void)hipFree(w->d_partial_hits);
      w->d_partial = nullptr;
      w->d_partial_hits = nullptr;
      w->partial_units = 0;
      if (hipMalloc(reinterpret_cast<void**>(&w->d_partial), sizeof(double) * 3 * kp.n_queue) != hipSuccess ||
          hipMalloc(reinterpret_cast<void**>(&w->d_partial_hits), sizeof(uint32_t) * kp.n_queue) != hipSuccess)
        return fail(RP_ENOMEM, "hipMalloc sample-batch workspace");
      w->partial_units = kp.n_queue;
    }
    kp.partial = w->d_partial;
    kp.partial_hits = w->d_partial_hits;
  }
  const uint64_t resident = (uint64_t)s->num_cu * (uint64_t)s->blocks_per_cu;
  rpk::KScene ks = s->ks;
  ks.rng_slab = w->d_slab;
  ks.spill = w->d_spill;
  auto grid_for = [&](uint64_t slots) {
    const uint64_t want = (slots + rpk::RENDER_BLOCK - 1) / rpk::RENDER_BLOCK;
    return (int)std::max<uint64_t>(1, std::min(want, resident));
  };
  if (tile_order_enabled() && t.n_shard_tiles > 1 && t.n_shard_tiles <= rpk::TILE_SORT_MAX) {
    // probe sample 0 of PROBE_PX pixels per tile, then sort the tiles by cost (same stream, no host sync)
    rpk::KParams pk = kp;
    pk.probe = 1;
    pk.spp = 1;
    // every pixel's sample 0 once spp is large enough to amortise it (a 1/spp extra), else a lattice
    // an n x n lattice of pixels per tile (RP_PROBE_N overrides n for tuning; 0 = every pixel)
    pk.probe_n = rpk::PROBE_LATTICE_N;
    if (const char* e = std::getenv("RP_PROBE_N")) pk.probe_n = (uint32_t)std::strtoul(e, nullptr, 10);
    pk.probe_n = std::min(pk.probe_n, std::min(t.tw, t.th));
    pk.probe_px = pk.probe_n ? pk.probe_n * pk.probe_n : t.tw * t.th;
    pk.n_slots = (uint64_t)t.n_shard_tiles * pk.probe_px;
    pk.nbatch = 1;
    pk.spp_batch = 1;
    pk.n_queue = pk.n_slots;
    pk.tile_cost = w->d_tile_cost;
    RP_HIP(hipMemsetAsync(w->d_probe_ctr, 0, sizeof(uint64_t) * rpk::CTR_N, st));
    RP_HIP(hipMemsetAsync(w->d_tile_cost, 0, sizeof(uint32_t) * 2 * rpk::TILE_SORT_MAX, st));
    int e = rpk::launch_render(ks, pk, d_rgb, nullptr, w->d_probe_ctr, grid_for(pk.n_slots), stream);
    if (e != 0) return fail(RP_EHIP, std::string("probe launch: ") + hipGetErrorString((hipError_t)e));
    e = rpk::launch_tile_sort(w->d_tile_cost, t.n_shard_tiles, pk.probe_px, w->d_tile_order, stream);
    if (e != 0) return fail(RP_EHIP, std::string("tile sort launch: ") + hipGetErrorString((hipError_t)e));
    kp.tile_order = w->d_tile_order;
  }
  int e = rpk::launch_render(ks, kp, d_rgb, d_fg, ctr, grid_for(kp.n_queue), stream);
  if (e != 0) return fail(RP_EHIP, std::string("render launch: ") + hipGetErrorString((hipError_t)e));
  if (kp.nbatch > 1) {
    e = rpk::launch_reduce_batches(kp, d_rgb, d_fg, stream);
    if (e != 0) return fail(RP_EHIP, std::string("reduce launch: ") + hipGetErrorString((hipError_t)e));
  }
  return RP_OK;
}

int rp_render(rp_scene* s, const rp_camera* cam, const rp_render_params* p, double* out_rgb, float* out_fg,
              rp_stats* stats) {
  if (!s || !cam || !out_rgb) return fail(RP_EINVAL, "scene, camera and output must be non-NULL");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  DeviceGuard g(s->device);
  double* d_rgb = nullptr;
  float* d_fg = nullptr;
  uint64_t* d_ctr = nullptr;
  hipStream_t st = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  int result = RP_OK;
  std::vector<double> shard(3 * (t.n_slots ? t.n_slots : 1));
  std::vector<float> shard_fg(out_fg ? (t.n_slots ? t.n_slots : 1) : 0);
  uint64_t ctr[rpk::CTR_N] = {0};
  float ms = 0.f;
  do {
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) { result = fail(RP_EHIP, "stream"); break; }
    if (hipMalloc(reinterpret_cast<void**>(&d_rgb), sizeof(double) * shard.size()) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_ctr), sizeof(uint64_t) * rpk::CTR_N) != hipSuccess ||
        (out_fg && hipMalloc(reinterpret_cast<void**>(&d_fg), sizeof(float) * shard_fg.size()) != hipSuccess)) {
      result = fail(RP_ENOMEM, "hipMalloc output");
      break;
    }
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) { result = fail(RP_EHIP, "event"); break; }
    (void)hipEventRecord(e0, st);
    result = rp_render_device(s, cam, p, d_rgb, d_fg, d_ctr, st);
    if (result) break;
    (void)hipEventRecord(e1, st);
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) { result = fail(RP_EHIP, std::string("render: ") + hipGetErrorString(e)); break; }
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (hipMemcpy(shard.data(), d_rgb, sizeof(double) * shard.size(), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost) != hipSuccess ||
        (out_fg && hipMemcpy(shard_fg.data(), d_fg, sizeof(float) * shard_fg.size(), hipMemcpyDeviceToHost) != hipSuccess)) {
      result = fail(RP_EHIP, "copy back");
      break;
    }
  } while (0);
  if (d_rgb) (void)hipFree(d_rgb);
  if (d_fg) (void)hipFree(d_fg);
  if (d_ctr) (void)hipFree(d_ctr);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (result) return result;
  if (ctr[rpk::CTR_STATUS] & rpk::STATUS_STACK_OVERFLOW) return fail(RP_EINTERNAL, "traversal stack overflow");
  if (t.n_slots) {
    rp_shard_unpack(p, shard.data(), 3, out_rgb);
    if (out_fg) {
      const uint64_t tile_px = (uint64_t)t.tw * t.th;
      for (uint32_t k = 0; k < t.n_shard_tiles; k++) {
        uint32_t tile = t.shard + k * t.shards;
        uint32_t ox = (tile % t.tiles_x) * t.tw, oy = (tile / t.tiles_x) * t.th;
        for (uint32_t lj = 0; lj < t.th && oy + lj < p->height; lj++)
          for (uint32_t li = 0; li < t.tw && ox + li < p->width; li++)
            out_fg[(uint64_t)(oy + lj) * p->width + ox + li] = shard_fg[k * tile_px + (uint64_t)lj * t.tw + li];
      }
    }
  }
  if (stats) {
    stats->rays = ctr[rpk::CTR_RAYS];
    stats->samples = ctr[rpk::CTR_SAMPLES];
    stats->pixels = ctr[rpk::CTR_PIXELS];
    stats->seconds = ms * 1e-3;
  }
  return RP_OK;
}

int rp_diagnostics(rp_scene* s, uint64_t* out, uint32_t n, int reset) {
  if (!s || (!out && n)) return fail(RP_EINVAL, "NULL argument");
  DeviceGuard g(s->device);
  uint64_t buf[rpk::DIAG_N];
  RP_HIP(hipDeviceSynchronize());
  RP_HIP(hipMemcpy(buf, s->d_diag, sizeof buf, hipMemcpyDeviceToHost));
  for (uint32_t i = 0; i < n; i++) out[i] = i < (uint32_t)rpk::DIAG_N ? buf[i] : 0;
  if (reset) RP_HIP(hipMemset(s->d_diag, 0, sizeof buf));
  return RP_OK;
}

int rp_intersect(rp_scene* s, const double* rays, uint64_t n, double* out_hit, uint32_t* out_material) {
  if (!s || (n && (!rays || !out_hit || !out_material))) return fail(RP_EINVAL, "NULL argument");
  if (n == 0) return RP_OK;
  DeviceGuard g(s->device);
  double *d_rays = nullptr, *d_hit = nullptr;
  uint32_t* d_mat = nullptr;
  uint64_t* d_ctr = nullptr;
  int result = RP_OK;
  uint64_t ctr[rpk::CTR_N] = {0};
  do {
    if (hipMalloc(reinterpret_cast<void**>(&d_rays), sizeof(double) * 8 * n) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_hit), sizeof(double) * 9 * n) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_mat), sizeof(uint32_t) * n) != hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&d_ctr), sizeof(uint64_t) * rpk::CTR_N) != hipSuccess) {
      result = fail(RP_ENOMEM, "hipMalloc");
      break;
    }
    if (hipMemcpy(d_rays, rays, sizeof(double) * 8 * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(d_ctr, 0, sizeof(uint64_t) * rpk::CTR_N) != hipSuccess) {
      result = fail(RP_EHIP, "hipMemcpy");
      break;
    }
    int e = rpk::launch_intersect(s->ks, d_rays, n, d_hit, d_mat, d_ctr, nullptr);
    if (e) { result = fail(RP_EHIP, std::string("intersect launch: ") + hipGetErrorString((hipError_t)e)); break; }
    hipError_t he = hipDeviceSynchronize();
    if (he != hipSuccess) { result = fail(RP_EHIP, std::string("intersect: ") + hipGetErrorString(he)); break; }
    if (hipMemcpy(out_hit, d_hit, sizeof(double) * 9 * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(out_material, d_mat, sizeof(uint32_t) * n, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost) != hipSuccess) {
      result = fail(RP_EHIP, "copy back");
      break;
    }
  } while (0);
  for (void* p : {(void*)d_rays, (void*)d_hit, (void*)d_mat, (void*)d_ctr})
    if (p) (void)hipFree(p);
  if (result) return result;
  if (ctr[rpk::CTR_STATUS] & rpk::STATUS_STACK_OVERFLOW) return fail(RP_EINTERNAL, "traversal stack overflow");
  return RP_OK;
}

}  // extern "C"
