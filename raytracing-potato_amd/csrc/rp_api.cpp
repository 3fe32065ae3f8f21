// rp_api.cpp -- implementation of the C-ABI in include/rp.h (librp.so).
//
// Host side of the drop-in: validates the reference-shaped scene (rp_scene_desc mirrors hittable.rs,
// mesh.rs, material.rs, texture.rs), builds the acceleration structure (rp_bvh.cpp / rp_bvh_gpu.hip),
// copies it to HBM once, launches the persistent render kernel (rp_kernel.hip) per frame / shard, and
// assembles multi-GPU frames with one RCCL all-gather over xGMI.  The library reads no
// environment variables: every knob is an argument (rp_scene_options, rp_render_params).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rp.h"
#include "rp_bvh.h"
#include "rp_kernel.h"

static_assert(rpk::CTR_N == RP_COUNTERS_LEN, "kernel counter block = the ABI's");
static_assert(rpk::CTR_RAYS == RP_CTR_RAYS && rpk::CTR_STATUS == RP_CTR_STATUS, "counter order");
static_assert(rpk::STATUS_STACK_OVERFLOW == RP_STATUS_STACK_OVERFLOW && rpk::STATUS_PLAN_MISMATCH == RP_STATUS_PLAN_MISMATCH,
              "status bits");
static_assert(sizeof(ncclUniqueId) == RP_COMM_ID_BYTES, "RCCL unique id size");
static_assert(sizeof(rp_render_params) == 48, "rp_render_params layout (bindings mirror it)");

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

#define RP_NCCL(call)                                                                           \
  do {                                                                                          \
    ncclResult_t r_ = (call);                                                                   \
    if (r_ != ncclSuccess) return fail(RP_ERCCL, std::string(#call) + ": " + ncclGetErrorString(r_)); \
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

template <class T>
bool dalloc(T** p, uint64_t n) {
  return hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (n ? n : 1)) == hipSuccess;
}

void dfree(void* p) {
  if (p) (void)hipFree(p);
}

// Defaults of rp_scene_options (the measured best).
constexpr uint32_t DEF_MAX_LEAF = 4, DEF_TRAV_THRESHOLD = 24, DEF_ALWAYS_MAX = 4;
constexpr uint32_t DEF_UNIT_QUEUES = RP_QUEUES_XCD_TILES;
constexpr uint32_t QUEUE_CHUNK_AUTO = 8;  // rp_scene_options.queue_chunk = 0: tiles per queue chunk (render_shard)
constexpr double DEF_COST_TRAVERSE = 0.7;
// Balanced plans under tile_order = RP_TILES_MORTON deal square blocks of tiles (rpk::launch_tile_plan): 4 x 4, or 2 x 2,
// as long as every rank still gets >= PLAN_UNITS_MIN of them (balance needs many units per rank), else single tiles.
// (AUTO is the cost order for every scene since v49, which deals tile by tile; the block deal runs only when a caller
// asks for Z-order tiles.)  The deal hands out U = block^2 consecutive positions of the block-sorted order: on a grid
// whose tiles_x or tiles_y is not a multiple of block, the edge blocks hold fewer than U tiles, so a unit after the
// first partial block straddles two blocks -- counts and balance are unchanged, only the squares are no longer whole
// (tests/test_dist.py test_block_deal_ragged_grid).
constexpr uint32_t PLAN_UNITS_MIN = 32;
uint32_t plan_block(uint32_t n_tiles, uint32_t nranks) {
  for (uint32_t b : {4u, 2u})
    if (n_tiles >= PLAN_UNITS_MIN * nranks * b * b) return b;
  return 1u;
}

}  // namespace

// Per-frame device state of a render (include/rp.h rp_workspace): frames with different workspaces may
// run concurrently on different streams.
struct rp_workspace {
  rp_scene* scene = nullptr;
  uint64_t* d_ctr = nullptr;         // counters when the caller passes none (CTR_N x u64)
  uint64_t* d_probe_ctr = nullptr;   // counters of the probe launch
  uint32_t* d_queue = nullptr;       // unit queues, one 128 B line each: the frame's groups, then the probe
  uint32_t* d_tile_cost = nullptr;   // cost probe output, 2 x rpk::TILE_SORT_MAX entries
  uint32_t* d_tile_order = nullptr;  // cost-ordered shard tiles, rpk::TILE_SORT_MAX entries
  uint32_t* d_slab = nullptr;        // keystream cache, one slab per resident render lane
  uint32_t* d_spill = nullptr;       // traversal-stack overflow entries of every resident lane (deep trees)
  uint32_t* d_t0 = nullptr;          // start time of each resident lane's measured unit (tile costs)
  // reserved by rp_workspace_reserve:
  double* d_partial = nullptr;       // per-batch sample sums of multi-batch frames
  uint32_t* d_partial_hits = nullptr;
  uint64_t partial_units = 0;        // capacity of d_partial / d_partial_hits in units
  // the learned per-unit order (rp_sched.hip): each unit's duration in the last render, the sort keys (two buffers),
  // the radix sort's scratch and the order; ucost_geom = the frame shape the durations belong to
  uint32_t* d_ucost = nullptr;
  uint64_t* d_ukey = nullptr;
  uint64_t* d_ukey2 = nullptr;
  uint32_t* d_uorder = nullptr;
  void* d_usort = nullptr;
  size_t usort_bytes = 0;
  uint64_t ucost_cap = 0;
  bool ucost_valid = false;
  uint32_t ucost_geom[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  double* d_gs_rgb = nullptr;        // gather staging: this rank's shard, padded to the stride (3 f64 / slot)
  double* d_gather_rgb = nullptr;    //   all ranks' shards (nranks x stride x 3 f64)
  uint64_t gs_slots = 0;             // capacity of d_gs_rgb in slots
  uint64_t gather_slots = 0;         // capacity of d_gather_rgb in slots (over all ranks)
  // a frame gather's one collective (rpk::launch_gather_pack): this rank's packed block -- counters, measured tile
  // costs, to_srgb_u8 bytes -- and every rank's
  uint32_t* d_pack_send = nullptr;
  uint32_t* d_pack_recv = nullptr;
  uint64_t pack_words = 0;           // capacity of d_pack_send in words
  uint64_t pack_recv_words = 0;      // capacity of d_pack_recv in words
  // the balanced tile plan (RP_SHARD_BALANCED) of the last frame rendered with this workspace: the deal order,
  // its inverse and its hash (rpk::launch_tile_plan), and the frame geometry it was made for
  uint32_t* d_plan = nullptr;
  bool plan_on = false;
  uint32_t plan_geom[5] = {0, 0, 0, 0, 0};  // width, height, tile_w, tile_h, num_shards
  // Measured tile costs (rp_kernel.h tile_meas / launch_learn_costs): the last render's per-shard-tile unit
  // durations, every rank's of them after a frame gather, and the learned per-frame-tile table the next frame of
  // the same geometry schedules with instead of a cost probe.
  uint32_t* d_meas = nullptr;     // 2 x TILE_SORT_MAX: [k] summed, [TILE_SORT_MAX + k] longest unit of shard tile k
  uint32_t* d_fcost = nullptr;    // learned table: 2 x TILE_SORT_MAX, by frame tile
  uint64_t* d_sort = nullptr;     // the tile sorts' keys (rpk::SORT_SCRATCH words: global memory, not LDS)
  bool meas_on = false;           // the last render measured (megakernel)
  bool fcost_valid = false;
  uint32_t fcost_geom[4] = {0, 0, 0, 0};  // width, height, tile_w, tile_h of the learned table
  uint32_t fcost_ranks = 0;               // ranks whose gather made it (1: a whole-frame render on one device)
  // A frame gather reads this workspace's measured costs (d_meas) and writes its learned table (d_fcost) on the gather
  // stream; the next render on the workspace reads the table and clears d_meas on ITS stream.  The gather records
  // this event at its end and render_shard waits on it, so a caller with separate render and gather streams cannot
  // race the two; on one stream the wait is already satisfied.
  hipEvent_t ev_gathered = nullptr;
  bool gathered_pending = false;
  uint32_t frame_flags = 0;  // RP_FRAME_* of the last render (rp_workspace_frame_info)
};

struct rp_scene {
  int device = 0;
  rpk::KScene ks{};
  rp_scene_options opt{};
  void* d_nodes = nullptr;  // rpl::Node4 or rpl::Node4Q (ks.node_format)
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
  double build_s[RP_BUILD_PHASES] = {0};  // rp_scene_build_times
  uint32_t tiles_auto = RP_TILES_COST;  // the tile order of RP_TILES_AUTO (scene_create)
  uint32_t max_depth = 0;
  int num_cu = 0;
  int blocks_per_cu = 0;
  uint64_t lanes() const { return (uint64_t)num_cu * (uint64_t)blocks_per_cu * rpk::RENDER_BLOCK; }
};

struct rp_comm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0, device = 0;
};

struct rp_multi {
  std::vector<int> devices;
  std::vector<rp_scene*> scenes;
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> streams;
  std::vector<uint64_t*> d_ctr;  // per device, CTR_N
  double* d_frame_rgb = nullptr;  // device 0: the assembled frame
  uint32_t* d_frame_bgra = nullptr;
  uint64_t frame_px = 0;
};

namespace {

void ws_release(rp_workspace* w) {
  for (void* p : {(void*)w->d_ctr, (void*)w->d_probe_ctr, (void*)w->d_queue, (void*)w->d_tile_cost,
                  (void*)w->d_tile_order, (void*)w->d_slab, (void*)w->d_spill, (void*)w->d_partial,
                  (void*)w->d_partial_hits, (void*)w->d_gs_rgb, (void*)w->d_gather_rgb, (void*)w->d_pack_send,
                  (void*)w->d_pack_recv, (void*)w->d_plan, (void*)w->d_meas, (void*)w->d_fcost, (void*)w->d_sort,
                  (void*)w->d_t0, (void*)w->d_ucost, (void*)w->d_ukey, (void*)w->d_ukey2, (void*)w->d_uorder,
                  w->d_usort})
    dfree(p);
  if (w->ev_gathered) (void)hipEventDestroy(w->ev_gathered);
  *w = rp_workspace{};
}

// Allocate a workspace for scene s (current device = the scene's): counters, queues, probe/sort buffers
// and a keystream slab for every lane the render grid can hold resident.
int ws_alloc(rp_scene* s, rp_workspace* w) {
  *w = rp_workspace{};
  w->scene = s;
  const uint64_t lanes = s->lanes();
  if (!dalloc(&w->d_ctr, rpk::CTR_N) || !dalloc(&w->d_probe_ctr, rpk::CTR_N) || !dalloc(&w->d_queue, rpk::QUEUE_WORDS) ||
      !dalloc(&w->d_tile_cost, 2 * rpk::TILE_SORT_MAX) || !dalloc(&w->d_tile_order, rpk::TILE_SORT_MAX) ||
      !dalloc(&w->d_plan, 2 * rpk::TILE_SORT_MAX + 2) || !dalloc(&w->d_meas, 2 * rpk::TILE_SORT_MAX) ||
      !dalloc(&w->d_fcost, 2 * rpk::TILE_SORT_MAX) || !dalloc(&w->d_sort, rpk::SORT_SCRATCH) ||
      !dalloc(reinterpret_cast<uint8_t**>(&w->d_slab), lanes * rpk::rng_slab_bytes_per_lane()) ||
      !dalloc(&w->d_spill, lanes * std::max<uint64_t>(1, s->ks.stack_depth - s->ks.lds_depth)) ||
      !dalloc(&w->d_t0, lanes) || hipEventCreateWithFlags(&w->ev_gathered, hipEventDisableTiming) != hipSuccess) {
    ws_release(w);
    return fail(RP_ENOMEM, "hipMalloc render workspace");
  }
  return RP_OK;
}

struct Tiling {
  uint32_t tw, th, shards, shard, tiles_x, tiles_y, n_tiles, n_shard_tiles;
  uint64_t n_slots;
  uint32_t sps, nbatch;  // RNG contract: samples per stream, batches per pixel
  bool balanced;         // RP_SHARD_BALANCED in effect: the tiles are dealt by a plan (frames of <= TILE_SORT_MAX tiles)
};

int make_tiling(const rp_render_params* p, Tiling& t) {
  if (!p) return fail(RP_EINVAL, "params is NULL");
  if (p->width == 0 || p->height == 0) return fail(RP_EINVAL, "width and height must be >= 1");
  if (p->width > 65535 || p->height > 65535) return fail(RP_EINVAL, "width and height must be <= 65535");
  t.tw = p->tile_w ? p->tile_w : 32;
  t.th = p->tile_h ? p->tile_h : 32;
  if (t.tw > 65535 || t.th > 65535) return fail(RP_EINVAL, "tile_w and tile_h must be <= 65535");
  t.shards = p->num_shards ? p->num_shards : 1;
  t.shard = p->shard;
  if (t.shard >= t.shards) return fail(RP_EINVAL, "shard must be < num_shards");
  t.tiles_x = (p->width + t.tw - 1) / t.tw;
  t.tiles_y = (p->height + t.th - 1) / t.th;
  t.n_tiles = t.tiles_x * t.tiles_y;
  t.n_shard_tiles = t.n_tiles > t.shard ? (t.n_tiles - t.shard + t.shards - 1) / t.shards : 0;
  t.n_slots = (uint64_t)t.n_shard_tiles * t.tw * t.th;
  if (t.n_slots >= 0xffffffffull) return fail(RP_EINVAL, "shard too large (>= 2^32 pixel slots)");
  t.sps = p->samples_per_stream ? p->samples_per_stream : RP_SAMPLES_PER_STREAM;
  t.nbatch = p->spp ? (uint32_t)(((uint64_t)p->spp + t.sps - 1) / t.sps) : 0;
  if (p->shard_map > RP_SHARD_BALANCED) return fail(RP_EINVAL, "shard_map must be RP_SHARD_INTERLEAVE or RP_SHARD_BALANCED");
  t.balanced = p->shard_map == RP_SHARD_BALANCED && t.n_tiles <= (uint32_t)rpk::TILE_SORT_MAX;
  return RP_OK;
}

// Scatter a compact shard buffer into a frame on the host (rp_shard_unpack), tiles dealt by `map` (the deal order
// of a balanced plan) or the interleave (map NULL).
void unpack_host(const rp_render_params* p, const Tiling& t, const uint32_t* map, const void* shard_buf, size_t elem,
                 uint32_t channels, void* frame) {
  const uint64_t tile_px = (uint64_t)t.tw * t.th;
  const char* src = static_cast<const char*>(shard_buf);
  char* dst = static_cast<char*>(frame);
  for (uint32_t k = 0; k < t.n_shard_tiles; k++) {
    const uint32_t dk = t.shard + k * t.shards, tile = map ? map[dk] : dk;
    const uint32_t ox = (tile % t.tiles_x) * t.tw, oy = (tile / t.tiles_x) * t.th;
    for (uint32_t lj = 0; lj < t.th && oy + lj < p->height; lj++)
      for (uint32_t li = 0; li < t.tw && ox + li < p->width; li++)
        std::memcpy(dst + ((uint64_t)(oy + lj) * p->width + ox + li) * channels * elem,
                    src + (k * tile_px + (uint64_t)lj * t.tw + li) * channels * elem, channels * elem);
  }
}

// The workspace's learned cost table describes frames of params' geometry.
bool fcost_matches(const rp_workspace* w, const rp_render_params* p, const Tiling& t) {
  return w->fcost_valid && w->fcost_geom[0] == p->width && w->fcost_geom[1] == p->height && w->fcost_geom[2] == t.tw &&
         w->fcost_geom[3] == t.th;
}

void set_fcost(rp_workspace* w, const rp_render_params* p, const Tiling& t, uint32_t ranks) {
  w->fcost_valid = true;
  const uint32_t geom[4] = {p->width, p->height, t.tw, t.th};
  std::memcpy(w->fcost_geom, geom, sizeof geom);
  w->fcost_ranks = ranks;
}

// The workspace's plan applies to frames of params' geometry (the render of this frame's shard made it).
bool plan_matches(const rp_workspace* w, const rp_render_params* p, const Tiling& t) {
  return w->plan_on && w->plan_geom[0] == p->width && w->plan_geom[1] == p->height && w->plan_geom[2] == t.tw &&
         w->plan_geom[3] == t.th && w->plan_geom[4] == t.shards;
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

rp_scene_options default_options() {
  rp_scene_options o{};
  o.builder = RP_BUILDER_AUTO;
  o.max_leaf = DEF_MAX_LEAF;
  o.cost_traverse = DEF_COST_TRAVERSE;
  o.always_max = (int32_t)DEF_ALWAYS_MAX;
  o.lds_depth = 0;
  o.self_check = 0;
  o.trav_threshold = 0;  // auto (scene_create): DEF_TRAV_THRESHOLD, or 32 for scenes past the Infinity Cache
  o.tile_order = 0;
  o.probe_n = rpk::PROBE_LATTICE_N;
  o.debug_stack_depth = 0;
  return o;
}

// Zero fields -> defaults; range checks.
int resolve_options(const rp_scene_options* in, rp_scene_options& o) {
  const rp_scene_options d = default_options();
  o = in ? *in : d;
  if (o.builder > RP_BUILDER_PLOC) return fail(RP_EINVAL, "options.builder must be RP_BUILDER_*");
  if (o.max_leaf == 0) o.max_leaf = d.max_leaf;
  if (o.max_leaf > rpl::LEAF_MAX) return fail(RP_EINVAL, "options.max_leaf must be 1..8");
  if (o.cost_traverse == 0.0) o.cost_traverse = d.cost_traverse;
  if (!(o.cost_traverse > 0.0) || !std::isfinite(o.cost_traverse)) return fail(RP_EINVAL, "options.cost_traverse must be > 0");
  if (o.always_max < 0) o.always_max = d.always_max;
  if (o.lds_depth != 0 && o.lds_depth < 8) return fail(RP_EINVAL, "options.lds_depth must be 0 or >= 8");
  if (o.trav_threshold > 64) return fail(RP_EINVAL, "options.trav_threshold must be 1..64");
  if (o.tile_order > RP_TILES_PROBE) return fail(RP_EINVAL, "options.tile_order must be RP_TILES_*");
  if (o.probe_n == 0) o.probe_n = d.probe_n;
  if (o.node_format > RP_NODES_W8) return fail(RP_EINVAL, "options.node_format must be RP_NODES_*");
  if (o.leaf_break > 64) return fail(RP_EINVAL, "options.leaf_break must be 0..64");
  if (o.unit_queues > RP_QUEUES_XCD_REGIONS) return fail(RP_EINVAL, "options.unit_queues must be RP_QUEUES_*");
  if (o.queue_chunk > 4096) return fail(RP_EINVAL, "options.queue_chunk must be 0..4096");
  if (o.debug_stack_depth != 0 && (o.debug_stack_depth < 8 || o.debug_stack_depth > 4096))
    return fail(RP_EINVAL, "options.debug_stack_depth must be 0 or 8..4096");
  if (o.collapse > RP_COLLAPSE_SAH) return fail(RP_EINVAL, "options.collapse must be RP_COLLAPSE_*");
  if (o.node_layout > RP_LAYOUT_DFS_LINE) return fail(RP_EINVAL, "options.node_layout must be RP_LAYOUT_*");
  if (o.unit_order > RP_UNITS_LEARNED) return fail(RP_EINVAL, "options.unit_order must be RP_UNITS_*");
  return RP_OK;
}

// Slots per rank buffer of a gathered frame: shard 0 holds the most tiles (one rank: the whole frame).
uint64_t stage_slots(const Tiling& t) {
  const uint32_t n0 = t.n_tiles ? (t.n_tiles + t.shards - 1) / t.shards : 0;
  return (uint64_t)n0 * t.tw * t.th;
}

// The learned per-unit order (rp.h RP_UNITS_*) for frames of nbatch sample streams per pixel: LEARNED always, AUTO
// for one stream per pixel (nbatch 1).  Measured with round 6's bucket fix (profiles/r6/c3_unit_order_fix_ab.json,
// lone C3 frames): one stream per pixel 220.1 ms against 260.8 ms in tile order -- the longest pixels (glass-bunny
// paths of ~2,000 rays) start first instead of ending the frame -- while 32-sample streams lose 4.4 % (213.8 vs 204.8:
// a wave's units become pixels scattered over the frame, and their 8 short streams leave no long tail to fix).
bool units_on(const rp_scene* s, uint32_t nbatch) {
  return s->opt.unit_order == RP_UNITS_LEARNED || (s->opt.unit_order == RP_UNITS_AUTO && nbatch == 1);
}

// Words of a rank's packed gather block (rpk::launch_gather_pack): the counter block and 2 x tiles per rank of measured
// costs (rounded up to even), then, when the frame gathers BGRA8, the shard's bytes (rounded up to even: every block
// starts 8-byte aligned for the u64 counters).
uint64_t pack_head(const Tiling& t) {
  const uint64_t st = (t.n_tiles + t.shards - 1) / t.shards;
  return 2ull * rpk::GATHER_CTR + ((2 * st + 1) & ~1ull);
}
uint64_t bgra_words(const Tiling& t) { return (stage_slots(t) + 1) & ~1ull; }
// (a gather of n frames' shards -- rp_frames_gather -- packs their BGRA8 bytes one after the other behind one head)
uint64_t pack_words(const Tiling& t, bool bgra, uint32_t n_frames = 1) {
  return pack_head(t) + (bgra ? n_frames * bgra_words(t) : 0ull);
}

// Grow a pair of device buffers (a, b) of na, nb elements per unit to `units` units (synchronous).
template <class A, class B>
int grow(A*& a, B*& b, uint64_t& cap, uint64_t units, uint64_t na, uint64_t nb, const char* what) {
  if (units <= cap) return RP_OK;
  dfree(a);
  dfree(b);
  a = nullptr;
  b = nullptr;
  cap = 0;
  if (!dalloc(&a, na * units) || !dalloc(&b, nb * units)) return fail(RP_ENOMEM, std::string("hipMalloc ") + what);
  cap = units;
  return RP_OK;
}

// Grow the workspace's reservation for renders of params' shape (synchronous): the multi-batch sums and,
// with `gather`, the staging and receive buffers of rp_frame_gather.
int ws_reserve(rp_scene* s, rp_workspace* w, const rp_render_params* p, bool gather, uint32_t n_frames = 1) {
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (n_frames == 0 || n_frames > RP_MAX_FRAMES) return fail(RP_EINVAL, "n_frames must be 1..RP_MAX_FRAMES");
  DeviceGuard g(s->device);
  const uint64_t units = t.nbatch > 1 ? t.n_slots * t.nbatch * n_frames : 0;
  if ((rc = grow(w->d_partial, w->d_partial_hits, w->partial_units, units, 3, 1, "sample-batch workspace"))) return rc;
  // the learned per-unit order: 4 + 8 + 8 + 4 bytes per unit and the sort's scratch (C3 one stream: 2.1 M units, 50 MB)
  const uint64_t n_units = t.n_slots * t.nbatch;
  if (units_on(s, t.nbatch) && n_units > w->ucost_cap && n_units < (1ull << 31)) {
    for (void* q : {(void*)w->d_ucost, (void*)w->d_ukey, (void*)w->d_ukey2, (void*)w->d_uorder, w->d_usort}) dfree(q);
    w->d_ucost = w->d_uorder = nullptr;
    w->d_ukey = w->d_ukey2 = nullptr;
    w->d_usort = nullptr;
    w->ucost_cap = 0;
    w->ucost_valid = false;
    w->usort_bytes = rpk::unit_order_scratch_bytes(n_units);
    if (!w->usort_bytes || !dalloc(&w->d_ucost, n_units) || !dalloc(&w->d_ukey, n_units) || !dalloc(&w->d_ukey2, n_units) ||
        !dalloc(&w->d_uorder, n_units) || !dalloc(reinterpret_cast<uint8_t**>(&w->d_usort), w->usort_bytes))
      return fail(RP_ENOMEM, "hipMalloc per-unit order");
    RP_HIP(hipMemset(w->d_ucost, 0, sizeof(uint32_t) * n_units));
    w->ucost_cap = n_units;
  }
  if (gather) {
    const uint64_t stride = stage_slots(t);
    auto grow1 = [&](auto*& b, uint64_t& cap, uint64_t want, const char* what) -> int {
      if (want <= cap) return RP_OK;
      dfree(b);
      b = nullptr;
      cap = 0;
      if (!dalloc(&b, want)) return fail(RP_ENOMEM, std::string("hipMalloc ") + what);
      cap = want;
      return RP_OK;
    };
    uint64_t rgb_cap = w->gs_slots * 3, rgb_g_cap = w->gather_slots * 3;
    if ((rc = grow1(w->d_gs_rgb, rgb_cap, stride * 3, "gather staging"))) return rc;
    if ((rc = grow1(w->d_gather_rgb, rgb_g_cap, stride * t.shards * 3, "gather buffers"))) return rc;
    w->gs_slots = rgb_cap / 3;
    w->gather_slots = rgb_g_cap / 3;
    const uint64_t pw = pack_words(t, true, n_frames);  // rp_frames_gather: all of a launch's frames in one block
    if ((rc = grow1(w->d_pack_send, w->pack_words, pw, "gather block"))) return rc;
    if ((rc = grow1(w->d_pack_recv, w->pack_recv_words, pw * t.shards, "gathered blocks"))) return rc;
  }
  return RP_OK;
}

size_t rp_node_bytes(uint32_t node_format) {
  return node_format == rpl::NODES_W8 ? sizeof(rpl::Node8Q) : node_format == rpl::NODES_Q8 ? sizeof(rpl::Node4Q) : sizeof(rpl::Node4);
}

int scene_create(const rp_scene_desc* desc, int device, const rp_scene_options* opt_in, rp_scene** out) {
  if (!out) return fail(RP_EINVAL, "out is NULL");
  *out = nullptr;
  rp_scene_options opt;
  int rc = resolve_options(opt_in, opt);
  if (rc) return rc;
  std::string err;
  const auto t_start = std::chrono::steady_clock::now();
  auto lap = [t = t_start]() mutable {
    const auto now = std::chrono::steady_clock::now();
    const double d = std::chrono::duration<double>(now - t).count();
    t = now;
    return d;
  };
  double phase[RP_BUILD_PHASES] = {0};
  rc = rpb::validate(desc, err);
  if (rc != RP_OK) return fail(rc, err);
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(RP_ENODEV, "no HIP device");
  if (device < 0 || device >= ndev) return fail(RP_EINVAL, "device index out of range");
  hipDeviceProp_t prop;
  RP_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(RP_ENODEV, std::string("librp.so is built for gfx950, device is ") + prop.gcnArchName);

  rpb::PackedScene ps;
  rpb::BuildOptions bo;
  // AUTO = the device PLOC build for scenes of >= 2^21 hittables (C5, 10 M triangles: its tree renders within
  // 1.5 % of the host binned SAH's and builds in a fraction of the host's 2.7 s), the host binned
  // SAH below (small scenes build in milliseconds, and only the host keeps always-tested primitives out of the
  // tree) and for 8-wide nodes; the LBVH stays an option (fastest build, ~46 % slower tree on C5).
  if (opt.builder == RP_BUILDER_AUTO && desc->n_hittables >= rpb::Q8_MIN_PRIMS && opt.node_format != RP_NODES_W8)
    opt.builder = RP_BUILDER_PLOC;
  const bool gpu_build = opt.builder == RP_BUILDER_DEVICE || opt.builder == RP_BUILDER_PLOC;
  const bool use_gpu = gpu_build && desc->n_hittables >= 2;  // the LBVH needs two primitives
  if (gpu_build && opt.node_format == RP_NODES_W8)
    return fail(RP_EINVAL, "the device builder makes 4-wide trees (options.node_format RP_NODES_F32 or RP_NODES_Q8)");
  bo.tables_only = use_gpu;
  bo.vertex_tables = false;  // uploaded straight from the meshes below
  bo.max_leaf = opt.max_leaf;
  bo.cost_traverse = opt.cost_traverse;
  bo.always_max = (uint32_t)opt.always_max;
  bo.collapse = opt.collapse == RP_COLLAPSE_GREEDY ? rpb::COLLAPSE_GREEDY : rpb::COLLAPSE_SAH;
  bo.node_format = opt.node_format;  // RP_NODES_AUTO (0) resolved by the builder
  phase[0] = lap();
  rc = rpb::build(desc, bo, ps, err);
  if (rc != RP_OK) return fail(rc, err);
  phase[1] = lap();

  DeviceGuard g(device);
  rp_scene* s = new rp_scene();
  s->device = device;
  s->opt = opt;
  s->num_cu = prop.multiProcessorCount;
  auto bail = [&](int code) { rp_scene_destroy(s); return code; };
  uint64_t n_tree_nodes = ps.n_nodes(), n_tree_prims = ps.prims.size();
  uint32_t node_format = ps.node_format;
  if (use_gpu) {
    rpb::PrimInput pin;
    if ((rc = rpb::prim_input(desc, pin, err))) return bail(fail(rc, err));
    phase[2] = lap();
    // AUTO: f32 for the LBVH (rp_bvh.h); the PLOC tree has the SAH tree's node count, so the host trees' size rule
    node_format = opt.node_format ? opt.node_format
                  : opt.builder == RP_BUILDER_PLOC ? rpb::auto_node_format(desc->n_hittables, pin.amax)
                                                   : (uint32_t)rpl::NODES_F32;
    rpg::GpuTree gt;
    const uint32_t algo = opt.builder == RP_BUILDER_PLOC ? rpg::GPU_PLOC : rpg::GPU_LBVH;
    // node families on 128-B lines (RP_LAYOUT_DFS_LINE) for 64-B quantized nodes; f32 nodes are a line each
    const uint32_t align = opt.node_layout == RP_LAYOUT_DFS_LINE && node_format == rpl::NODES_Q8 ? 2u : 1u;
    if ((rc = rpg::build_gpu(pin, opt.max_leaf, node_format, algo, opt.cost_traverse, align, gt, err)))
      return bail(fail(rc, err));
    s->d_nodes = gt.d_nodes;
    s->d_prims = gt.d_prims;
    s->d_prim_refs = gt.d_prim_refs;
    ps.root = 0;
    ps.max_depth = gt.max_depth;
    ps.n_leaves = gt.n_leaves;
    ps.qbound = gt.qbound;
    ps.node_format = node_format;
    n_tree_nodes = gt.n_nodes;
    n_tree_prims = pin.prims.size();
    if (opt.self_check) {
      // the structural self-check of the host builder on the device-built tree (tests)
      rpb::PackedScene chk;
      chk.node_format = node_format;
      void* host_nodes;
      if (node_format == rpl::NODES_Q8) {
        chk.qnodes.resize(n_tree_nodes);
        host_nodes = chk.qnodes.data();
      } else {
        chk.nodes.resize(n_tree_nodes);
        host_nodes = chk.nodes.data();
      }
      chk.prims.resize(n_tree_prims);
      chk.prim_refs.resize(n_tree_prims);
      RP_HIP(hipMemcpy(host_nodes, s->d_nodes, rp_node_bytes(node_format) * n_tree_nodes, hipMemcpyDeviceToHost));
      RP_HIP(hipMemcpy(chk.prims.data(), s->d_prims, sizeof(rpl::Prim) * n_tree_prims, hipMemcpyDeviceToHost));
      RP_HIP(hipMemcpy(chk.prim_refs.data(), s->d_prim_refs, sizeof(rpl::PrimRef) * n_tree_prims, hipMemcpyDeviceToHost));
      chk.root = 0;
      chk.max_depth = gt.max_depth;
      chk.n_leaves = gt.n_leaves;
      chk.qbound = gt.qbound;
      if ((rc = rpb::check(chk, err))) return bail(fail(rc, "device BVH self-check: " + err));
    }
  } else if ((rc = node_format == rpl::NODES_W8   ? upload(ps.wnodes, (rpl::Node8Q**)&s->d_nodes)
                   : node_format == rpl::NODES_Q8 ? upload(ps.qnodes, (rpl::Node4Q**)&s->d_nodes)
                                                  : upload(ps.nodes, (rpl::Node4**)&s->d_nodes)) ||
             (rc = upload(ps.prims, &s->d_prims)) ||
             (rc = upload(ps.prim_refs, &s->d_prim_refs))) {
    return bail(rc);
  }
  phase[3] = lap();  // the device build, or the host tree's upload
  // vertex normals and uvs (read at a closest hit), mesh after mesh from the caller's arrays: no host copy
  uint64_t n_vert = 0;
  for (uint32_t i = 0; i < desc->n_meshes; i++) n_vert += desc->meshes[i].n_vertices;
  if (!dalloc(&s->d_vnrm, 3 * n_vert + 3) || !dalloc(&s->d_vuv, 2 * n_vert + 2)) return bail(fail(RP_ENOMEM, "hipMalloc vertex tables"));
  for (uint64_t i = 0, vb = 0; i < desc->n_meshes; vb += desc->meshes[i].n_vertices, i++) {
    const rp_mesh& m = desc->meshes[i];
    if (!m.n_vertices) continue;
    if (hipMemcpy(s->d_vnrm + 3 * vb, m.normals, sizeof(double) * 3 * m.n_vertices, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(s->d_vuv + 2 * vb, m.uvs, sizeof(double) * 2 * m.n_vertices, hipMemcpyHostToDevice) != hipSuccess)
      return bail(fail(RP_EHIP, "vertex table upload"));
  }
  if ((rc = upload(ps.materials, &s->d_mats)) || (rc = upload(ps.textures, &s->d_texs)) ||
      (rc = upload(ps.texels, &s->d_texels)))
    return bail(rc);
  if (!dalloc(&s->d_diag, rpk::DIAG_N) || hipMemset(s->d_diag, 0, sizeof(uint64_t) * rpk::DIAG_N) != hipSuccess)
    return bail(fail(RP_ENOMEM, "hipMalloc diagnostics"));
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
  s->ks.qbound = ps.qbound;
  s->ks.node_format = node_format;
  // a wide node pushes at most 3 entries (its non-nearest hits) per level below the root; +3 spare
  // entries for the kernel's branchless push (rp_kernel.hip STACK_SLACK)
  s->ks.stack_depth = 3 * ps.max_depth + 4 + 3;
  // Node8Q: groups of two words, per level at most the rest of a node group and one primitive group
  if (node_format == rpl::NODES_W8) s->ks.stack_depth = 4 * (ps.max_depth + 1) + 3;
  // floor of 17 entries: the spill split below never keeps fewer in LDS (options.lds_depth tests force 17)
  if (s->ks.stack_depth < 17) s->ks.stack_depth = 17;
  // test-only: a stack too small for the tree (the kernels flag RP_STATUS_STACK_OVERFLOW, never write past it)
  const bool debug_stack = opt.debug_stack_depth != 0;
  if (debug_stack) s->ks.stack_depth = opt.debug_stack_depth;
  s->n_nodes = n_tree_nodes;
  s->n_leaves = ps.n_leaves;
  s->n_prims = desc->n_hittables;
  s->max_depth = ps.max_depth;
  s->device_bytes = rp_node_bytes(node_format) * n_tree_nodes + (sizeof(rpl::Prim) + sizeof(rpl::PrimRef)) * n_tree_prims +
                    sizeof(double) * 5 * n_vert + sizeof(rpl::Material) * ps.materials.size() +
                    sizeof(rpl::Texture) * ps.textures.size() + sizeof(uint32_t) * ps.texels.size();
  // Cost-ordered tiles for every scene: cache-resident scenes (C3: 11 MB) gain ~15 % from them (short frame tail);
  // past the 256 MB Infinity Cache (C5: 2.5 GB) the Z-order once won (one device-wide queue: cost order scattered the
  // tiles in flight, +7 %), but with per-XCD queues and costs learned from the previous frame the cost order is even
  // or better there too (round 4: C5 -0.8 % on one box, -7.5 % on another, where the Z-order ran 11 % slower than
  // usual).  MORTON stays an option, and with it the balanced plan's square tile blocks.
  s->tiles_auto = RP_TILES_COST;
  // the speculative-traversal exit: C3 246.3 ms at 8 (3: 248.2, 12: 248.5); C5 at 16 (per-XCD queues, ab34: 12 +0.4 %,
  // 20 +0.1 %, 24 +0.7 %)
  s->ks.leaf_break = opt.leaf_break ? opt.leaf_break : (s->device_bytes > (256ull << 20) ? 16u : 8u);
  // lanes still traversing before the finished ones shade: C3 24 (16: +0.2 %, 32: +0.7 %), C5 32 (-1.6 %)
  if (s->opt.trav_threshold == 0) s->opt.trav_threshold = s->device_bytes > (256ull << 20) ? 32u : DEF_TRAV_THRESHOLD;
  // LDS holds the whole stack unless that costs resident blocks: then the deepest entries spill to a
  // per-lane global run (rp_kernel.hip stk_put/stk_get) and LDS keeps the largest depth that still fits
  // the occupancy of a shallow stack (C5's 43-entry stack: 3 -> 4 blocks per CU).  options.lds_depth
  // forces a depth (>= 17) for tests and tuning.
  s->ks.lds_depth = s->ks.stack_depth;
  int bpc = 0;
  if (rpk::render_blocks_per_cu(s->ks.stack_depth, false, node_format, &bpc) != 0 || bpc < 1) bpc = 1;
  int bpc_spill = 0;
  if (!debug_stack && rpk::render_blocks_per_cu(17, true, node_format, &bpc_spill) == 0 && bpc_spill > bpc) {
    uint32_t L = s->ks.stack_depth - 1;
    int b = 0;
    while (L > 17 && (rpk::render_blocks_per_cu(L, true, node_format, &b) != 0 || b < bpc_spill)) L--;
    s->ks.lds_depth = L;
    bpc = bpc_spill;
  }
  if (!debug_stack && opt.lds_depth && opt.lds_depth < s->ks.stack_depth) {
    s->ks.lds_depth = opt.lds_depth;
    if (rpk::render_blocks_per_cu(opt.lds_depth, true, node_format, &bpc) != 0 || bpc < 1) bpc = 1;
  }
  s->blocks_per_cu = bpc;
  phase[4] = lap();
  if ((rc = ws_alloc(s, &s->ws0))) return bail(rc);
  phase[5] = lap();
  std::memcpy(s->build_s, phase, sizeof phase);
  *out = s;
  return RP_OK;
}

// The render of one shard on `stream` (rp_render_device_ws's body).
int render_shard(rp_scene* s, rp_workspace* w, const rp_camera* cam, const rp_render_params* p, double* d_rgb,
                 float* d_fg, uint64_t* d_counters, void* stream, uint32_t n_frames = 1,
                 uint32_t frame_order = RP_FRAME_ORDER_AUTO) {
  if (!s || !cam || !d_rgb) return fail(RP_EINVAL, "scene, camera and output must be non-NULL");
  if (!w || w->scene != s) return fail(RP_EINVAL, "workspace is NULL or belongs to another scene");
  w->frame_flags = 0;  //  before any return: an spp = 0 or refused render reports no scheduling
  if (n_frames == 0 || n_frames > RP_MAX_FRAMES) return fail(RP_EINVAL, "n_frames must be 1..RP_MAX_FRAMES");
  if (frame_order > RP_FRAME_ORDER_PIXEL) return fail(RP_EINVAL, "frame_order must be an RP_FRAME_ORDER_* value");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (p->max_bounce < 1) return fail(RP_EINVAL, "max_bounce must be >= 1 (render.rs:97 assert!(depth >= 1))");
  DeviceGuard g(s->device);
  uint64_t* ctr = d_counters ? d_counters : w->d_ctr;
  hipStream_t st = (hipStream_t)stream;
  // the last frame gather on this workspace (another stream, perhaps) has read d_meas and written d_fcost
  if (w->gathered_pending) {
    RP_HIP(hipStreamWaitEvent(st, w->ev_gathered, 0));
    w->gathered_pending = false;
  }
  RP_HIP(hipMemsetAsync(ctr, 0, sizeof(uint64_t) * rpk::CTR_N, st));
  if (t.n_slots == 0) return RP_OK;
  if (p->spp == 0) {
    // main.rs:86-87 with num_samples = 0: (0,0,0) / 0 and 0 / 0 are NaN; all-ones bits are a NaN.
    RP_HIP(hipMemsetAsync(d_rgb, 0xff, sizeof(double) * 3 * t.n_slots * n_frames, st));
    if (d_fg) RP_HIP(hipMemsetAsync(d_fg, 0xff, sizeof(float) * t.n_slots * n_frames, st));
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
  kp.trav_threshold = s->opt.trav_threshold;
  kp.spp_batch = t.sps;  // the RNG contract's samples per stream (rp_render_params.samples_per_stream)
  kp.nbatch = t.nbatch;
  kp.n_queue = t.n_slots * kp.nbatch * n_frames;  // every frame's units
  kp.n_frames = n_frames;
  kp.dv_tiles = rpk::make_div32(std::max(1u, t.n_shard_tiles));
  kp.dv_frames = rpk::make_div32(n_frames);
  kp.frames_inter = n_frames > 1 && frame_order != RP_FRAME_ORDER_SEQUENTIAL ? 1u : 0u;
  kp.out_stride = 3 * t.n_slots;
  // Per-XCD queues (rp.h RP_QUEUES_*): groups of blocks blockIdx mod 8 share an XCD (MI355X_MICROARCH.md,
  // observed round-robin dispatch; speed only -- any placement gives the same image).
  uint32_t qmode = s->opt.unit_queues == RP_QUEUES_AUTO ? (uint32_t)DEF_UNIT_QUEUES : s->opt.unit_queues;
  kp.queue_groups = qmode == RP_QUEUES_SINGLE ? 1u : (uint32_t)rpk::QUEUE_GROUPS;
  // Default chunk: up to 8 consecutive (virtual) tiles of the order per queue at a time, while every queue still gets >= 16
  // chunks -- the tiles one XCD runs together are then neighbours in cost and, inside a cost bucket, in Z-order (a whole C3
  // frame, 2,040 tiles: chunks of 8, -1.0 % against chunks of one; an 8-way shard, 255 tiles: chunks of one, 8 cost
  // +3.8 % at one frame per launch); with interleaved frames a whole number of tiles of every frame (n_frames >= 8: one
  // tile of every frame, so one XCD renders a tile for all the launch's frames and its L2 serves the same pixels' rays
  // n_frames times: C3 -1.3 %, 8-way shards -1.9 %)
  const uint64_t vtiles = (uint64_t)t.n_shard_tiles * n_frames;
  uint32_t chunk_auto = 1;
  while (chunk_auto < QUEUE_CHUNK_AUTO && 2ull * chunk_auto * 8 * 16 <= vtiles) chunk_auto *= 2;
  if (kp.frames_inter) chunk_auto = n_frames * ((chunk_auto + n_frames - 1) / n_frames);
  kp.queue_chunk = qmode == RP_QUEUES_XCD_REGIONS ? (t.n_shard_tiles + kp.queue_groups - 1) / kp.queue_groups
                  : kp.queue_groups > 1 ? (s->opt.queue_chunk ? s->opt.queue_chunk : chunk_auto) : 1u;
  if (kp.queue_chunk == 0) kp.queue_chunk = 1;
  // RP_FRAME_ORDER_PIXEL needs a queue's runs of n_frames virtual tiles to be one tile of every frame: single queue, or
  // chunks of whole multiples of n_frames (the default chunk is); otherwise it is INTERLEAVED
  if (kp.frames_inter && frame_order == RP_FRAME_ORDER_PIXEL && (kp.queue_groups == 1 || kp.queue_chunk % n_frames == 0))
    kp.frames_inter = 2;
  // a 32-bit queue word takes its units, plus one failed fetch per resident lane after the last unit (single
  // queue) or one per fetch that passes a drained queue on the way to another (per-XCD queues)
  if ((kp.queue_groups > 1 ? 2 * kp.n_queue : kp.n_queue) + s->lanes() >= 0xffffffffull)
    return fail(RP_EINVAL, "shard too large (>= 2^32 pixel-batch units with the resident lanes)");
  // the unit decode divides by launch constants with 31-bit numerators (rpk::make_div32)
  if (kp.n_queue >= (1ull << 31)) return fail(RP_EINVAL, "shard too large (>= 2^31 pixel-batch units)");
  kp.dv_units = rpk::make_div32(t.tw * t.th * kp.nbatch);
  kp.dv_nbatch = rpk::make_div32(kp.nbatch ? kp.nbatch : 1u);
  kp.dv_tiles_x = rpk::make_div32(t.tiles_x);
  kp.dv_tw = rpk::make_div32(t.tw);
  kp.dv_chunk = rpk::make_div32(kp.queue_chunk);
  if (kp.nbatch > 1) {
    if (kp.n_queue > w->partial_units)
      return fail(RP_EINVAL, n_frames > 1 ? "workspace not reserved for these frames' sample batches: call "
                                            "rp_workspace_reserve_frames"
                                          : "workspace not reserved for this frame's sample batches: call rp_workspace_reserve");
    kp.partial = w->d_partial;
    kp.partial_hits = w->d_partial_hits;
  }
  const uint64_t resident = (uint64_t)s->num_cu * (uint64_t)s->blocks_per_cu;
  rpk::KScene ks = s->ks;
  ks.rng_slab = w->d_slab;
  ks.spill = w->d_spill;
  ks.unit_t0 = w->d_t0;
  auto grid_for = [&](uint64_t slots) {
    const uint64_t want = (slots + rpk::RENDER_BLOCK - 1) / rpk::RENDER_BLOCK;
    return (int)std::max<uint64_t>(1, std::min(want, resident));
  };
  RP_HIP(hipMemsetAsync(w->d_queue, 0, sizeof(uint32_t) * rpk::QUEUE_WORDS, st));
  const uint32_t tiles_y = t.tiles_y;
  uint32_t order_mode = s->opt.tile_order;
  if (order_mode == RP_TILES_AUTO) order_mode = s->tiles_auto;
  // The cost probe: sample 0 of an n x n lattice of pixels per tile traced by the probe instantiation of the
  // render kernel, which adds up per tile the traversal work and shaded rays (summed and costliest sample) --
  // over the shard's tiles, or over the whole frame for a balanced plan (same stream, no host sync).
  auto probe = [&](uint32_t shard, uint32_t nshards, uint32_t n_tiles, uint32_t lattice, uint32_t& probe_px) -> int {
    rpk::KParams pk = kp;
    pk.probe = 1;
    pk.spp = 1;
    pk.n_frames = 1;
    pk.shard = shard;
    pk.nshards = nshards;
    pk.n_shard_tiles = n_tiles;
    pk.probe_n = std::min(lattice, std::min(t.tw, t.th));
    pk.probe_px = pk.probe_n * pk.probe_n;
    pk.n_slots = (uint64_t)n_tiles * pk.probe_px;
    pk.nbatch = 1;
    pk.spp_batch = 1;
    pk.n_queue = pk.n_slots;
    pk.queue_groups = 1;
    pk.queue_chunk = 1;
    pk.tile_cost = w->d_tile_cost;
    pk.tile_order = nullptr;
    pk.tile_map = nullptr;
    probe_px = pk.probe_px;
    RP_HIP(hipMemsetAsync(w->d_probe_ctr, 0, sizeof(uint64_t) * rpk::CTR_N, st));
    w->frame_flags |= RP_FRAME_PROBED;
    RP_HIP(hipMemsetAsync(w->d_tile_cost, 0, sizeof(uint32_t) * 2 * rpk::TILE_SORT_MAX, st));
    int e = rpk::launch_render(ks, pk, d_rgb, nullptr, w->d_probe_ctr, w->d_queue + rpk::QUEUE_PROBE, grid_for(pk.n_slots), stream);
    if (e != 0) return fail(RP_EHIP, std::string("probe launch: ") + hipGetErrorString((hipError_t)e));
    return RP_OK;
  };
  // both sorts key the tiles by their Z-order code (frame grids up to 256 x 256 tiles; larger ones keep shard
  // order)
  const bool sortable = t.n_shard_tiles > 1 && t.n_shard_tiles <= rpk::TILE_SORT_MAX && t.tiles_x <= 256 &&
                        tiles_y <= 256;
  rpk::TileGeom tg{t.tiles_x, kp.shard, kp.nshards, nullptr, 0, 0};
  uint32_t probe_px = 0;
  const uint32_t* frame_cost = nullptr;  // per-frame-tile costs (sum, max) the plan and the shard order use
  w->plan_on = false;
  // Scheduling costs.  The megakernel measures every unit's duration into its tile's cost (kp.tile_meas); once a
  // frame of this geometry has been rendered whole on one device, or gathered from all ranks, the workspace holds a
  // learned per-tile table and the next frame schedules from it -- no probe launch.  For a balanced plan over
  // N > 1 ranks the table must come from a gather over the same N ranks: every rank then holds the same bytes and
  // deals the same plan.  Otherwise a probe (the first frame) supplies the costs.
  // (the measured table holds TILE_SORT_MAX tiles: a shard of more tiles -- 8 x 8 tiles at 1080p, say -- is not
  // measured, and its frame keeps the probe / interleave)
  const bool measure = t.n_shard_tiles <= (uint32_t)rpk::TILE_SORT_MAX;
  const bool probe_order = order_mode == RP_TILES_PROBE;
  if (probe_order) order_mode = RP_TILES_COST;
  const bool learned = measure && !probe_order && fcost_matches(w, p, t);
  const uint32_t learned_px = t.tw * t.th * std::max(1u, t.nbatch);  // units per tile: sum / units = mean unit
  if (learned) w->frame_flags |= RP_FRAME_LEARNED_ORDER;
  if (t.balanced) {
    // RP_SHARD_BALANCED: deal the frame's tiles to the ranks by cost (rpk::launch_tile_plan).  Without a learned
    // table, probe the whole frame (deterministic costs, rp_device.h trav_step COUNT); scenes past the Infinity
    // Cache (Z-order tiles, no cost order inside the shard) probe a sparser 4 x 4 lattice.
    if (learned && (t.shards == 1 || w->fcost_ranks == t.shards)) {
      frame_cost = w->d_fcost;
      probe_px = learned_px;
    } else {
      const uint32_t lattice = order_mode == RP_TILES_COST ? s->opt.probe_n : std::min(s->opt.probe_n, 4u);
      if ((rc = probe(0, 1, t.n_tiles, lattice, probe_px))) return rc;
      frame_cost = w->d_tile_cost;
    }
    // Z-order tiles (tile_order = MORTON, on request only) deal square blocks of tiles: a rank's tiles stay in compact
    // squares of the frame, so its working set does too (C5 8-way shards: DESIGN.md 6); the cost order (AUTO, every
    // scene) deals tile by tile
    const uint32_t block = order_mode == RP_TILES_MORTON ? plan_block(t.n_tiles, t.shards) : 1u;
    int e = rpk::launch_tile_plan(frame_cost, t.n_tiles, t.shards, t.tiles_x, block, w->d_plan, w->d_sort, stream);
    if (e != 0) return fail(RP_EHIP, std::string("tile plan launch: ") + hipGetErrorString((hipError_t)e));
    kp.tile_map = w->d_plan;
    tg.map = w->d_plan;
    tg.map_tiles = t.n_tiles;
    w->plan_on = true;
    const uint32_t geom[5] = {p->width, p->height, t.tw, t.th, t.shards};
    std::memcpy(w->plan_geom, geom, sizeof geom);
  } else if (learned) {
    frame_cost = w->d_fcost;  // the shard order only: no agreement between ranks needed
    probe_px = learned_px;
  }
  if (order_mode == RP_TILES_MORTON && sortable) {
    int e = rpk::launch_tile_sort(nullptr, t.n_shard_tiles, 1, tg, w->d_tile_order, w->d_sort, stream);
    if (e != 0) return fail(RP_EHIP, std::string("tile sort launch: ") + hipGetErrorString((hipError_t)e));
    kp.tile_order = w->d_tile_order;
  }
  if (order_mode == RP_TILES_COST && sortable) {
    // the shard's tiles by cost: the learned table or the balanced plan's frame probe, else a probe of the shard
    if (!frame_cost && (rc = probe(kp.shard, kp.nshards, t.n_shard_tiles, s->opt.probe_n, probe_px))) return rc;
    tg.cost_by_tile = frame_cost ? 1u : 0u;
    int e = rpk::launch_tile_sort(frame_cost ? frame_cost : w->d_tile_cost, t.n_shard_tiles, probe_px, tg,
                                  w->d_tile_order, w->d_sort, stream);
    if (e != 0) return fail(RP_EHIP, std::string("tile sort launch: ") + hipGetErrorString((hipError_t)e));
    kp.tile_order = w->d_tile_order;
  }
  // The learned per-unit order (rp.h RP_UNITS_*, units_on): units longest first by the last render's durations on this
  // workspace -- same frame shape and shard, one frame per launch (or any launch under LEARNED: a unit's n_frames frames
  // are then handed out together), and not a balanced plan over several ranks (its tiles may move) -- and such renders
  // store their units' durations for the next one.  The workspace's durations and order
  // are committed only once the launch is enqueued.
  const uint64_t n_units = t.n_slots * t.nbatch;
  const uint32_t ugeom[8] = {p->width, p->height, t.tw, t.th, p->spp, t.sps, t.shard, t.shards};
  // (launches of several frames: LEARNED only -- AUTO keeps their interleaved tile order)
  const bool ufit = (n_frames == 1 || s->opt.unit_order == RP_UNITS_LEARNED) && units_on(s, t.nbatch) && w->d_ucost &&
                    n_units <= w->ucost_cap && (!t.balanced || t.shards == 1);
  bool uorder = false;
  if (ufit && w->ucost_valid && std::memcmp(ugeom, w->ucost_geom, sizeof ugeom) == 0) {
    int e = rpk::launch_unit_order(w->d_ucost, n_units, w->d_ukey, w->d_ukey2, w->d_usort, w->usort_bytes, w->d_uorder,
                                   stream);
    if (e != 0) return fail(RP_EHIP, std::string("unit order launch: ") + hipGetErrorString((hipError_t)e));
    kp.unit_order = w->d_uorder;
    kp.order_chunk = rpk::UNIT_ORDER_CHUNK;
    kp.dv_ochunk = rpk::make_div32(kp.order_chunk);
    kp.dv_tile_px = rpk::make_div32(t.tw * t.th);
    uorder = true;
  }
  if (ufit) kp.unit_cost = w->d_ucost;
  RP_HIP(hipMemsetAsync(w->d_meas, 0, sizeof(uint32_t) * 2 * rpk::TILE_SORT_MAX, st));
  kp.tile_meas = measure ? w->d_meas : nullptr;
  w->meas_on = measure;
  int e = rpk::launch_render(ks, kp, d_rgb, d_fg, ctr, w->d_queue, grid_for(kp.n_queue), stream);
  if (e != 0) {
    w->ucost_valid = false;  // the durations may be partly overwritten
    return fail(RP_EHIP, std::string("render launch: ") + hipGetErrorString((hipError_t)e));
  }
  if (uorder) w->frame_flags |= RP_FRAME_UNIT_ORDER;
  w->ucost_valid = ufit;
  if (ufit) std::memcpy(w->ucost_geom, ugeom, sizeof ugeom);
  if (kp.nbatch > 1) {
    for (uint32_t f = 0; f < n_frames; f++) {  // each frame's batch sums, added in batch order
      rpk::KParams kf = kp;
      kf.partial = kp.partial + 3 * (uint64_t)f * t.n_slots * kp.nbatch;
      kf.partial_hits = kp.partial_hits + (uint64_t)f * t.n_slots * kp.nbatch;
      e = rpk::launch_reduce_batches(kf, d_rgb + (uint64_t)f * kp.out_stride, d_fg ? d_fg + (uint64_t)f * t.n_slots : nullptr,
                                     stream);
      if (e != 0) return fail(RP_EHIP, std::string("reduce launch: ") + hipGetErrorString((hipError_t)e));
    }
  }
  // a whole frame on one device: its measured costs are the next frame's table (several ranks: the frame gather's)
  if (measure && t.shards == 1 && t.n_tiles <= (uint32_t)rpk::TILE_SORT_MAX) {
    e = rpk::launch_learn_costs(w->d_meas, w->d_meas + rpk::TILE_SORT_MAX, 0, 1, t.n_tiles, kp.tile_map, w->d_fcost,
                                stream);
    if (e != 0) return fail(RP_EHIP, std::string("cost table launch: ") + hipGetErrorString((hipError_t)e));
    set_fcost(w, p, t, 1);
  }
  return RP_OK;
}

// ---- multi-GPU frame assembly, in three phases so one thread can drive several devices (rp_multi):
// (1) stage the rank's shard (to_srgb_u8 bytes and/or a padded f64 copy), (2) the RCCL collectives,
// (3) de-interleave the gathered shards into frame order.

struct GatherPlan {
  Tiling t;
  uint64_t stride;  // slots per rank buffer
  uint32_t stride_tiles;  // tiles per rank buffer (shard 0's count)
  uint64_t head;          // words of the packed block before the BGRA8 bytes (pack_head)
  uint32_t nf;            // frames whose BGRA8 bytes the block carries (rp_frames_gather; 1 otherwise)
  rpk::FrameGeom geom;
  const uint32_t* plan_hash;  // the workspace's plan hash (balanced frames), NULL = interleave
};

int gather_plan(rp_scene* s, rp_workspace* w, int nranks, int rank, const rp_render_params* p, GatherPlan& gp,
                uint32_t nf = 1) {
  if (!s || !w || w->scene != s) return fail(RP_EINVAL, "scene / workspace mismatch");
  gp.nf = nf;
  int rc = make_tiling(p, gp.t);
  if (rc) return rc;
  if ((int)gp.t.shards != nranks || (int)gp.t.shard != rank)
    return fail(RP_EINVAL, "params.shard / num_shards must be the communicator's rank / size");
  gp.stride = stage_slots(gp.t);
  gp.stride_tiles = (gp.t.n_tiles + gp.t.shards - 1) / gp.t.shards;
  gp.head = pack_head(gp.t);
  if (gp.stride > w->gs_slots || gp.stride * (uint64_t)nranks > w->gather_slots || pack_words(gp.t, true, nf) > w->pack_words ||
      pack_words(gp.t, true, nf) * nranks > w->pack_recv_words)
    return fail(RP_EINVAL, nf > 1 ? "workspace not reserved for these frames' gather: call rp_workspace_reserve_frames"
                                  : "workspace not reserved for this frame's gather: call rp_workspace_reserve");
  gp.geom.W = p->width;
  gp.geom.H = p->height;
  gp.geom.tw = gp.t.tw;
  gp.geom.th = gp.t.th;
  gp.geom.tiles_x = gp.t.tiles_x;
  gp.geom.nranks = (uint32_t)nranks;
  gp.geom.stride = gp.stride;
  gp.geom.rank_words = 0;
  gp.geom.tile_pos = nullptr;
  gp.plan_hash = nullptr;
  if (gp.t.balanced) {
    if (!plan_matches(w, p, gp.t))
      return fail(RP_EINVAL, "balanced frame: render this rank's shard with the same workspace before gathering it");
    gp.geom.tile_pos = w->d_plan + gp.t.n_tiles;
    gp.plan_hash = w->d_plan + 2 * gp.t.n_tiles;
  }
  return RP_OK;
}

// (1) this rank's packed block for the one collective -- its counters (and plan hash), its measured tile costs, its
// to_srgb_u8 bytes -- and/or a padded f64 copy of the shard
int gather_stage(rp_scene* s, rp_workspace* w, const GatherPlan& gp, const double* d_shard_rgb, bool bgra, bool rgb,
                 const uint64_t* d_counters, hipStream_t st) {
  DeviceGuard g(s->device);
  // the measured costs travel only for frames whose tiles fit the table (gather_learn's condition)
  const uint32_t* meas = gp.t.n_tiles <= (uint32_t)rpk::TILE_SORT_MAX ? w->d_meas : nullptr;
  int e = rpk::launch_gather_pack(d_counters, gp.plan_hash, meas, gp.stride_tiles, w->d_pack_send, st);
  if (e != 0) return fail(RP_EHIP, std::string("gather pack launch: ") + hipGetErrorString((hipError_t)e));
  for (uint32_t f = 0; bgra && gp.t.n_slots && f < gp.nf; f++) {  // frame f's bytes at head + f x bgra_words
    e = rpk::launch_srgb_bgra(srgb_table(), d_shard_rgb + 3 * gp.t.n_slots * (uint64_t)f, gp.t.n_slots,
                              reinterpret_cast<uint8_t*>(w->d_pack_send + gp.head + bgra_words(gp.t) * f), st);
    if (e != 0) return fail(RP_EHIP, std::string("output stage launch: ") + hipGetErrorString((hipError_t)e));
  }
  if (rgb && gp.t.n_slots && d_shard_rgb != w->d_gs_rgb)
    RP_HIP(hipMemcpyAsync(w->d_gs_rgb, d_shard_rgb, sizeof(double) * 3 * gp.t.n_slots, hipMemcpyDeviceToDevice, st));
  return RP_OK;
}

// (2) the collectives: ONE all-gather of the packed blocks (counters -- status bits are OR-ed, not summed, and the plan
// hashes compared --, measured tile costs, BGRA8 bytes), then the f64 shards when asked for (rp.h: every rank passes
// the same NULL / non-NULL outputs, so every rank gathers the same block size).  One collective instead of four: an
// RCCL all-gather kernel on gfx950 needs 37.7 KB of LDS and 256 VGPRs per lane, so with frames in flight each one
// waits ~8-24 ms for a CU the render waves leave (profiles/r5/c3_gather_lds_wait.json).
int gather_collectives(ncclComm_t comm, rp_workspace* w, const GatherPlan& gp, bool bgra, bool rgb, hipStream_t st) {
  RP_NCCL(ncclAllGather(w->d_pack_send, w->d_pack_recv, pack_words(gp.t, bgra, gp.nf), ncclUint32, comm, st));
  if (rgb) RP_NCCL(ncclAllGather(w->d_gs_rgb, w->d_gather_rgb, 3 * gp.stride, ncclFloat64, comm, st));
  return RP_OK;
}

// (3a) the gathered tile costs -> the workspace's learned table (on every device of the frame)
int gather_learn(rp_scene* s, rp_workspace* w, const GatherPlan& gp, const rp_render_params* p, bool bgra,
                 hipStream_t st) {
  DeviceGuard g(s->device);
  if (!w->meas_on || gp.t.n_tiles > (uint32_t)rpk::TILE_SORT_MAX) {
    w->fcost_valid = false;
  } else {
    // rank r's sums at r * block + 2 GATHER_CTR, its maxima stride_tiles further
    const uint32_t* sums = w->d_pack_recv + 2 * rpk::GATHER_CTR;
    int e = rpk::launch_learn_costs(sums, sums + gp.stride_tiles, (uint32_t)pack_words(gp.t, bgra, gp.nf), gp.geom.nranks,
                                    gp.t.n_tiles, gp.t.balanced ? w->d_plan : nullptr, w->d_fcost, st);
    if (e != 0) return fail(RP_EHIP, std::string("cost table launch: ") + hipGetErrorString((hipError_t)e));
    set_fcost(w, p, gp.t, gp.geom.nranks);
  }
  // the next render on this workspace waits for the collectives (which read d_meas) and the table (ev_gathered)
  RP_HIP(hipEventRecord(w->ev_gathered, st));
  w->gathered_pending = true;
  return RP_OK;
}

// (3) counters reduced (sums, status OR), shards de-interleaved into frame order
int gather_assemble(rp_scene* s, rp_workspace* w, const GatherPlan& gp, uint8_t* d_frame_bgra, double* d_frame_rgb,
                    uint64_t* d_counters, hipStream_t st) {
  DeviceGuard g(s->device);
  const uint64_t block = pack_words(gp.t, d_frame_bgra != nullptr, gp.nf);
  int e = rpk::launch_counters_reduce(reinterpret_cast<const uint64_t*>(w->d_pack_recv), gp.geom.nranks, block,
                                      d_counters ? d_counters : w->d_ctr, st);
  if (e != 0) return fail(RP_EHIP, std::string("counter reduce launch: ") + hipGetErrorString((hipError_t)e));
  for (uint32_t f = 0; d_frame_bgra && f < gp.nf; f++) {  // frame f into its own W x H x 4 bytes
    rpk::FrameGeom fg = gp.geom;
    fg.rank_words = block;
    e = rpk::launch_frame_assemble(fg, w->d_pack_recv + gp.head + bgra_words(gp.t) * f, 1,
                                   reinterpret_cast<uint32_t*>(d_frame_bgra + 4ull * gp.geom.W * gp.geom.H * f), st);
    if (e != 0) return fail(RP_EHIP, std::string("frame assembly launch: ") + hipGetErrorString((hipError_t)e));
  }
  if (d_frame_rgb) {
    e = rpk::launch_frame_assemble(gp.geom, reinterpret_cast<const uint32_t*>(w->d_gather_rgb), 6,
                                   reinterpret_cast<uint32_t*>(d_frame_rgb), st);
    if (e != 0) return fail(RP_EHIP, std::string("frame assembly launch: ") + hipGetErrorString((hipError_t)e));
  }
  return RP_OK;
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

#ifndef RP_BUILD_ID
#define RP_BUILD_ID "unknown"
#endif

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
  for (void* p : {(void*)s->d_nodes, (void*)s->d_prims, (void*)s->d_prim_refs, (void*)s->d_vnrm, (void*)s->d_vuv,
                  (void*)s->d_mats, (void*)s->d_texs, (void*)s->d_texels, (void*)s->d_diag})
    dfree(p);
  delete s;
}

int rp_scene_options_init(rp_scene_options* opt) {
  if (!opt) return fail(RP_EINVAL, "opt is NULL");
  *opt = default_options();
  return RP_OK;
}

int rp_scene_create_ex(const rp_scene_desc* desc, int device, const rp_scene_options* opt, rp_scene** out) {
  return scene_create(desc, device, opt, out);
}

int rp_scene_create(const rp_scene_desc* desc, int device, rp_scene** out) {
  return scene_create(desc, device, nullptr, out);
}

int rp_scene_build_times(const rp_scene* s, double* seconds, uint32_t n) {
  if (!s || (!seconds && n)) return fail(RP_EINVAL, "NULL argument");
  for (uint32_t i = 0; i < n; i++) seconds[i] = i < (uint32_t)RP_BUILD_PHASES ? s->build_s[i] : 0.0;
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
  if (t.balanced) return fail(RP_EINVAL, "balanced frame: unpack with rp_shard_unpack_map and rp_workspace_tile_map");
  unpack_host(p, t, nullptr, shard_buf, sizeof(double), channels, frame);
  return RP_OK;
}

int rp_shard_unpack_map(const rp_render_params* p, const uint32_t* tile_map, const double* shard_buf, uint32_t channels,
                        double* frame) {
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (!shard_buf || !frame || channels == 0) return fail(RP_EINVAL, "NULL buffer or zero channels");
  if (tile_map) {
    std::vector<uint8_t> seen(t.n_tiles, 0);
    for (uint32_t i = 0; i < t.n_tiles; i++) {
      if (tile_map[i] >= t.n_tiles || seen[tile_map[i]]) return fail(RP_EINVAL, "tile_map is not a permutation of the frame's tiles");
      seen[tile_map[i]] = 1;
    }
  }
  unpack_host(p, t, tile_map, shard_buf, sizeof(double), channels, frame);
  return RP_OK;
}

int rp_workspace_tile_map(rp_scene* s, rp_workspace* w, const rp_render_params* p, uint32_t* tile_map, uint32_t n) {
  if (!s || !tile_map) return fail(RP_EINVAL, "scene and tile_map must be non-NULL");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (n < t.n_tiles) return fail(RP_EINVAL, "tile_map holds fewer entries than the frame has tiles");
  if (!t.balanced) {
    for (uint32_t i = 0; i < t.n_tiles; i++) tile_map[i] = i;
    return RP_OK;
  }
  if (!plan_matches(w, p, t)) return fail(RP_EINVAL, "no balanced plan for this frame in the workspace: render it first");
  DeviceGuard g(s->device);
  RP_HIP(hipDeviceSynchronize());
  RP_HIP(hipMemcpy(tile_map, w->d_plan, sizeof(uint32_t) * t.n_tiles, hipMemcpyDeviceToHost));
  return RP_OK;
}

int rp_workspace_frame_info(const rp_scene* s, const rp_workspace* w, uint32_t* flags) {
  if (!s || !flags) return fail(RP_EINVAL, "scene and flags must be non-NULL");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  *flags = w->frame_flags;
  return RP_OK;
}

int rp_workspace_unit_order(rp_scene* s, rp_workspace* w, uint32_t* durations, uint32_t* order, uint64_t n) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  if (n > w->ucost_cap) return fail(RP_EINVAL, "n exceeds the workspace's per-unit reservation");
  if (n == 0) return RP_OK;
  DeviceGuard g(s->device);
  RP_HIP(hipDeviceSynchronize());
  if (durations) RP_HIP(hipMemcpy(durations, w->d_ucost, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
  if (order) RP_HIP(hipMemcpy(order, w->d_uorder, sizeof(uint32_t) * n, hipMemcpyDeviceToHost));
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

int rp_workspace_reserve(rp_scene* s, rp_workspace* w, const rp_render_params* p) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  return ws_reserve(s, w, p, true);
}

int rp_render_device(rp_scene* s, const rp_camera* cam, const rp_render_params* p, double* d_rgb, float* d_fg,
                     uint64_t* d_counters, void* stream) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  return render_shard(s, &s->ws0, cam, p, d_rgb, d_fg, d_counters, stream);
}

int rp_render_device_ws(rp_scene* s, rp_workspace* w, const rp_camera* cam, const rp_render_params* p, double* d_rgb,
                        float* d_fg, uint64_t* d_counters, void* stream) {
  return render_shard(s, w, cam, p, d_rgb, d_fg, d_counters, stream);
}

int rp_workspace_reserve_frames(rp_scene* s, rp_workspace* w, const rp_render_params* p, uint32_t n_frames) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  return ws_reserve(s, w, p, true, n_frames);
}

int rp_render_frames_device_ws(rp_scene* s, rp_workspace* w, const rp_camera* cam, const rp_render_params* p,
                               uint32_t n_frames, uint32_t frame_order, double* d_rgb, float* d_fg, uint64_t* d_counters,
                               void* stream) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  if (!w) w = &s->ws0;
  return render_shard(s, w, cam, p, d_rgb, d_fg, d_counters, stream, n_frames, frame_order);
}

int rp_render(rp_scene* s, const rp_camera* cam, const rp_render_params* p, double* out_rgb, float* out_fg,
              rp_stats* stats) {
  if (!s || !cam || !out_rgb) return fail(RP_EINVAL, "scene, camera and output must be non-NULL");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if ((rc = ws_reserve(s, &s->ws0, p, false))) return rc;
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
    if (!dalloc(&d_rgb, shard.size()) || !dalloc(&d_ctr, rpk::CTR_N) || (out_fg && !dalloc(&d_fg, shard_fg.size()))) {
      result = fail(RP_ENOMEM, "hipMalloc output");
      break;
    }
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) { result = fail(RP_EHIP, "event"); break; }
    (void)hipEventRecord(e0, st);
    result = render_shard(s, &s->ws0, cam, p, d_rgb, d_fg, d_ctr, st);
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
  dfree(d_rgb);
  dfree(d_fg);
  dfree(d_ctr);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  if (st) (void)hipStreamDestroy(st);
  if (result) return result;
  if (ctr[rpk::CTR_STATUS] & rpk::STATUS_STACK_OVERFLOW) return fail(RP_EINTERNAL, "traversal stack overflow");
  if (t.n_slots) {
    std::vector<uint32_t> map;
    if (t.balanced) {
      map.resize(t.n_tiles);
      if ((result = rp_workspace_tile_map(s, &s->ws0, p, map.data(), t.n_tiles))) return result;
    }
    unpack_host(p, t, t.balanced ? map.data() : nullptr, shard.data(), sizeof(double), 3, out_rgb);
    if (out_fg) unpack_host(p, t, t.balanced ? map.data() : nullptr, shard_fg.data(), sizeof(float), 1, out_fg);
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
    if (!dalloc(&d_rays, 8 * n) || !dalloc(&d_hit, 9 * n) || !dalloc(&d_mat, n) || !dalloc(&d_ctr, rpk::CTR_N)) {
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
  for (void* p : {(void*)d_rays, (void*)d_hit, (void*)d_mat, (void*)d_ctr}) dfree(p);
  if (result) return result;
  if (ctr[rpk::CTR_STATUS] & rpk::STATUS_STACK_OVERFLOW) return fail(RP_EINTERNAL, "traversal stack overflow");
  return RP_OK;
}

// ---------------------------------------------------------------- multi-GPU ------------------------

int rp_gather_stride(const rp_render_params* p, uint64_t* stride) {
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (!stride) return fail(RP_EINVAL, "stride is NULL");
  *stride = stage_slots(t);
  return RP_OK;
}

int rp_frame_assemble(const rp_render_params* p, const void* d_gathered, uint32_t words, void* d_frame, void* stream) {
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (!d_gathered || !d_frame || words == 0) return fail(RP_EINVAL, "NULL buffer or zero words per slot");
  if (t.balanced) return fail(RP_EINVAL, "balanced frame: assemble with rp_frame_assemble_ws (the workspace holds the plan)");
  rpk::FrameGeom g{p->width, p->height, t.tw, t.th, t.tiles_x, t.shards, stage_slots(t), 0, nullptr};
  int e = rpk::launch_frame_assemble(g, static_cast<const uint32_t*>(d_gathered), words, static_cast<uint32_t*>(d_frame),
                                     stream);
  if (e != 0) return fail(RP_EHIP, std::string("frame assembly launch: ") + hipGetErrorString((hipError_t)e));
  return RP_OK;
}

int rp_workspace_tile_costs(rp_scene* s, rp_workspace* w, const rp_render_params* p, uint32_t* costs, uint32_t n) {
  if (!s || !costs) return fail(RP_EINVAL, "scene and costs must be non-NULL");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (n < 2 * t.n_shard_tiles) return fail(RP_EINVAL, "costs holds fewer than 2 x the shard's tiles");
  if (!w->meas_on) return fail(RP_EINVAL, "the workspace's last render did not measure tile costs");
  if (t.n_shard_tiles > (uint32_t)rpk::TILE_SORT_MAX) return fail(RP_EINVAL, "more than 16384 shard tiles");
  DeviceGuard g(s->device);
  RP_HIP(hipDeviceSynchronize());
  RP_HIP(hipMemcpy(costs, w->d_meas, sizeof(uint32_t) * t.n_shard_tiles, hipMemcpyDeviceToHost));
  RP_HIP(hipMemcpy(costs + t.n_shard_tiles, w->d_meas + rpk::TILE_SORT_MAX, sizeof(uint32_t) * t.n_shard_tiles,
                   hipMemcpyDeviceToHost));
  return RP_OK;
}

int rp_workspace_set_tile_costs(rp_scene* s, rp_workspace* w, const rp_render_params* p, const uint32_t* costs,
                                uint32_t ranks) {
  if (!s || !costs || ranks == 0) return fail(RP_EINVAL, "scene and costs must be non-NULL, ranks >= 1");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (t.n_tiles > (uint32_t)rpk::TILE_SORT_MAX) return fail(RP_EINVAL, "more than 16384 frame tiles");
  DeviceGuard g(s->device);
  RP_HIP(hipDeviceSynchronize());
  RP_HIP(hipMemcpy(w->d_fcost, costs, sizeof(uint32_t) * t.n_tiles, hipMemcpyHostToDevice));
  RP_HIP(hipMemcpy(w->d_fcost + rpk::TILE_SORT_MAX, costs + t.n_tiles, sizeof(uint32_t) * t.n_tiles,
                   hipMemcpyHostToDevice));
  set_fcost(w, p, t, ranks);
  return RP_OK;
}

int rp_frame_assemble_ws(rp_scene* s, rp_workspace* w, const rp_render_params* p, const void* d_gathered,
                         uint32_t words, void* d_frame, void* stream) {
  if (!s) return fail(RP_EINVAL, "scene is NULL");
  if (!w) w = &s->ws0;
  if (w->scene != s) return fail(RP_EINVAL, "workspace belongs to another scene");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if (!d_gathered || !d_frame || words == 0) return fail(RP_EINVAL, "NULL buffer or zero words per slot");
  rpk::FrameGeom g{p->width, p->height, t.tw, t.th, t.tiles_x, t.shards, stage_slots(t), 0, nullptr};
  if (t.balanced) {
    if (!plan_matches(w, p, t)) return fail(RP_EINVAL, "no balanced plan for this frame in the workspace: render it first");
    g.tile_pos = w->d_plan + t.n_tiles;
  }
  DeviceGuard dg(s->device);
  int e = rpk::launch_frame_assemble(g, static_cast<const uint32_t*>(d_gathered), words, static_cast<uint32_t*>(d_frame),
                                     stream);
  if (e != 0) return fail(RP_EHIP, std::string("frame assembly launch: ") + hipGetErrorString((hipError_t)e));
  return RP_OK;
}

int rp_comm_unique_id(uint8_t id[RP_COMM_ID_BYTES]) {
  if (!id) return fail(RP_EINVAL, "id is NULL");
  ncclUniqueId u;
  RP_NCCL(ncclGetUniqueId(&u));
  std::memcpy(id, &u, sizeof u);
  return RP_OK;
}

int rp_comm_create(const uint8_t id[RP_COMM_ID_BYTES], int nranks, int rank, int device, rp_comm** out) {
  if (!out) return fail(RP_EINVAL, "out is NULL");
  *out = nullptr;
  if (!id || nranks < 1 || rank < 0 || rank >= nranks) return fail(RP_EINVAL, "bad id / nranks / rank");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return fail(RP_EINVAL, "device index out of range");
  DeviceGuard g(device);
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  rp_comm* c = new rp_comm();
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(RP_ERCCL, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  }
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  *out = c;
  return RP_OK;
}

void rp_comm_destroy(rp_comm* c) {
  if (!c) return;
  DeviceGuard g(c->device);
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

int rp_comm_info(const rp_comm* c, int* nranks, int* rank, int* device) {
  if (!c) return fail(RP_EINVAL, "comm is NULL");
  if (nranks) *nranks = c->nranks;
  if (rank) *rank = c->rank;
  if (device) *device = c->device;
  return RP_OK;
}

int rp_frame_gather(rp_comm* c, rp_scene* s, rp_workspace* w, const rp_render_params* p, const double* d_shard_rgb,
                    uint8_t* d_frame_bgra, double* d_frame_rgb, uint64_t* d_counters, void* stream) {
  if (!c || !s || !d_shard_rgb) return fail(RP_EINVAL, "comm, scene and shard must be non-NULL");
  if (!w) w = &s->ws0;
  if (c->device != s->device) return fail(RP_EINVAL, "the communicator's device is not the scene's");
  if (reinterpret_cast<uintptr_t>(d_frame_bgra) % 4 != 0) return fail(RP_EINVAL, "d_frame_bgra must be 4-byte aligned");
  GatherPlan gp;
  int rc = gather_plan(s, w, c->nranks, c->rank, p, gp);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const bool bgra = d_frame_bgra != nullptr, rgb = d_frame_rgb != nullptr;
  DeviceGuard g(s->device);
  if ((rc = gather_stage(s, w, gp, d_shard_rgb, bgra, rgb, d_counters, st))) return rc;
  if ((rc = gather_collectives(c->comm, w, gp, bgra, rgb, st))) return rc;
  if ((rc = gather_learn(s, w, gp, p, bgra, st))) return rc;
  return gather_assemble(s, w, gp, d_frame_bgra, d_frame_rgb, d_counters, st);
}

int rp_frames_gather(rp_comm* c, rp_scene* s, rp_workspace* w, const rp_render_params* p, uint32_t n_frames,
                     const double* d_shard_rgb, uint8_t* d_frames_bgra, uint64_t* d_counters, void* stream) {
  if (!c || !s || !d_shard_rgb) return fail(RP_EINVAL, "comm, scene and shards must be non-NULL");
  if (n_frames == 0 || n_frames > RP_MAX_FRAMES) return fail(RP_EINVAL, "n_frames must be 1..RP_MAX_FRAMES");
  if (!w) w = &s->ws0;
  if (c->device != s->device) return fail(RP_EINVAL, "the communicator's device is not the scene's");
  if (reinterpret_cast<uintptr_t>(d_frames_bgra) % 4 != 0) return fail(RP_EINVAL, "d_frames_bgra must be 4-byte aligned");
  GatherPlan gp;
  int rc = gather_plan(s, w, c->nranks, c->rank, p, gp, n_frames);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const bool bgra = d_frames_bgra != nullptr;
  DeviceGuard g(s->device);
  if ((rc = gather_stage(s, w, gp, d_shard_rgb, bgra, false, d_counters, st))) return rc;
  if ((rc = gather_collectives(c->comm, w, gp, bgra, false, st))) return rc;
  if ((rc = gather_learn(s, w, gp, p, bgra, st))) return rc;
  return gather_assemble(s, w, gp, d_frames_bgra, nullptr, d_counters, st);
}

int rp_frames_block_words(const rp_render_params* p, uint32_t n_frames, uint64_t* words) {
  if (!words) return fail(RP_EINVAL, "words is NULL");
  if (n_frames == 0 || n_frames > RP_MAX_FRAMES) return fail(RP_EINVAL, "n_frames must be 1..RP_MAX_FRAMES");
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  *words = pack_words(t, true, n_frames);
  return RP_OK;
}

// rp_frames_gather's stage (1) and its stages (3a, 3) around the caller's collective: the workspace's own send / receive
// buffers are the ones rp_frames_gather uses, copied from / to the caller's.
int rp_frames_pack(rp_scene* s, rp_workspace* w, const rp_render_params* p, uint32_t n_frames, const double* d_shard_rgb,
                   const uint64_t* d_counters, uint32_t* d_send, void* stream) {
  if (!s || !d_shard_rgb || !d_send || !p) return fail(RP_EINVAL, "scene, params, shards and send buffer must be non-NULL");
  if (n_frames == 0 || n_frames > RP_MAX_FRAMES) return fail(RP_EINVAL, "n_frames must be 1..RP_MAX_FRAMES");
  if (!w) w = &s->ws0;
  GatherPlan gp;
  int rc = gather_plan(s, w, p->num_shards ? (int)p->num_shards : 1, (int)p->shard, p, gp, n_frames);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  DeviceGuard g(s->device);
  if ((rc = gather_stage(s, w, gp, d_shard_rgb, true, false, d_counters, st))) return rc;
  RP_HIP(hipMemcpyAsync(d_send, w->d_pack_send, sizeof(uint32_t) * pack_words(gp.t, true, n_frames),
                        hipMemcpyDeviceToDevice, st));
  return RP_OK;
}

int rp_frames_unpack(rp_scene* s, rp_workspace* w, const rp_render_params* p, uint32_t n_frames, const uint32_t* d_recv,
                     uint8_t* d_frames_bgra, uint64_t* d_counters, void* stream) {
  if (!s || !d_recv || !d_frames_bgra || !p) return fail(RP_EINVAL, "scene, params and buffers must be non-NULL");
  if (n_frames == 0 || n_frames > RP_MAX_FRAMES) return fail(RP_EINVAL, "n_frames must be 1..RP_MAX_FRAMES");
  if (reinterpret_cast<uintptr_t>(d_frames_bgra) % 4 != 0) return fail(RP_EINVAL, "d_frames_bgra must be 4-byte aligned");
  if (!w) w = &s->ws0;
  GatherPlan gp;
  int rc = gather_plan(s, w, p->num_shards ? (int)p->num_shards : 1, (int)p->shard, p, gp, n_frames);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  DeviceGuard g(s->device);
  RP_HIP(hipMemcpyAsync(w->d_pack_recv, d_recv, sizeof(uint32_t) * pack_words(gp.t, true, n_frames) * gp.geom.nranks,
                        hipMemcpyDeviceToDevice, st));
  if ((rc = gather_learn(s, w, gp, p, true, st))) return rc;
  return gather_assemble(s, w, gp, d_frames_bgra, nullptr, d_counters, st);
}

int rp_render_gather(rp_comm* c, rp_scene* s, rp_workspace* w, const rp_camera* cam, const rp_render_params* p,
                     uint8_t* d_frame_bgra, double* d_frame_rgb, uint64_t* d_counters, void* stream) {
  if (!c || !s) return fail(RP_EINVAL, "comm and scene must be non-NULL");
  if (!w) w = &s->ws0;
  Tiling t;
  int rc = make_tiling(p, t);
  if (rc) return rc;
  if ((int)t.shards != c->nranks || (int)t.shard != c->rank)
    return fail(RP_EINVAL, "params.shard / num_shards must be the communicator's rank / size");
  if (stage_slots(t) > w->gs_slots) return fail(RP_EINVAL, "workspace not reserved for this frame's gather: call rp_workspace_reserve");
  if ((rc = render_shard(s, w, cam, p, w->d_gs_rgb, nullptr, d_counters, stream))) return rc;
  return rp_frame_gather(c, s, w, p, w->d_gs_rgb, d_frame_bgra, d_frame_rgb, d_counters, stream);
}

void rp_multi_destroy(rp_multi* m) {
  if (!m) return;
  for (size_t k = 0; k < m->devices.size(); k++) {
    DeviceGuard g(m->devices[k]);
    if (k < m->comms.size() && m->comms[k]) (void)ncclCommDestroy(m->comms[k]);
    if (k < m->streams.size() && m->streams[k]) (void)hipStreamDestroy(m->streams[k]);
    if (k < m->d_ctr.size()) dfree(m->d_ctr[k]);
    if (k == 0) {
      dfree(m->d_frame_rgb);
      dfree(m->d_frame_bgra);
    }
  }
  for (rp_scene* s : m->scenes) rp_scene_destroy(s);
  delete m;
}

int rp_multi_create(const rp_scene_desc* desc, const int* devices, int n, const rp_scene_options* opt, rp_multi** out) {
  if (!out) return fail(RP_EINVAL, "out is NULL");
  *out = nullptr;
  if (!devices || n < 1) return fail(RP_EINVAL, "devices must list >= 1 device");
  for (int a = 0; a < n; a++)
    for (int b = a + 1; b < n; b++)
      if (devices[a] == devices[b]) return fail(RP_EINVAL, "devices must be distinct");
  rp_multi* m = new rp_multi();
  m->devices.assign(devices, devices + n);
  int rc = RP_OK;
  for (int k = 0; k < n && rc == RP_OK; k++) {
    rp_scene* s = nullptr;
    rc = scene_create(desc, devices[k], opt, &s);
    if (rc == RP_OK) m->scenes.push_back(s);
  }
  if (rc) {
    std::string e = g_err;
    rp_multi_destroy(m);
    return fail(rc, e);
  }
  m->comms.assign(n, nullptr);
  ncclResult_t r = ncclCommInitAll(m->comms.data(), n, devices);
  if (r != ncclSuccess) {
    m->comms.assign(n, nullptr);
    rp_multi_destroy(m);
    return fail(RP_ERCCL, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
  }
  m->streams.assign(n, nullptr);
  m->d_ctr.assign(n, nullptr);
  for (int k = 0; k < n; k++) {
    DeviceGuard g(devices[k]);
    if (hipStreamCreateWithFlags(&m->streams[k], hipStreamNonBlocking) != hipSuccess || !dalloc(&m->d_ctr[k], rpk::CTR_N)) {
      rp_multi_destroy(m);
      return fail(RP_EHIP, "stream / counter allocation");
    }
  }
  *out = m;
  return RP_OK;
}

int rp_render_multi(rp_multi* m, const rp_camera* cam, const rp_render_params* p_in, double* out_rgb, uint8_t* out_bgra,
                    rp_stats* stats) {
  if (!m || !cam || !p_in) return fail(RP_EINVAL, "multi, camera and params must be non-NULL");
  const int n = (int)m->devices.size();
  const bool bgra = out_bgra != nullptr, rgb = out_rgb != nullptr;
  std::vector<rp_render_params> ps(n, *p_in);
  std::vector<GatherPlan> plans(n);
  for (int k = 0; k < n; k++) {
    ps[k].shard = (uint32_t)k;
    ps[k].num_shards = (uint32_t)n;
    int rc = ws_reserve(m->scenes[k], &m->scenes[k]->ws0, &ps[k], true);
    if (rc) return rc;
  }
  const uint64_t frame_px = (uint64_t)p_in->width * p_in->height;
  if (frame_px > m->frame_px) {
    DeviceGuard g(m->devices[0]);
    dfree(m->d_frame_rgb);
    dfree(m->d_frame_bgra);
    m->d_frame_rgb = nullptr;
    m->d_frame_bgra = nullptr;
    m->frame_px = 0;
    if (!dalloc(&m->d_frame_rgb, 3 * frame_px) || !dalloc(&m->d_frame_bgra, frame_px))
      return fail(RP_ENOMEM, "hipMalloc frame");
    m->frame_px = frame_px;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < n; k++) {  // every device renders its shard into its staging buffer
    rp_scene* s = m->scenes[k];
    int rc = render_shard(s, &s->ws0, cam, &ps[k], s->ws0.d_gs_rgb, nullptr, m->d_ctr[k], m->streams[k]);
    if (rc) return rc;
    if ((rc = gather_plan(s, &s->ws0, n, k, &ps[k], plans[k]))) return rc;
    if ((rc = gather_stage(s, &s->ws0, plans[k], s->ws0.d_gs_rgb, bgra, rgb, m->d_ctr[k], m->streams[k]))) return rc;
  }
  // one thread drives every device: the collectives of all ranks form one group
  RP_NCCL(ncclGroupStart());
  for (int k = 0; k < n; k++) {
    DeviceGuard g(m->devices[k]);
    int rc = gather_collectives(m->comms[k], &m->scenes[k]->ws0, plans[k], bgra, rgb, m->streams[k]);
    if (rc) {
      (void)ncclGroupEnd();
      return rc;
    }
  }
  RP_NCCL(ncclGroupEnd());
  for (int k = 0; k < n; k++) {
    int rc = gather_learn(m->scenes[k], &m->scenes[k]->ws0, plans[k], &ps[k], bgra, m->streams[k]);
    if (rc) return rc;
  }
  rp_scene* s0 = m->scenes[0];
  int rc = gather_assemble(s0, &s0->ws0, plans[0], bgra ? reinterpret_cast<uint8_t*>(m->d_frame_bgra) : nullptr,
                           rgb ? m->d_frame_rgb : nullptr, m->d_ctr[0], m->streams[0]);
  if (rc) return rc;
  for (int k = 0; k < n; k++) {
    DeviceGuard g(m->devices[k]);
    hipError_t e = hipStreamSynchronize(m->streams[k]);
    if (e != hipSuccess) return fail(RP_EHIP, std::string("render: ") + hipGetErrorString(e));
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  DeviceGuard g(m->devices[0]);
  uint64_t ctr[rpk::CTR_N];
  RP_HIP(hipMemcpy(ctr, m->d_ctr[0], sizeof ctr, hipMemcpyDeviceToHost));
  // status bits OR-ed over the devices (gather_assemble)
  if (ctr[rpk::CTR_STATUS] & rpk::STATUS_STACK_OVERFLOW) return fail(RP_EINTERNAL, "traversal stack overflow");
  if (ctr[rpk::CTR_STATUS] & rpk::STATUS_PLAN_MISMATCH) return fail(RP_EINTERNAL, "devices made different tile plans");
  if (ctr[rpk::CTR_STATUS]) return fail(RP_EINTERNAL, "render kernel reported status " + std::to_string(ctr[rpk::CTR_STATUS]));
  if (rgb) RP_HIP(hipMemcpy(out_rgb, m->d_frame_rgb, sizeof(double) * 3 * frame_px, hipMemcpyDeviceToHost));
  if (bgra) RP_HIP(hipMemcpy(out_bgra, m->d_frame_bgra, 4 * frame_px, hipMemcpyDeviceToHost));
  if (stats) {
    stats->rays = ctr[rpk::CTR_RAYS];
    stats->samples = ctr[rpk::CTR_SAMPLES];
    stats->pixels = ctr[rpk::CTR_PIXELS];
    stats->seconds = secs;
  }
  return RP_OK;
}

}  // extern "C"
