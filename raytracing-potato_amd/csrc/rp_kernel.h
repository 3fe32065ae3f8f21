// rp_kernel.h -- host-visible interface of the HIP kernels (rp_kernel.hip).  No HIP types.
#pragma once
#include <stdint.h>

#include "rp_layout.h"

namespace rpk {

struct KScene {
  const void* nodes;     // rpl::Node4 or rpl::Node4Q records (node_format)
  const rpl::Prim* prims;
  const rpl::PrimRef* prim_refs;
  const double* vnrm;
  const double* vuv;
  const rpl::Material* mats;
  const rpl::Texture* texs;
  const uint32_t* texels;
  rpl::Emit background;
  uint32_t root;
  uint32_t always_first, n_always;  // prims tested before the tree for every ray (rp_bvh.h BuildOptions)
  double qbound;         // Node4Q: bound on every node frame's |o| and 255 s (rp_layout.h qbound): the slab slack
  uint32_t node_format;  // rpl::NODES_F32 / NODES_Q8: picks the kernel instantiation
  uint32_t leaf_break;   // trav_step leaves the inner-node loop once at most this many lanes still seek a leaf
  uint32_t stack_depth;  // traversal stack entries per lane (3 x max_depth + 7)
  uint32_t lds_depth;    // entries of it in LDS; entries [lds_depth, stack_depth) spill to `spill`
  uint64_t* diag;        // diagnostic counters (RPK_DIAG builds), DIAG_N x u64
  uint32_t* rng_slab;    // per-lane keystream cache, render_lanes x rng_slab_bytes_per_lane() bytes
  uint32_t* spill;       // per-lane stack overflow, render_lanes x (stack_depth - lds_depth) entries
  uint32_t* unit_t0;     // per-lane start time of the lane's measured unit (tile costs), render_lanes words
};

// Bytes of keystream cache (ChaCha key, ring of main-stream blocks, jitter blocks) per resident lane of
// the render kernel; the render grid never exceeds the lanes the slab was sized for.
uint64_t rng_slab_bytes_per_lane();
enum { RENDER_BLOCK = 64 };

// Diagnostic counters (RPK_DIAG builds): wave-cycles per phase {fetch, new sample, traverse, shade,
// tail}, wave loop iterations, active lanes at traverse, traversal wave-trips, lane node visits,
// lane primitive tests.
// [352 + b] units whose duration (100 MHz ticks) has floor(log2) = b + DIAG_DUR_LOG0 (clamped to 0..23), [376 + b]
// their rays summed.
enum { DIAG_N = 416, DIAG_DUR = 352, DIAG_DUR_N = 24, DIAG_DUR_LOG0 = 10 };
// Cycle regions (RPK_DIAG builds), from DIAG_N index DIAG_CYC: wave-cycles spent executing each code region
enum { DIAG_CYC = 320 };
enum {
  DCYC_SURF, DCYC_SPHUV, DCYC_TEXISSUE, DCYC_SCATTER, DCYC_TEXVAL, DCYC_EMIT, DCYC_START_SAMPLE, DCYC_END_SAMPLE,
  DCYC_NEWRAY, DCYC_REFILL, DCYC_NEXT_BOUNCE, DCYC_NODE_LOOP, DCYC_PRIM_LOOP, DCYC_N
};
// Timeline histograms (RPK_DIAG builds), 64 bins of DIAG_BIN_TICKS (100 MHz real-time clock) from the
// block's start: [64 + b] lanes retiring in bin b, [128 + b] rays of the pixels fetched in bin b,
// [192 + b] pixels fetched in bin b, [256 + b] the most rays of one unit fetched in bin b.
#ifndef RPK_DIAG_BIN_TICKS
#define RPK_DIAG_BIN_TICKS 1000000
#endif
enum { DIAG_HIST = 64, DIAG_BIN_TICKS = RPK_DIAG_BIN_TICKS };
// Region counters (RPK_DIAG builds), from DIAG_N index 16: per code region r, [16 + 2r] = wave
// executions and [17 + 2r] = active lanes summed over them (lane utilisation = lanes / (64 x execs)).
enum {
  DREG_NODE, DREG_PRIM, DREG_STEP, DREG_SHADE, DREG_SURF, DREG_SPHUV, DREG_TEX, DREG_LAMBERT, DREG_METAL,
  DREG_DIELEC, DREG_LOOP_LAMBERT, DREG_LOOP_METAL, DREG_END_SAMPLE, DREG_END_PIXEL, DREG_START_SAMPLE,
  DREG_REFILL, DREG_RNG_FALLBACK, DREG_JIT_FALLBACK, DREG_BEGIN_PIXEL, DREG_RING_LOAD, DREG_ROUND, DREG_MISS, DREG_N
};

// Division by a launch constant d >= 1 of numerators n < 2^31 (Granlund & Montgomery 1994, Thm 4.2 with N = 31):
// l = ceil(log2 d), s = 31 + l, m = ceil(2^s / d) < 2^32 (m d - 2^s < d <= 2^l), and floor(n / d) = (n m) >> s.
// The unit decode of every fetch (rp_device.h fetch_pixel) divides by five per-launch values; the compiler's
// division by a run-time divisor is ~25 VALU each.
struct Div32 {
  uint32_t m, s;
};
inline Div32 make_div32(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < (uint64_t)d) l++;
  const uint32_t s = 31 + l;
  return Div32{(uint32_t)(((1ull << s) + d - 1) / d), s};
}

struct KParams {
  double orient[9];
  double pos[3];
  double aspect, tan_fov, focal, lens;
  uint64_t seed;
  uint32_t W, H, spp, max_bounce;
  uint32_t tw, th, shard, nshards;
  uint32_t tiles_x, n_shard_tiles;
  uint64_t n_slots;  // n_shard_tiles * tw * th
  uint32_t trav_threshold;  // resume shading once fewer than this many lanes of a wave still traverse
  uint32_t probe;           // 1 = cost probe: sample 0 of probe_px pixels per tile
  uint32_t probe_px;        // probe: pixels probed per tile: every pixel (tw * th) or an n x n lattice (n^2)
  uint32_t probe_n;         // probe: lattice side n, 0 = every pixel
  uint32_t nbatch;          // sample batches (RNG streams) per pixel: ceil(spp / spp_batch); 1 in a probe
  uint32_t spp_batch;       // samples per batch: SPP_BATCH (the contract); other values for timing studies only
  uint64_t n_queue;         // queue entries: n_slots * nbatch units (render), probed pixels (probe)
  uint32_t queue_groups;    // render: unit queues (1, or QUEUE_GROUPS: one per group blockIdx mod 8 = one XCD)
  uint32_t queue_chunk;     // render: queue g serves the chunks g, g + G, ... of queue_chunk consecutive tiles (>= 1)
  // render: make_div32 of tw * th * nbatch (a tile's units), nbatch, tiles_x, tw, queue_chunk (n_queue < 2^31)
  Div32 dv_units, dv_nbatch, dv_tiles_x, dv_tw, dv_chunk;
  double* partial;          // nbatch > 1: per unit (slot * nbatch + batch) the batch's sample sum, 3 f64
  uint32_t* partial_hits;   // nbatch > 1: per unit, samples whose first ray hit (foreground)
  const uint32_t* tile_order;  // render: queue position k -> shard tile index (NULL = identity)
  const uint32_t* tile_map;    // the frame's tile deal order (RP_SHARD_BALANCED plan): shard tile k is frame tile
                               // tile_map[shard + k * nshards] (NULL = interleave: tile shard + k * nshards)
  uint32_t* tile_meas;         // render (NULL = off): measured cost of shard tile k -- [k] its units' summed durations,
                               // [TILE_SORT_MAX + k] the longest, in MEAS_SHIFT-scaled 100 MHz ticks (zeroed by the caller)
  uint32_t* tile_cost;         // probe: [k] cost (rp_device.h WORK_*: node visits, primitive tests, rays)
                               // summed over the tile's probed samples, [TILE_SORT_MAX + k] the costliest
                               // probed sample (zeroed by the caller)
  // Learned per-unit order (launch_unit_order): render -- every unit's duration (100 MHz ticks) is stored at
  // unit_cost[slot * nbatch + batch] (NULL = off); and when unit_order is set the queues hand out units in its order
  // (position p -> unit unit_order[p]; queue g serves the chunks g, g + G, ... of order_chunk positions) instead of
  // tile by tile.
  uint32_t* unit_cost;
  const uint32_t* unit_order;
  uint32_t order_chunk;
  Div32 dv_ochunk, dv_tile_px;  // make_div32(order_chunk), make_div32(tw * th)
  // Several frames in one launch (rp.h rp_render_frames_device_ws): frame f is the frame of these params whose sample
  // batches are f * nbatch .. f * nbatch + nbatch - 1 of the RNG contract (seed + (f nbatch + b) W H + j W + i); the
  // queues hand out n_frames x n_shard_tiles virtual tiles -- frame by frame (virtual tile f * n_shard_tiles + k is frame
  // f's k-th tile) or, frames_inter, rank by rank (virtual tile k * n_frames + f: the frames' k-th tiles of the cost order
  // together) -- a unit carries its global batch f * nbatch + b, and frame f writes out + f * out_stride (out_fg + f *
  // n_slots) or its batch sums at partial + 3 (f * n_slots + slot) * nbatch.
  uint32_t n_frames;            // >= 1
  uint32_t frames_inter;        // 1: rank by rank; 2: rank by rank, a unit's frames consecutive (RP_FRAME_ORDER_PIXEL)
  Div32 dv_tiles, dv_frames;    // make_div32(n_shard_tiles), make_div32(n_frames)
  uint64_t out_stride;          // doubles between frames' shard buffers (3 * n_slots)
};

// Cost-ordered tile scheduling.  A frame's tail (waves holding a few lanes that still finish the last
// pixels after the queue drained) was ~23% of the C3 frame; handing out the expensive tiles first
// (longest-processing-time-first) leaves cheap, uniform tiles for the end.  The order comes from a probe
// launch of the same kernel (sample 0 of a 16 x 16 lattice of pixels per tile: the exact
// paths of the frame) and a one-block sort.  Tiles holding the costliest samples go first (cost = traversal
// work + shaded rays: on C5 the rays differ far more in node visits than in path length): a unit's samples
// run sequentially on one lane, so one expensive unit fetched late becomes a latency-bound tail by itself.
// Results do not depend on the order (per-pixel seeding).
enum { PROBE_LATTICE_N = 16, TILE_SORT_MAX = 16384 };
// Measured tile costs: unit durations in 100 MHz ticks >> MEAS_SHIFT (0.64 us): a C4 tile's 32768 units of ~100 us
// sum to ~5e6, far from 2^32; the sort's log2 buckets of the longest unit stay below their cap up to ~40 ms.
enum { MEAS_SHIFT = 6 };
// Learned cost table: frame tile t's measured cost ([t] sum, [TILE_SORT_MAX + t] longest unit) from the measured
// shard-tile costs of nranks ranks (rank r's [k] at sum[r * rank_stride + k], max[r * rank_stride + k]; shard tile k
// of rank r is frame tile plan[r + k * nranks], or r + k * nranks without a plan).  One thread per tile.
int launch_learn_costs(const uint32_t* sum, const uint32_t* max, uint32_t rank_stride, uint32_t nranks, uint32_t n_tiles,
                       const uint32_t* plan, uint32_t* fcost, void* stream);

// RNG streams per (pixel, batch of SPP_BATCH samples) -- include/rp.h RP_SAMPLES_PER_STREAM.  The queue
// hands out units (pixel, batch), so one pixel's samples run on several lanes at once; a unit of a
// multi-batch frame leaves its sample sum in `partial` and reduce_batches adds them in batch order.
// 32 samples: a C3 pixel's 256 samples become 8 units (an 8-GPU shard: ~2 M units for 262 k lanes); 64 ran
// 0.8% faster on one GPU but left an 8-GPU shard with a 30% latency-bound tail (projection, 70% vs 84%
// efficiency).
enum { SPP_BATCH = 32 };

// Unit-queue words of a workspace: group g's counter at g * QUEUE_STRIDE (own 128 B line), the probe's at
// QUEUE_PROBE.
enum { QUEUE_GROUPS = 8, QUEUE_STRIDE = 32, QUEUE_PROBE = QUEUE_GROUPS * QUEUE_STRIDE, QUEUE_WORDS = QUEUE_PROBE + QUEUE_STRIDE };

// Counter block layout (RP_COUNTERS_LEN x uint64 in device memory), see rp.h rp_render_device.
enum { CTR_RAYS = 0, CTR_SAMPLES = 1, CTR_PIXELS = 2, CTR_STATUS = 3, CTR_N = 4 };
enum : uint64_t { STATUS_STACK_OVERFLOW = 1, STATUS_PLAN_MISMATCH = 2 };
// Counter block one rank contributes to a frame gather: its CTR_N counters, then its tile plan's hash (0 for the
// interleave), padded to GATHER_CTR words.
enum { GATHER_CTR = 8, GATHER_CTR_HASH = 4 };

// Launch the persistent render kernel on `stream` (hipStream_t).  `counters` and the unit-queue word
// `queue` (workspace-owned) must have been zeroed on the same stream.  Returns a hipError_t as int.
int launch_render(const KScene& s, const KParams& p, double* out_rgb, float* out_fg, uint64_t* counters,
                  uint32_t* queue, int grid, void* stream);

// Learned per-unit order (rp_sched.hip): the n units sorted by the previous frame's durations `cost`, longest first, in
// log-spaced buckets (UNIT_ORDER_Q per octave, unit_bucket) that keep shard order inside -> order[0, n).  keys, keys2: n
// u64 each; scratch: unit_order_scratch_bytes(n) bytes (hipCUB radix sort of UNIT_KEY_BITS bits).  n < 2^31.
enum { UNIT_ORDER_Q = 4, UNIT_ORDER_CHUNK = 256, UNIT_KEY_BITS = 40 };
size_t unit_order_scratch_bytes(uint64_t n);
int launch_unit_order(const uint32_t* cost, uint64_t n, uint64_t* keys, uint64_t* keys2, void* scratch,
                      size_t scratch_bytes, uint32_t* order, void* stream);

// Sort the n (<= TILE_SORT_MAX) probed shard tiles by descending (costliest sample, mean cost per probed
// pixel), log-quantized, ties by tile index, into order[] (shard tile indices).  One block.
// With cost == NULL: the shard's tiles in Z-order of their frame-grid coordinates (tiles_x, tiles_y <= 256),
// so tiles processed at the same time are neighbours (the scene's cache working set stays small).
struct TileGeom {
  uint32_t tiles_x, shard, nshards;
  const uint32_t* map;    // a launch_tile_plan plan (order, then its inverse) of map_tiles frame tiles, NULL = interleave
  uint32_t map_tiles;
  uint32_t cost_by_tile;  // 1: cost[] is indexed by frame tile (a whole-frame probe), 0: by shard tile
};
// scratch: SORT_SCRATCH words of device memory (the sort's keys, the plan's hash word and its per-block costs; not
// LDS, see rp_kernel.hip SORT_BLOCK).
enum { SORT_SCRATCH = 2 * TILE_SORT_MAX + 1 };
int launch_tile_sort(const uint32_t* cost, uint32_t n, uint32_t probe_px, const TileGeom& g, uint32_t* order,
                     uint64_t* scratch, void* stream);

// Final pass of a multi-batch frame: per shard slot, the batch sums added in batch order, / spp.
int launch_reduce_batches(const KParams& p, double* out_rgb, float* out_fg, void* stream);

// Output stage: thresholds of to_srgb_u8 (thr[k] = smallest x whose byte is >= k, k = 1..255; thr[0] unused)
// and the launch converting n slots of linear f64 RGB into B, G, R, 255 bytes (4-byte aligned output).
struct SrgbTable {
  double thr[256];
};
int launch_srgb_bgra(const SrgbTable& tab, const double* rgb, uint64_t n, uint8_t* bgra, void* stream);

// Frame assembly of a multi-GPU frame: `gathered` holds nranks shard buffers of `stride` slots each (rank r
// at r * stride, `words` 32-bit words per slot: 1 for BGRA8, 6 for f64 RGB); every frame pixel (i, j)
// takes its slot from the rank that owns its tile (tile t -> rank t % nranks, shard slot k * tw * th +
// row-major offset inside the tile, k = t / nranks: rp_shard_unpack's order).  One thread per pixel.
struct FrameGeom {
  uint32_t W, H, tw, th, tiles_x, nranks;
  uint64_t stride;           // slots per rank buffer
  uint64_t rank_words;       // 32-bit words from one rank's buffer to the next (0 = stride * words: packed shards)
  const uint32_t* tile_pos;  // frame tile -> its position in the deal order (rank = pos % nranks, shard tile k =
                             // pos / nranks); NULL = interleave (pos = the tile index)
};

// Balanced tile plan (rp.h RP_SHARD_BALANCED): from per-frame-tile costs (cost[t]: a learned table, or a whole-frame
// probe, deterministic: the probe traverses without the speculative and early-exit steps), the n frame tiles are
// grouped into blocks of block x block tiles (block = 1: single tiles), the blocks sorted by summed cost (descending,
// ties by block index) and dealt in rounds of nranks blocks alternating direction ("snake"), the tiles past the last
// whole round one at a time -- every rank receiving exactly the interleave's tile count.  Blocks keep a rank's tiles
// in compact squares of the frame, so a scene past the Infinity Cache keeps its working set small on every rank.
// Writes plan[0, n) = the deal order (tile of shard s, shard tile k at plan[s + k * nranks]), plan[n, 2n) = its
// inverse and plan[2n, 2n+2) = a 64-bit hash of the order (compared across ranks in the frame gather).  One block.
int launch_tile_plan(const uint32_t* cost, uint32_t n, uint32_t nranks, uint32_t tiles_x, uint32_t block, uint32_t* plan,
                     uint64_t* scratch, void* stream);
// Counters of a frame gather: stage this rank's block (ctr may be NULL = zeros; hash may be NULL = 0) for the
// all-gather, and reduce the gathered blocks of nranks ranks into out (sums; status bits OR-ed, plus
// STATUS_PLAN_MISMATCH when two ranks' plan hashes differ).
// A frame gather's one collective carries, per rank, a packed block of 32-bit words (GATHER_HEAD + 2 x stride_tiles,
// rounded up to even, then the BGRA8 shard): [0, 2 GATHER_CTR) the counter block (GATHER_CTR u64), then the measured
// tile costs -- stride_tiles sums, stride_tiles maxima (zeros past the table) -- then the to_srgb_u8 bytes.
// launch_gather_pack writes the first two parts (ctr / hash NULL = zeros, meas = the workspace's 2 x TILE_SORT_MAX
// measured costs, NULL = zeros); launch_counters_reduce reads nranks blocks `rank_words` apart.
int launch_gather_pack(const uint64_t* ctr, const uint32_t* hash, const uint32_t* meas, uint32_t stride_tiles,
                       uint32_t* send, void* stream);
int launch_counters_reduce(const uint64_t* gathered, uint32_t nranks, uint64_t rank_words, uint64_t* out, void* stream);
int launch_frame_assemble(const FrameGeom& g, const uint32_t* gathered, uint32_t words, uint32_t* frame,
                          void* stream);

// Blocks of 256 threads resident per CU for the render kernel with this stack depth (occupancy query).
int render_blocks_per_cu(uint32_t lds_depth, bool spill, uint32_t node_format, int* blocks);

// Closest-hit query kernel (one ray per thread).
int launch_intersect(const KScene& s, const double* rays, uint64_t n, double* out_hit, uint32_t* out_mat,
                     uint64_t* counters, void* stream);

}  // namespace rpk
