/*
 * rp.h -- C-ABI of the MI355X path-tracing hot path (librp.so).
 *
 * Drop-in boundary for alucas2/raytracing-potato ("scaling-potato", crate raytracing2).
 * The reference has no FFI; its seam is the per-pixel worker loop
 *   main.rs:61-92  (make_uv_jitter -> Camera::shoot -> trace_path -> accumulate -> average)
 * calling
 *   render.rs:94-146 trace_path / trace_path_first / trace_path_continue
 * over the scene types
 *   hittable.rs:10-15 (Hittable), mesh.rs:18-22 (Mesh), material.rs:19-91 (Scatter/Emit/Absorb/Material),
 *   texture.rs:10-18 (Texture), render.rs:10-25 (SceneData, Camera).
 * rp_render() replaces that whole per-pixel loop for one frame (or one shard of it); the host keeps
 * scene construction, OBJ/TGA loading and image output (example_scenes.rs, mesh.rs:145, image.rs:73,116).
 *
 * Conventions
 *   - Plain C types only; no HIP/C++ types or exceptions cross this boundary.
 *   - Every function returning int returns RP_OK (0) or a negative rp_status; rp_last_error() gives a
 *     thread-local message for the last failure on the calling thread.  Nothing aborts or panics.
 *   - Ownership: the caller owns every buffer it passes.  rp_scene_create deep-copies the scene into
 *     device memory (HBM); the scene is immutable afterwards.
 *   - Determinism (the RNG contract): the samples of pixel (i, j) are drawn in batches of
 *     N = params.samples_per_stream (0 -> RP_SAMPLES_PER_STREAM = 32); batch b (samples N*b .. N*b+N-1)
 *     is rendered with its own StdRng::seed_from_u64(params.seed + b*width*height + j*width + i)
 *     (rand 0.8 StdRng = ChaCha12) and the unchanged per-pixel body of main.rs:70-85 over its samples
 *     (make_uv_jitter from a clone of the batch stream's start).  The pixel value is (S_0 + S_1 + ...) /
 *     spp, batch sums added in batch order (main.rs:80,86).  With N >= spp (e.g. samples_per_stream =
 *     spp) this is SURVEY.md 8c's one stream per pixel, seed + j*width + i, for any spp.  Output depends
 *     only on (scene, camera, seed, width, height, spp, max_bounce, samples_per_stream) -- never on
 *     tiling, sharding, device count, scheduling or the environment.  (The reference draws every pixel of
 *     a worker's tiles from one from_entropy() stream, main.rs:52, so its output is not reproducible; a
 *     pixel's samples are sequential in a stream, so batching them is what lets one pixel's work spread
 *     over lanes/GPUs: the default 32 keeps an 8-GPU shard's longest unit short.)
 *   - No allocation happens inside the asynchronous calls (rp_render_device*, rp_frame_gather,
 *     rp_render_gather): device memory they need is reserved up front (rp_workspace_reserve), so they
 *     can be captured into a hipGraph and never synchronise the device.
 *   - Arithmetic is IEEE binary64 throughout, as the reference (utility.rs:14 `type Real = f64`).
 *   - Image layout: row-major, pixel (i, j) at index j*width + i, row j = 0 is the BOTTOM row
 *     (image.rs:31-33, main.rs:119, tga::save writes bottom-left origin).  RGB are linear f64 averages
 *     (main.rs:86), i.e. before to_srgb_u8 (utility.rs:212).
 */
#ifndef RP_H
#define RP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RP_ABI_VERSION 9

/* Default samples per RNG stream (see "Determinism" above; rp_render_params.samples_per_stream = 0). */
#define RP_SAMPLES_PER_STREAM 32

/* Device counter block of the asynchronous renders: RP_COUNTERS_LEN uint64 {rays, samples, pixels,
 * status}.  Nothing else is written through the pointer (the unit queue lives in the workspace). */
#define RP_COUNTERS_LEN 4
enum { RP_CTR_RAYS = 0, RP_CTR_SAMPLES = 1, RP_CTR_PIXELS = 2, RP_CTR_STATUS = 3 };
/* status bits (OR-ed over the ranks of a frame gather, never summed) */
#define RP_STATUS_STACK_OVERFLOW 1u  /* a lane's traversal stack overflowed (entries dropped: the frame is wrong) */
#define RP_STATUS_PLAN_MISMATCH 2u   /* ranks of a balanced frame made different tile plans (frame invalid) */

/* Bytes of an RCCL unique id (rp_comm_unique_id). */
#define RP_COMM_ID_BYTES 128

typedef enum rp_status {
  RP_OK = 0,
  RP_EINVAL = -1,    /* bad argument / malformed scene (the reference would panic: index out of range, etc.) */
  RP_EHIP = -2,      /* HIP runtime error */
  RP_ENOMEM = -3,    /* host or device allocation failed */
  RP_ENODEV = -4,    /* no usable gfx950 device */
  RP_EINTERNAL = -5, /* kernel reported an internal error (e.g. traversal stack overflow) */
  RP_ERCCL = -6      /* RCCL (collective communication) error */
} rp_status;

/* ---------------------------------------------------------------- scene description ----------- */

/* hittable.rs:10-15.  List/Bvh aggregates are expressed by rp_scene_desc.root_kind. */
enum { RP_HITTABLE_SPHERE = 0, RP_HITTABLE_TRIANGLE = 1 };

typedef struct rp_hittable {
  uint32_t kind;       /* RP_HITTABLE_* */
  uint32_t material;   /* Sphere {material: MaterialId} */
  uint32_t mesh;       /* Triangle {mesh: MeshId} */
  uint32_t triangle;   /* Triangle {triangle: TriangleId} = offset of the first of 3 indices (mesh.rs:33) */
  double center[3];    /* Sphere {center} */
  double radius;       /* Sphere {radius} */
} rp_hittable;

/* mesh.rs:7-22: Vertex {position, normal, uv} stored as three interleaved arrays. */
typedef struct rp_mesh {
  uint32_t n_vertices;
  uint32_t n_indices;      /* multiple of 3 */
  const double* positions; /* 3 * n_vertices (x, y, z per vertex) */
  const double* normals;   /* 3 * n_vertices */
  const double* uvs;       /* 2 * n_vertices */
  const uint32_t* indices; /* n_indices */
  uint32_t material;       /* Mesh.material (MaterialId) */
  uint32_t reserved;
} rp_mesh;

/* material.rs:19-24 */
enum { RP_SCATTER_NONE = 0, RP_SCATTER_LAMBERT = 1, RP_SCATTER_METAL = 2, RP_SCATTER_DIELECTRIC = 3 };
/* material.rs:66-71 */
enum { RP_ABSORB_BLACK_BODY = 0, RP_ABSORB_WHITE_BODY = 1, RP_ABSORB_ALBEDO = 2, RP_ABSORB_ALBEDO_MAP = 3 };
/* material.rs:40-46 */
enum { RP_EMIT_NONE = 0, RP_EMIT_DEBUG_NORMALS = 1, RP_EMIT_COLOR = 2, RP_EMIT_SKY_GRADIENT = 3,
       RP_EMIT_SKY_SPHERE = 4 };
/* texture.rs:10-18 */
enum { RP_TEXTURE_MISSING = 0, RP_TEXTURE_DEBUG_UVS = 1, RP_TEXTURE_SOLID = 2, RP_TEXTURE_IMAGE = 3,
       RP_TEXTURE_CHECKER = 4, RP_TEXTURE_NOISE = 5, RP_TEXTURE_PERLIN = 6 };

typedef struct rp_scatter {
  uint32_t kind;       /* RP_SCATTER_* */
  uint32_t reserved;
  double param;        /* Metal {fuzziness} | Dielectric {refraction_index} */
} rp_scatter;

typedef struct rp_absorb {
  uint32_t kind;       /* RP_ABSORB_* */
  uint32_t texture;    /* AlbedoMap(TextureId) */
  double color[3];     /* Albedo(Color) */
} rp_absorb;

typedef struct rp_emit {
  uint32_t kind;       /* RP_EMIT_* */
  uint32_t texture;    /* SkySphere(TextureId) */
  double color[3];     /* Color(Color) */
} rp_emit;

/* material.rs:87-91; evaluation order scatter -> absorb -> emit (material.rs:104-110) */
typedef struct rp_material {
  rp_scatter scatter;
  rp_absorb absorb;
  rp_emit emit;
} rp_material;

typedef struct rp_texture {
  uint32_t kind;         /* RP_TEXTURE_* */
  uint32_t odd, even;    /* Checker {odd, even} (TextureId) */
  uint32_t width, height;/* Image: Array2d<[u8;4]> dimensions */
  uint32_t reserved;
  int64_t seed;          /* Noise {seed} | Perlin {seed} (isize) */
  double color[3];       /* Solid(Color) */
  const uint8_t* rgba;   /* Image: width*height*4 bytes, texel (i, j) at 4*(i + j*width), j = 0 bottom row */
} rp_texture;

enum { RP_ROOT_BVH = 0, RP_ROOT_LIST = 1 };

/* render.rs:10-14 SceneData + example_scenes.rs:14-19 root/background. */
typedef struct rp_scene_desc {
  uint32_t root_kind;                  /* Hittable::Bvh (any tree shape) or Hittable::List */
  uint32_t n_hittables;
  const rp_hittable* hittables;
  uint32_t n_meshes;
  const rp_mesh* meshes;
  uint32_t n_materials;
  const rp_material* materials;
  uint32_t n_textures;
  const rp_texture* textures;
  rp_emit background;
} rp_scene_desc;

/* render.rs:19-25 + utility.rs:160-163.  orientation is column-major as nalgebra's Matrix3
 * (columns x, y, z of Transformation::lookat, utility.rs:172-177). */
typedef struct rp_camera {
  double aspect_ratio, fov, focal_dist, lens_radius;
  double orientation[9];
  double position[3];
} rp_camera;

/* One frame (or one shard of it).  The frame is cut into tile_w x tile_h tiles in row-major tile
 * order (image.rs:151-167), and the tiles are dealt to the S shards (GPUs) by shard_map:
 *   RP_SHARD_INTERLEAVE: shard s renders tiles t with t % S == s, its k-th tile is t = s + k*S.
 *   RP_SHARD_BALANCED: a tile plan deals them by cost.  The render of a shard first traces a cost probe of the
 *     WHOLE frame (sample 0 of a lattice of pixels per tile, traversal work counted without any dependence on
 *     the scheduling, so every rank measures the same costs) and deals the tiles, costliest first, in rounds of
 *     S alternating direction; shard s's k-th tile is the deal order's entry s + k*S.  Every shard holds exactly
 *     the interleave's number of tiles (same buffer sizes and gather strides), and every rank computes the same
 *     plan (the frame gather compares their hashes: RP_STATUS_PLAN_MISMATCH).  The plan lives in the workspace of
 *     the render; rp_workspace_tile_map returns it.  Frames of more than 16384 tiles are dealt as the interleave.
 * Neither choice changes a pixel (per-pixel seeding): only which GPU renders it. */
enum { RP_SHARD_INTERLEAVE = 0, RP_SHARD_BALANCED = 1 };
typedef struct rp_render_params {
  uint32_t width, height;   /* Multisampler {width, height} */
  uint32_t spp;             /* Multisampler {num_samples} */
  uint32_t max_bounce;      /* trace_path depth (main.rs:25); >= 1 (render.rs:97) */
  uint64_t seed;            /* base seed of the RNG contract */
  uint32_t tile_w, tile_h;  /* 0 -> 32 (main.rs:26) */
  uint32_t shard, num_shards;/* num_shards 0 -> 1 */
  uint32_t samples_per_stream; /* RNG contract batch size N, 0 -> RP_SAMPLES_PER_STREAM; N >= spp: one
                                  stream per pixel */
  uint32_t shard_map;       /* RP_SHARD_INTERLEAVE (0) or RP_SHARD_BALANCED */
} rp_render_params;
/* A shard holds at most 2^31 - 1 (pixel, sample stream) units -- its pixels x ceil(spp / samples_per_stream) -- and
 * with the default per-XCD unit queues half the 32-bit queue word less the resident lanes; larger shards are refused
 * with RP_EINVAL (e.g. 8192 x 8192 pixels at 1024 spp: split the frame into shards). */

/* Scene build and kernel tuning options (rp_scene_create_ex).  None of them changes an image beyond
 * exact-t ties between primitives (the closest hit does not depend on the tree).
 * Zero-initialised fields take the defaults; rp_scene_options_init fills them in explicitly. */
/* Builders: HOST = multi-threaded binned SAH on the CPU; DEVICE = LBVH on the GPU (Karras 2012: fastest build,
 * Morton-split tree); PLOC = agglomerative clustering on the GPU (Meister & Bittner 2018: SAH-quality tree). */
enum { RP_BUILDER_AUTO = 0, RP_BUILDER_HOST = 1, RP_BUILDER_DEVICE = 2, RP_BUILDER_PLOC = 3 };
/* Wide-node formats: 128 B f32 child boxes, or 64 B child boxes quantized to 8 bits per plane in a per-node
 * f32 frame (half the node bytes, more ALU per visit).  AUTO = Q8 for host-built trees of >= 2^21 hittables,
 * F32 otherwise. */
enum { RP_NODES_AUTO = 0, RP_NODES_F32 = 1, RP_NODES_Q8 = 2, RP_NODES_W8 = 3 };
/* Tile orders: PLAIN = shard order (row-major); COST = the costliest tiles go first (short frame tail), by the
 * workspace's learned costs of the previous frame (see rp_workspace_tile_costs) or, without them, by a probe
 * launch that traces sample 0 of a lattice of pixels per tile; PROBE = COST always from the probe; MORTON = Z-order
 * of the tiles (neighbouring tiles run together: a small cache working set; a balanced multi-GPU plan then deals
 * square blocks of tiles).  AUTO = COST (round 4; rounds 2-3: MORTON for scenes past the 256 MB Infinity Cache). */
enum { RP_TILES_AUTO = 0, RP_TILES_PLAIN = 1, RP_TILES_COST = 2, RP_TILES_MORTON = 3, RP_TILES_PROBE = 4 };
/* Unit queues: SINGLE = one device-wide queue over the tile order; XCD_TILES = eight queues, one per group of
 * render blocks sharing an XCD (and its L2), tile k of the order served by queue k mod 8 (a tile's pixels
 * run on one XCD); XCD_REGIONS = queue g serves the g-th eighth of the tile order (a compact region per XCD
 * under Z-order).  A drained queue's blocks take units from the others.  AUTO = XCD_TILES. */
enum { RP_QUEUES_AUTO = 0, RP_QUEUES_SINGLE = 1, RP_QUEUES_XCD_TILES = 2, RP_QUEUES_XCD_REGIONS = 3 };
/* How the binary SAH tree is collapsed into 4-wide nodes (host builder; ABI v6): AUTO = SAH; GREEDY opens the child
 * of largest surface area until a node has 4 children; SAH takes the cut through the binary subtree that minimises
 * the 4-wide tree's SAH cost (dynamic program).  Never changes an image beyond exact-t ties. */
enum { RP_COLLAPSE_AUTO = 0, RP_COLLAPSE_GREEDY = 1, RP_COLLAPSE_SAH = 2 };
/* rp_scene_options.node_layout (ABI v7): the memory order of a device-built (PLOC) tree's wide nodes.  DFS: depth-first,
 * a node's inner children as one consecutive family; DFS_LINE: the same with every family starting on a 128-B cache
 * line (64-B quantized nodes: a pad slot after odd families; f32 nodes are one line each, so the same as DFS).  Speed
 * only: the image never depends on it. */
enum { RP_LAYOUT_AUTO = 0, RP_LAYOUT_DFS = 1, RP_LAYOUT_DFS_LINE = 2 };
/* rp_scene_options.unit_order (ABI v8): the order the unit queues hand out a shard's (pixel, sample stream) units.
 * TILES: tile by tile (tile_order), a tile's pixels row-major.  LEARNED: every render of one frame per launch stores each
 * unit's duration, and the next such frame of the same shape on the same workspace hands out its units longest first
 * (log-spaced buckets, shard order inside; a frame ends with its longest unit), on one device or interleaved shards (a
 * balanced plan's tiles may move between frames: those frames keep TILES).  AUTO (ABI v9) = LEARNED for one stream per
 * pixel (samples_per_stream >= spp: lone C3 frames 220 vs 261 ms), TILES for several streams per pixel (32-sample streams:
 * +4.4 %) and for launches of several frames (their interleaved tile order, rp_render_frames_device_ws);
 * LEARNED also orders such launches, a unit's frames handed out together.  Results never depend on it. */
enum { RP_UNITS_AUTO = 0, RP_UNITS_TILES = 1, RP_UNITS_LEARNED = 2 };
typedef struct rp_scene_options {
  uint32_t builder;         /* RP_BUILDER_*: AUTO = HOST (multi-threaded binned SAH); DEVICE = LBVH (faster
                               build, ~24 % slower traversal on 10 M triangles); PLOC */
  uint32_t max_leaf;        /* primitives per leaf, 1..8 (0 -> 4) */
  double cost_traverse;     /* SAH node cost relative to a primitive test (0 -> 0.7) */
  int32_t always_max;       /* primitives tested before the tree for every ray (-1 -> 4; 0 = none) */
  uint32_t lds_depth;       /* traversal-stack entries kept in LDS (0 -> automatic; >= 8 forces a split) */
  uint32_t self_check;      /* 1: structural self-check of a device-built tree (slow; tests) */
  uint32_t trav_threshold;  /* lanes of a wave still traversing before the finished ones shade (0 -> 24 for
                               scenes within the 256 MB Infinity Cache, 32 above; 1..64) */
  uint32_t tile_order;      /* RP_TILES_*: the order the unit queue hands out a shard's tiles */
  uint32_t probe_n;         /* cost probe lattice n x n per tile (0 -> 16) */
  uint32_t node_format;     /* RP_NODES_* */
  uint32_t leaf_break;      /* speculative traversal: a wave moves to the leaf tests once at most this many of its
                               lanes still look for a leaf (0 -> 8 for scenes within the 256 MB Infinity Cache,
                               16 above; 1..64) */
  uint32_t unit_queues;     /* RP_QUEUES_*: how the render blocks share out the units */
  uint32_t queue_chunk;     /* XCD_TILES: consecutive tiles of the order dealt to one queue at a time (0: up to 8 while
                               every queue gets >= 16 chunks; a launch of n interleaved frames: rounded up to a multiple
                               of n, whole tiles of every frame) */
  uint32_t debug_stack_depth; /* TESTS ONLY (0 = off): traversal-stack entries per lane, 8..4096, instead of the
                               depth the tree needs.  Too small a stack drops entries -- wrong frames -- and the
                               render reports RP_STATUS_STACK_OVERFLOW / RP_EINTERNAL: the error path made reachable. */
  uint32_t collapse;        /* RP_COLLAPSE_*: the 4-wide collapse of the host-built tree (ABI v6) */
  uint32_t node_layout;     /* RP_LAYOUT_*: node order of a device-built (PLOC) tree (ABI v7) */
  uint32_t unit_order;      /* RP_UNITS_*: tile order or the learned per-unit order (ABI v8) */
} rp_scene_options;
/* ABI v9 removed the measured-and-lost options of v5-v8: `engine` / `wf_slots` (the stage-split
 * engine) and `primary` (the coherent primary pass). */

typedef struct rp_stats {
  uint64_t rays;      /* root scene.hit() calls, primary + secondary (render.rs:105,133) */
  uint64_t samples;   /* camera samples traced */
  uint64_t pixels;    /* pixels written */
  double seconds;     /* device time of the render (HIP events) */
} rp_stats;

typedef struct rp_scene rp_scene;   /* opaque: device-resident scene + acceleration structure */
typedef struct rp_workspace rp_workspace;  /* opaque: per-frame device state of a render (see below) */

/* Library / device queries.  rp_build_id: a hash of the machine code that decides a frame's per-ray work -- the render
 * kernel, the tree builders and the scheduling code -- this library was built from (profile records of the kernel carry
 * it; a record of another build is stale). */
int rp_abi_version(void);
const char* rp_build_id(void);
const char* rp_last_error(void);
int rp_device_count(int* count);

/* Build the acceleration structure and copy the scene to device `device`.  Validates every index the
 * reference would bounds-check (material/mesh/texture ids, triangle offsets, checker recursion).
 * rp_scene_create uses the default options; the library reads no environment variables. */
int rp_scene_create(const rp_scene_desc* desc, int device, rp_scene** out);
int rp_scene_options_init(rp_scene_options* opt);
int rp_scene_create_ex(const rp_scene_desc* desc, int device, const rp_scene_options* opt, rp_scene** out);
void rp_scene_destroy(rp_scene* scene);
/* Acceleration-structure statistics: node count, leaf count, max depth, primitive count. */
int rp_scene_info(const rp_scene* scene, uint64_t* n_nodes, uint64_t* n_leaves, uint32_t* max_depth,
                  uint64_t* n_prims, uint64_t* device_bytes);

/* Host wall-clock seconds of rp_scene_create's phases: {validation, host tree (or the shading tables alone for a
 * device build), device builder input (primitive records and boxes), device build (or the host tree's upload),
 * vertex/shading tables upload, workspace}.  RP_BUILD_PHASES values; n may be smaller. */
#define RP_BUILD_PHASES 6
int rp_scene_build_times(const rp_scene* scene, double* seconds, uint32_t n);

/* Number of pixels in shard params->shard (the length of the compact shard buffer). */
int rp_shard_pixel_count(const rp_render_params* params, uint64_t* count);
/* Scatter a compact shard buffer (shard order: its tiles in deal order k = 0, 1, ..., row-major inside a
 * tile) into a full frame; `channels` values per pixel.  RP_SHARD_INTERLEAVE frames only (a balanced frame is
 * refused with RP_EINVAL): rp_shard_unpack_map takes the deal order of a balanced frame (rp_workspace_tile_map;
 * NULL = the interleave). */
int rp_shard_unpack(const rp_render_params* params, const double* shard_buf, uint32_t channels,
                    double* frame);
int rp_shard_unpack_map(const rp_render_params* params, const uint32_t* tile_map, const double* shard_buf,
                        uint32_t channels, double* frame);

/* Render synchronously into host memory.  out_rgb: width*height*3 doubles (only the shard's pixels are
 * written).  out_foreground (nullable): width*height floats, fraction of samples whose first ray hit
 * geometry (main.rs:81-87).  stats nullable.  Reserves the scene workspace for params as needed. */
int rp_render(rp_scene* scene, const rp_camera* camera, const rp_render_params* params,
              double* out_rgb, float* out_foreground, rp_stats* stats);

/* Asynchronous device-resident render on `stream` (a hipStream_t, NULL = default stream) of the scene's
 * device.  d_shard_rgb: shard_pixel_count*3 doubles in device memory, compact shard order.
 * d_shard_fg (nullable): shard_pixel_count floats.  d_counters (nullable): RP_COUNTERS_LEN uint64 in
 * device memory that receive {rays, samples, pixels, status}; they are zeroed on the stream before the
 * launch.  No host synchronisation, copy or allocation happens inside.  A frame of more than one sample
 * batch (spp > samples_per_stream) keeps 3 doubles + 1 uint32 per pixel and batch in the workspace:
 * reserve them first (rp_workspace_reserve), else the call returns RP_EINVAL. */
int rp_render_device(rp_scene* scene, const rp_camera* camera, const rp_render_params* params,
                     double* d_shard_rgb, float* d_shard_fg, uint64_t* d_counters, void* stream);

/* Frames in flight.  A render's per-frame device state -- the keystream cache of the resident lanes,
 * the unit queues, the cost-probe and tile-order buffers, the multi-batch sums, the gather staging of
 * rp_frame_gather -- lives in a workspace.  The scene owns one, which rp_render and rp_render_device use
 * (their frames must therefore be ordered on one stream).  Frames rendered with different workspaces may
 * run concurrently on different streams: the end of one frame, when its last units leave most of the GPU
 * idle, then overlaps the start of the next.  A workspace serves one frame at a time (the caller orders
 * its reuse on streams); destroy workspaces before their scene.  Same arguments and results as
 * rp_render_device. */
int rp_workspace_create(rp_scene* scene, rp_workspace** out);
void rp_workspace_destroy(rp_workspace* workspace);
int rp_render_device_ws(rp_scene* scene, rp_workspace* workspace, const rp_camera* camera,
                        const rp_render_params* params, double* d_shard_rgb, float* d_shard_fg,
                        uint64_t* d_counters, void* stream);
/* Reserve the device memory renders of `params`' shape need in `workspace` (NULL = the scene's own):
 * the multi-batch sums of the shard and, when params->num_shards > 1, the staging buffers rp_frame_gather
 * uses for this frame size.  Synchronous (allocates; may free a smaller reservation); idempotent for a
 * shape it already covers.  rp_render reserves for itself. */
int rp_workspace_reserve(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params);
/* Scheduling costs.  Every render of the megakernel measures its units' durations per tile; a workspace that
 * rendered a whole frame on one device (num_shards = 1), or gathered one with rp_frame_gather, keeps them as a
 * learned per-tile cost table, and its next frame of the same geometry orders its tiles -- and deals them
 * (RP_SHARD_BALANCED) -- from that table instead of tracing a cost probe.  A balanced plan over N ranks only uses a
 * table gathered from N ranks (identical bytes on every rank, hence identical plans).  Callers that move shards
 * with their own collective get a render's measured costs with rp_workspace_tile_costs (2 x the shard's tile
 * count: summed unit durations per shard tile, then the longest unit; synchronises the device) and install a
 * frame's table, assembled through the deal order, with rp_workspace_set_tile_costs (2 x the frame's tile count:
 * sums, then longest units, by frame tile; `ranks` = how many ranks' renders it combines).  Results never
 * depend on any of it. */
int rp_workspace_tile_costs(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params,
                            uint32_t* costs, uint32_t n);
int rp_workspace_set_tile_costs(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params,
                                const uint32_t* costs, uint32_t ranks);
/* Several frames in ONE persistent launch (ABI v8).  Frame f = 0 .. n_frames - 1 is exactly the frame of `params` with
 * its sample batches numbered f * B .. f * B + B - 1, B = ceil(spp / samples_per_stream) -- i.e. the frame rp_render_device
 * renders with params.seed + f * B * width * height (the RNG contract's seeds of batches past the frame's own): n_frames
 * independent frames of the same scene, camera and sampling.  The queues hand out the frames' units one frame after
 * the other, so the lanes a frame's tail leaves take the next frame's units at once instead of idling in sparse waves
 * (a frame's tail: ~4 % of a C3 frame, ~20 % of an 8-way C3 shard).  d_shard_rgb holds n_frames shard
 * buffers back to back (3 x rp_shard_pixel_count doubles each), d_shard_fg (nullable) n_frames x pixel count floats;
 * d_counters: the n_frames frames' counts summed (status bits OR-ed).  The workspace must be reserved for n_frames
 * (rp_workspace_reserve_frames; it also reserves what rp_workspace_reserve does).  The shard's tiles (a balanced plan)
 * and their order are made once for the launch: from the workspace's learned cost table, or from a probe of frame 0 --
 * a probed plan follows its seed, so a balanced shard of frame f > 1 may hold other tiles than rp_render_device's frame
 * of that seed would (the pixels are the same; rp_workspace_tile_map gives the launch's deal).  n_frames <= RP_MAX_FRAMES.
 * frame_order (RP_FRAME_ORDER_*): SEQUENTIAL hands out frame 0's units, then frame 1's, ...; INTERLEAVED hands out the
 * frames' k-th tiles of the cost order together, for k = 0, 1, ... -- the units in flight at any moment come from a
 * narrower band of the cost order (fewer lanes idle in a wave whose neighbours run longer paths), every frame ends near
 * the launch's end.  PIXEL (ABI v9) is INTERLEAVED with a tile's units handed out pixel by pixel, each pixel's frames
 * consecutive (a wave holds a few pixels x their frames).  AUTO = INTERLEAVED.  The frames' pixels do not depend on it. */
#define RP_MAX_FRAMES 64
enum { RP_FRAME_ORDER_AUTO = 0, RP_FRAME_ORDER_SEQUENTIAL = 1, RP_FRAME_ORDER_INTERLEAVED = 2, RP_FRAME_ORDER_PIXEL = 3 };
int rp_workspace_reserve_frames(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params,
                                uint32_t n_frames);
int rp_render_frames_device_ws(rp_scene* scene, rp_workspace* workspace, const rp_camera* camera,
                               const rp_render_params* params, uint32_t n_frames, uint32_t frame_order,
                               double* d_shard_rgb,
                               float* d_shard_fg, uint64_t* d_counters, void* stream);
/* How the last render enqueued with `workspace` (NULL = the scene's) was scheduled (ABI v8): RP_FRAME_* bits (0 after
 * a render that launched nothing: spp = 0, an empty shard, a refused call).  Host state only (no device
 * synchronisation); results never depend on any of it.  (Bit 1 belonged to the coherent primary pass, removed in v9.) */
enum {
  RP_FRAME_LEARNED_ORDER = 2, /* tiles ordered / dealt from the workspace's learned cost table */
  RP_FRAME_PROBED = 4,        /* a cost probe launch ran */
  RP_FRAME_UNIT_ORDER = 8     /* units handed out in the learned per-unit order (rp_scene_options.unit_order) */
};
int rp_workspace_frame_info(const rp_scene* scene, const rp_workspace* workspace, uint32_t* flags);
/* Inspection of the learned per-unit order (ABI v9; tests and tools): the last render with `workspace` (NULL = the
 * scene's) stored each of its units' durations in 100 MHz ticks -- unit u = slot * nbatch + batch in shard order --
 * when it could learn them (one frame per launch, unit_order LEARNED or AUTO with one stream per pixel, a reserved
 * workspace), and handed its units out in `order` when its frame_info has RP_FRAME_UNIT_ORDER.  Copies n entries of each
 * (NULL = skip) to the host; n must not exceed the workspace's reservation.  Synchronises the device. */
int rp_workspace_unit_order(rp_scene* scene, rp_workspace* workspace, uint32_t* durations, uint32_t* order, uint64_t n);
/* The deal order of params' frame (one entry per frame tile; shard s's k-th tile is tile_map[s + k*num_shards]):
 * for RP_SHARD_BALANCED the plan the last render of this frame in `workspace` (NULL = the scene's) made, for the
 * interleave 0, 1, 2, ...  n >= the frame's tile count.  Synchronises the device. */
int rp_workspace_tile_map(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params,
                          uint32_t* tile_map, uint32_t n);

/* Output stage on the device: the reference's to_srgb_u8 (utility.rs:212-220, alpha 255) of every slot of
 * a compact shard buffer, bytes in tga::save's pixel order B, G, R, A (image.rs:116-137), so a gathered
 * and de-interleaved frame is the body of the reference's output.tga (18-byte header: rph_tga_save).
 * d_shard_bgra: shard_pixel_count * 4 bytes, 4-byte aligned.  Asynchronous on `stream`.  Bytes are
 * identical to to_srgb_u8 evaluated with the host libm's pow: the device looks x up in the 255
 * thresholds of that step function (rp_srgb_thresholds), it evaluates no pow of its own. */
int rp_shard_to_bgra8(rp_scene* scene, const rp_render_params* params, const double* d_shard_rgb,
                      uint8_t* d_shard_bgra, void* stream);
/* The threshold table of rp_shard_to_bgra8: out[k] (k = 1..255) is the smallest x whose to_srgb_u8 byte
 * is >= k; out[0] = -inf.  256 doubles.  Host only (no device needed). */
int rp_srgb_thresholds(double* out);

/* Closest-hit query (Hittable::hit on the root, hittable.rs:18 / bvh.rs:121) for n rays, synchronous,
 * host buffers.  rays: n * 8 doubles {origin xyz, direction xyz, t_min, t_max} (utility.rs:52-57).
 * out_hit: n * 9 doubles {t, position xyz, normal xyz, u, v} (utility.rs:84-89), t = +inf on a miss.
 * out_material: n uint32 (MaterialId, 0xffffffff on a miss).  Used to test the traversal in isolation. */
int rp_intersect(rp_scene* scene, const double* rays, uint64_t n, double* out_hit, uint32_t* out_material);

/* Diagnostic counters accumulated by renders since the last reset (non-zero only in the diagnostic
 * build lib/librp_diag.so, whose kernel carries s_memtime phase stamps): wave-cycles per phase
 * {fetch, new sample, traverse, shade, tail}, wave loop iterations, active lanes at traversal,
 * traversal wave-trips, lane node visits, lane primitive tests.  Synchronises the device. */
int rp_diagnostics(rp_scene* scene, uint64_t* out, uint32_t n, int reset);

/* ---------------------------------------------------------------- multi-GPU -- */
/* Image tiles are dealt across the GPUs (params.shard = rank, params.shard_map: the interleave tile t -> rank
 * t % nranks, or the balanced plan), every GPU holds its own copy of the scene, and one RCCL all-gather over xGMI
 * per frame moves the shards; each rank then de-interleaves them into frame order on its device.  This replaces the reference's
 * thread tile queue (main.rs:36-106, num_workers main.rs:27).  The per-pixel RNG contract makes the
 * gathered frame bitwise identical for any number of GPUs. */
typedef struct rp_comm rp_comm;     /* opaque: one rank's RCCL communicator (one device) */
typedef struct rp_multi rp_multi;   /* opaque: a scene on several devices of this process + communicator */

/* One process per GPU (torch.distributed / MPI style): rank 0 makes the id, every rank receives its bytes
 * out of band and joins.  `device` is the rank's HIP device (the scene's). */
int rp_comm_unique_id(uint8_t id[RP_COMM_ID_BYTES]);
int rp_comm_create(const uint8_t id[RP_COMM_ID_BYTES], int nranks, int rank, int device, rp_comm** out);
void rp_comm_destroy(rp_comm* comm);
int rp_comm_info(const rp_comm* comm, int* nranks, int* rank, int* device);

/* Collective over all ranks of `comm`, asynchronous on `stream` (every rank must call it, in the same
 * order relative to its other collectives on comm).  params: this rank's shard (shard = rank, num_shards
 * = nranks), the workspace reserved for it (rp_workspace_reserve) -- for RP_SHARD_BALANCED the workspace that
 * rendered the shard (it holds the plan).  d_shard_rgb: the rank's finished shard (rp_render_device_ws output).
 * Outputs (either nullable, on the rank's device, frame order, row 0 = bottom): d_frame_bgra width*height*4
 * bytes = to_srgb_u8 in tga::save byte order (rp_shard_to_bgra8) -- the body of output.tga; d_frame_rgb
 * width*height*3 linear f64.  Every rank must pass the same NULL / non-NULL combination of d_frame_bgra and
 * d_frame_rgb: the collectives issued are, in this order, ONE all-gather of every rank's packed block -- its counter
 * block, its measured tile costs (zeros for frames of more than 16384 tiles) and, with d_frame_bgra, its BGRA8
 * shard -- and, with d_frame_rgb, one of the f64 shards.  d_counters (nullable): the rank's
 * RP_COUNTERS_LEN counters in, the frame's out -- rays, samples and pixels summed over the ranks, status bits
 * OR-ed over them, plus RP_STATUS_PLAN_MISMATCH when the ranks' balanced plans differ.  A caller that does not
 * pass counters does not learn the status.  Tile costs (the collectives also all-gather every rank's measured
 * tile costs for frames of <= 16384 tiles) and the balanced plan live in the workspace: the gather reads the
 * workspace's plan and measured costs and writes its learned cost table on `stream`, and the next render with the
 * same workspace rewrites the first two and reads the third on ITS stream.  The library orders the two itself: the
 * gather records an event in the workspace at its end, and the next render with that workspace makes its stream wait
 * on it (a caller with separate render and gather streams cannot race them).  Frames in flight use one workspace
 * per frame. */
int rp_frame_gather(rp_comm* comm, rp_scene* scene, rp_workspace* workspace, const rp_render_params* params,
                    const double* d_shard_rgb, uint8_t* d_frame_bgra, double* d_frame_rgb,
                    uint64_t* d_counters, void* stream);
/* rp_frame_gather for the n_frames shards of one rp_render_frames_device_ws launch (d_shard_rgb: its n_frames shard
 * buffers back to back) in ONE all-gather: every rank's packed block carries its counter block (the launch's sums),
 * its measured tile costs and the n_frames shards' BGRA8 bytes one after the other; d_frames_bgra (nullable) receives
 * n_frames assembled frames of width*height*4 bytes back to back.  BGRA8 only (rp_frame_gather gathers f64 frames).
 * One collective per launch instead of one per frame: an RCCL all-gather kernel waits for a CU the render waves leave
 * (DESIGN.md 6).  The workspace must be reserved with rp_workspace_reserve_frames for n_frames. */
int rp_frames_gather(rp_comm* comm, rp_scene* scene, rp_workspace* workspace, const rp_render_params* params,
                     uint32_t n_frames, const double* d_shard_rgb, uint8_t* d_frames_bgra, uint64_t* d_counters,
                     void* stream);
/* rp_frames_gather in two halves around a collective of the caller's own (ABI v9; MPI, a torch.distributed
 * all-gather, tests): rp_frames_block_words gives the words (uint32) of one rank's packed block for n_frames frames of
 * params' shape -- the counter block and plan hash, the measured tile costs, then frame f's to_srgb_u8 bytes at a fixed
 * offset per frame; rp_frames_pack writes this rank's block (params.shard of params.num_shards) into d_send; the caller
 * all-gathers the num_shards blocks rank by rank into d_recv (rank r's block at r * words); rp_frames_unpack then does
 * what rp_frames_gather does after its collective: counters reduced into d_counters (sums, status OR-ed, plan hashes
 * compared), the gathered tile costs learned, and the n_frames frames assembled into d_frames_bgra.  Same workspace
 * reservation and rules as rp_frames_gather; asynchronous on `stream`. */
int rp_frames_block_words(const rp_render_params* params, uint32_t n_frames, uint64_t* words);
int rp_frames_pack(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params, uint32_t n_frames,
                   const double* d_shard_rgb, const uint64_t* d_counters, uint32_t* d_send, void* stream);
int rp_frames_unpack(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params, uint32_t n_frames,
                     const uint32_t* d_recv, uint8_t* d_frames_bgra, uint64_t* d_counters, void* stream);
/* The frame assembly step alone, for callers that move the shards with their own collective (MPI, a
 * torch.distributed all-gather): d_gathered holds params->num_shards shard buffers of `stride` slots each
 * (rp_gather_stride: the largest shard, shard 0), rank r's at slot r * stride, `words_per_slot` 32-bit words
 * per slot (1 for the BGRA8 bytes of rp_shard_to_bgra8, 6 for f64 RGB); d_frame receives width*height
 * slots in frame order.  Asynchronous on `stream`, on the current device. */
int rp_gather_stride(const rp_render_params* params, uint64_t* stride);
/* RP_SHARD_INTERLEAVE frames; a balanced frame is refused (RP_EINVAL): rp_frame_assemble_ws assembles with the
 * plan held by the workspace that rendered this rank's shard of the frame. */
int rp_frame_assemble(const rp_render_params* params, const void* d_gathered, uint32_t words_per_slot,
                      void* d_frame, void* stream);
int rp_frame_assemble_ws(rp_scene* scene, rp_workspace* workspace, const rp_render_params* params,
                         const void* d_gathered, uint32_t words_per_slot, void* d_frame, void* stream);

/* rp_render_device_ws into the workspace's shard buffer, then rp_frame_gather, on one stream. */
int rp_render_gather(rp_comm* comm, rp_scene* scene, rp_workspace* workspace, const rp_camera* camera,
                     const rp_render_params* params, uint8_t* d_frame_bgra, double* d_frame_rgb,
                     uint64_t* d_counters, void* stream);

/* One process, several GPUs (the reference's single-process model): a scene copy per device, one
 * communicator over them (ncclCommInitAll), one stream per device. */
int rp_multi_create(const rp_scene_desc* desc, const int* devices, int n_devices, const rp_scene_options* opt,
                    rp_multi** out);
void rp_multi_destroy(rp_multi* multi);
/* Synchronous frame on every device of `multi` (params.shard / num_shards are ignored: device k renders
 * shard k of n_devices; params.shard_map applies -- RP_SHARD_BALANCED is the better split).  out_rgb
 * (nullable): width*height*3 doubles on the host, frame order; out_bgra (nullable): width*height*4 bytes
 * (to_srgb_u8, tga::save order).  stats (nullable): summed counters, seconds = wall time of the frame.  Returns
 * RP_EINTERNAL when any device reported a status bit (stack overflow, plan mismatch). */
int rp_render_multi(rp_multi* multi, const rp_camera* camera, const rp_render_params* params,
                    double* out_rgb, uint8_t* out_bgra, rp_stats* stats);

#ifdef __cplusplus
}
#endif

#endif /* RP_H */
