/*
 * rp_host.h -- C-ABI of librp_host.so: the host pieces around the hot path, in C++ (the reference's
 * Rust host -- example_scenes.rs, mesh.rs obj::load, image.rs tga::load/save, utility.rs lookat /
 * to_srgb_u8 -- cannot be built in this image).  A Rust host keeps its own; these exist so that C/C++
 * and Python callers (tests, bench.py) can build the reference scenes without Rust.
 * No GPU code: this library loads and runs on any host.
 */
#ifndef RP_HOST_H
#define RP_HOST_H

#include <stdint.h>

#include "rp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* mesh.rs:145-183 obj::load: v/vn/vt/f lines, 1-based indices, (p, n, t) tuples deduplicated in
 * first-use order, missing normal -> (0,0,0), missing uv -> (0,0), non-triangular faces rejected.
 * Arrays are allocated by the library; release with rph_mesh_free. */
typedef struct rph_mesh {
  uint32_t n_vertices, n_indices;
  double* positions; /* 3 * n_vertices */
  double* normals;   /* 3 * n_vertices */
  double* uvs;       /* 2 * n_vertices */
  uint32_t* indices; /* n_indices */
} rph_mesh;

int rph_obj_load(const char* path, rph_mesh* out);  /* RP_OK or RP_EINVAL (message: rph_last_error) */
void rph_mesh_free(rph_mesh* m);

/* image.rs:73-114 tga::load: uncompressed 24/32-bit only; returns RGBA8 with row 0 = bottom row. */
int rph_tga_load(const char* path, uint32_t* width, uint32_t* height, uint8_t** rgba);
/* image.rs:116-137 tga::save: 32-bit BGRA, bottom-left origin. */
int rph_tga_save(const char* path, uint32_t width, uint32_t height, const uint8_t* rgba);
void rph_free(void* p);

/* utility.rs:212-220 to_srgb_u8 over n pixels of linear RGB (f64) -> RGBA8 (alpha 255). */
void rph_to_srgb_u8(const double* rgb, uint64_t n_pixels, uint8_t* rgba);

/* utility.rs:172-177 Transformation::lookat -> column-major orientation for rp_camera. */
void rph_lookat(const double position[3], const double target[3], const double up[3], double orientation[9]);

/* Deterministic stand-in for assets/sky_panorama.tga, which is missing from the reference mount
 * (.MISSING_LARGE_BLOBS:1): an equirectangular RGBA8 sky (gradient, sun disc, hashed value-noise
 * clouds built on randomness.rs noise::integer).  Row 0 = bottom (nadir), as tga::load stores it.
 * Pure integer and +,-,*,/,sqrt arithmetic: bit-identical on every IEEE host. */
int rph_sky_panorama(uint32_t width, uint32_t height, uint8_t* rgba);

/* Self-check of the acceleration-structure builder used by librp.so on a scene (CPU only):
 * validates the scene, builds the host tree in `node_format` (RP_NODES_*, AUTO = librp.so's size rule)
 * and checks its invariants.  stats (nullable, 4 values): {nodes, leaves, max_depth, primitives}. */
int rph_bvh_selfcheck(const rp_scene_desc* desc, uint32_t node_format, uint64_t* stats);

/* CPU model of the device traversal over the same packed tree in `node_format` (diagnostics): for n rays
 * (layout of rp_intersect) writes n x 3 {node records visited, primitive tests, closest hittable id or
 * 2^64-1}. */
int rph_bvh_traversal_stats(const rp_scene_desc* desc, const double* rays, uint64_t n, uint32_t node_format,
                            uint64_t* per_ray);
/* The two above with the 4-wide collapse chosen (RP_COLLAPSE_*, include/rp.h: the library's AUTO is SAH). */
int rph_bvh_selfcheck_ex(const rp_scene_desc* desc, uint32_t node_format, uint32_t collapse, uint64_t* stats);
int rph_bvh_traversal_stats_ex(const rp_scene_desc* desc, const double* rays, uint64_t n, uint32_t node_format,
                               uint32_t collapse, uint64_t* per_ray);

/* Hash (FNV-1a) of the packed host tree (node records and leaf-ordered primitive references) built with
 * `threads` build threads (0 = the machine's, at most 16): the tree does not depend on the thread count. */
int rph_bvh_tree_hash(const rp_scene_desc* desc, uint32_t node_format, uint32_t threads, uint64_t* hash);

/* rand 0.8 StdRng (ChaCha12, rand_chacha 0.3 stream: 64-bit block counter, zero nonce) keyed by the 32-byte
 * seed (StdRng::from_seed; seed_from_u64 seeds come from its PCG32 expansion): n consecutive next_u64
 * draws starting at draw index `first` (two keystream words each, little-endian).  Host bulk scene
 * generation (the synthetic C5 mesh: 120 M draws); multi-threaded. */
int rph_stdrng_u64(const uint8_t seed[32], uint64_t first, uint64_t n, uint64_t* out);

/* Test hook: the magic numbers of the render kernel's unit decode (raytracing-potato_amd/csrc/rp_kernel.h
 * rpk::make_div32, the same header the library's launches use): for a divisor d >= 1, m and s such that
 * floor(n / d) == (n * m) >> s (64-bit product) for every n < 2^31.  RP_EINVAL for d == 0. */
int rph_make_div32(uint32_t d, uint32_t* m, uint32_t* s);

const char* rph_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
