/*
 * rp_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, IEEE binary64, no FMA contraction) of alucas2/raytracing-potato's hot path,
 * used as the parity checker for librp.so and as the bench's cpu_baseline ("port": the Rust reference
 * cannot be built in this image -- no rustc/cargo, no vendored crates).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 * The product (librp.so, raytracing-potato_amd/) never links, loads or calls it.
 *
 * Parity status: the ChaCha/StdRng stream is pinned by known-answer vectors (RFC 7539 ChaCha20 block,
 * rand 0.8's own StdRng value-stability vector); image-level results are "parity unpinned" against the
 * Rust binary itself (it cannot run here) and are cross-checked by an independent Python restatement
 * (tests/golden/make_golden.py).
 */
#ifndef RP_ORACLE_H
#define RP_ORACLE_H

#include <stdint.h>
#include "../include/rp.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- rand 0.8 StdRng (rand_chacha 0.3 ChaCha12Rng, BlockRng with a 64-word buffer) ---- */
typedef struct or_rng {
  uint32_t key[8];
  uint64_t counter;     /* next block counter */
  uint32_t buf[64];     /* 4 blocks, as rand_chacha 0.3 refills */
  uint32_t index;       /* 0..64; 64 = empty */
  uint32_t rounds;      /* 12 for StdRng */
} or_rng;

void or_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, uint32_t rounds,
                     uint32_t out[16]);
void or_rng_from_seed(or_rng* r, const uint8_t seed[32], uint32_t rounds);
void or_rng_seed_from_u64(or_rng* r, uint64_t state);
uint32_t or_rng_next_u32(or_rng* r);
uint64_t or_rng_next_u64(or_rng* r);
void or_rng_fill_bytes(or_rng* r, uint8_t* dest, uint64_t len);
double or_rng_gen_f64(or_rng* r);
/* n draws of next_u64 from seed_from_u64(seed) (convenience for tests) */
void or_stream_u64(uint64_t seed, uint64_t n, uint64_t* out);

/* distributions (randomness.rs:9-82): write the sample(s) to out */
void or_sample_unit_disk(or_rng* r, double out[2]);
void or_sample_unit_ball(or_rng* r, double out[3]);
void or_sample_unit_sphere(or_rng* r, double out[3]);
int or_sample_bernoulli(or_rng* r, double p);
int64_t or_noise_integer(int64_t x, int64_t y, int64_t z, int64_t seed);
double or_noise_real(int64_t x, int64_t y, int64_t z, int64_t seed);

/* ---- camera frame (utility.rs:172-177) ---- */
void or_lookat(const double position[3], const double target[3], const double up[3], double orient[9]);

/* ---- scene ---- */
typedef struct or_scene or_scene;

/* counters[0..4] = {rays (root hit calls), aabb tests, triangle tests, sphere tests, samples} */
enum { OR_C_RAYS = 0, OR_C_BOX, OR_C_TRI, OR_C_SPH, OR_C_SAMPLES, OR_C_TRI_HITS, OR_C_TEXELS, OR_C_N };

or_scene* or_scene_create(const rp_scene_desc* desc);  /* builds the reference median-split BVH */
void or_scene_destroy(or_scene* s);
int or_scene_info(const or_scene* s, uint32_t* n_nodes, uint32_t* depth);

/* Hittable::hit on the root for n rays (same layout as rp_intersect). */
int or_intersect(or_scene* s, const double* rays, uint64_t n, double* out_hit, uint32_t* out_material,
                 uint64_t* counters);

/* Samples per RNG stream of the RNG contract (include/rp.h RP_SAMPLES_PER_STREAM). */
#define OR_SAMPLES_PER_STREAM RP_SAMPLES_PER_STREAM

/* Per-pixel-seeded render (the RNG contract: one stream per pixel and batch of OR_SAMPLES_PER_STREAM
 * samples), same output convention as rp_render (full frame, only the shard's pixels written).
 * threads >= 1; the result does not depend on it. */
int or_render(or_scene* s, const rp_camera* cam, const rp_render_params* p, double* out_rgb,
              float* out_fg, uint64_t* counters, int threads);

/* The reference driver (main.rs:36-106): LIFO tile queue behind a mutex, `workers` threads each with its
 * own StdRng (seed_from_u64(seed + worker) in place of from_entropy), recursive trace_path.  Returns the
 * wall seconds of the worker phase; out_rgb (nullable) receives the frame; counters summed. */
double or_render_baseline(or_scene* s, const rp_camera* cam, uint32_t width, uint32_t height,
                          uint32_t spp, uint32_t max_bounce, uint32_t tile, uint32_t workers,
                          uint64_t seed, double* out_rgb, uint64_t* counters);

/* ---- host I/O restatements (mesh.rs:145-183, image.rs:73-137, utility.rs:212-220) ---- */
typedef struct or_mesh_data {
  uint32_t n_vertices, n_indices;
  double *positions, *normals, *uvs;
  uint32_t* indices;
} or_mesh_data;
int or_obj_load(const char* path, or_mesh_data* out);  /* 0 ok, <0 error */
void or_mesh_free(or_mesh_data* m);
int or_tga_load(const char* path, uint32_t* w, uint32_t* h, uint8_t** rgba);
int or_tga_save(const char* path, uint32_t w, uint32_t h, const uint8_t* rgba);
void or_free(void* p);
void or_to_srgb_u8(const double* rgb, uint64_t n_pixels, uint8_t* rgba);

#ifdef __cplusplus
}
#endif
#endif
