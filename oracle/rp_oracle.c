/*
 * rp_oracle.c -- TEST INFRASTRUCTURE ONLY (see rp_oracle.h).
 *
 * Plain-C restatement of alucas2/raytracing-potato, operation for operation, in IEEE binary64.
 * Build with -O2 -ffp-contract=off -fno-fast-math (see Makefile): Rust does not contract a*b+c into an
 * FMA, so neither may we.  Every function cites the reference file:line it restates.  Third-party
 * arithmetic restated from the published algorithms of the crates pinned in Cargo.toml:8-12:
 *   rand 0.8.4 -> rand_core 0.6 (BlockRng, seed_from_u64 = PCG32 expansion), rand_chacha 0.3 (ChaCha12,
 *   64-bit block counter in words 12-13, zero nonce, 4-block buffer), Standard f64 = (u64 >> 11) * 2^-53;
 *   nalgebra 0.29 (dot = (x*x' + y*y') + z*z', normalize = component / norm, Matrix3 * Vector3 =
 *   column axpy ((c0*v0 + c1*v1) + c2*v2), cross);  nom 7.1 `double` == correctly rounded strtod.
 */
#include "rp_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* Per-event counters (box / triangle / sphere tests, triangle hits, texels) for the algorithmic-bytes
 * figures (tests/golden/event_counts.json).  The timed CPU baseline (liboracle_fast.so) is built with
 * -DOR_NO_EVENT_COUNTERS so it runs the reference's work and nothing more; rays and samples are always
 * counted (the Mrays/s numerator). */
#ifdef OR_NO_EVENT_COUNTERS
#define OR_EVENT(C, k) ((void)0)
#else
#define OR_EVENT(C, k) ((C)->c[k]++)
#endif

/* ================================================================ RNG ======================== */

static inline uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

#define QR(a, b, c, d)                  \
  a += b; d ^= a; d = rotl32(d, 16);    \
  c += d; b ^= c; b = rotl32(b, 12);    \
  a += b; d ^= a; d = rotl32(d, 8);     \
  c += d; b ^= c; b = rotl32(b, 7);

/* ChaCha block function (D. J. Bernstein; rand_chacha 0.3 guts.rs with a 64-bit counter in words
 * 12-13 and a 64-bit stream id in words 14-15). */
void or_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, uint32_t rounds,
                     uint32_t out[16]) {
  uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u,
                    key[0], key[1], key[2], key[3], key[4], key[5], key[6], key[7],
                    (uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)stream,
                    (uint32_t)(stream >> 32)};
  uint32_t x[16];
  memcpy(x, s, sizeof x);
  for (uint32_t r = 0; r < rounds; r += 2) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

static void rng_refill(or_rng* r) {
  /* rand_chacha 0.3 refills 4 consecutive blocks into a 64-word buffer */
  for (int b = 0; b < 4; b++) or_chacha_block(r->key, r->counter + (uint64_t)b, 0, r->rounds, r->buf + 16 * b);
  r->counter += 4;
}

/* rand_chacha 0.3 ChaChaXCore::from_seed: key = seed (LE words), counter 0, nonce 0. */
void or_rng_from_seed(or_rng* r, const uint8_t seed[32], uint32_t rounds) {
  for (int i = 0; i < 8; i++)
    r->key[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
                ((uint32_t)seed[4 * i + 3] << 24);
  r->counter = 0;
  r->index = 64;
  r->rounds = rounds;
  memset(r->buf, 0, sizeof r->buf);
}

/* rand_core 0.6 SeedableRng::seed_from_u64: PCG32 expansion of the u64 into the 32-byte seed. */
void or_rng_seed_from_u64(or_rng* r, uint64_t state) {
  const uint64_t MUL = 6364136223846793005ull, INC = 11634580027462260723ull;
  uint8_t seed[32];
  for (int c = 0; c < 8; c++) {
    state = state * MUL + INC;
    uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
    uint32_t rot = (uint32_t)(state >> 59);
    uint32_t x = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    seed[4 * c + 0] = (uint8_t)x;
    seed[4 * c + 1] = (uint8_t)(x >> 8);
    seed[4 * c + 2] = (uint8_t)(x >> 16);
    seed[4 * c + 3] = (uint8_t)(x >> 24);
  }
  or_rng_from_seed(r, seed, 12);
}

/* rand_core 0.6 BlockRng::next_u32 */
uint32_t or_rng_next_u32(or_rng* r) {
  if (r->index >= 64) { rng_refill(r); r->index = 0; }
  return r->buf[r->index++];
}

/* rand_core 0.6 BlockRng::next_u64 (all three index cases) */
uint64_t or_rng_next_u64(or_rng* r) {
  uint32_t idx = r->index;
  if (idx < 63) {
    r->index += 2;
    return ((uint64_t)r->buf[idx + 1] << 32) | r->buf[idx];
  } else if (idx >= 64) {
    rng_refill(r);
    r->index = 2;
    return ((uint64_t)r->buf[1] << 32) | r->buf[0];
  } else {
    uint64_t x = r->buf[63];
    rng_refill(r);
    r->index = 1;
    uint64_t y = r->buf[0];
    return (y << 32) | x;
  }
}

/* rand_core 0.6 BlockRng::fill_bytes / fill_via_u32_chunks */
void or_rng_fill_bytes(or_rng* r, uint8_t* dest, uint64_t len) {
  uint64_t read = 0;
  while (read < len) {
    if (r->index >= 64) { rng_refill(r); r->index = 0; }
    uint64_t avail_words = 64 - r->index;
    uint64_t want = len - read;
    uint64_t nbytes = want < avail_words * 4 ? want : avail_words * 4;
    for (uint64_t b = 0; b < nbytes; b++) dest[read + b] = (uint8_t)(r->buf[r->index + b / 4] >> (8 * (b % 4)));
    r->index += (uint32_t)((nbytes + 3) / 4);
    read += nbytes;
  }
}

/* rand 0.8 Standard for f64: multiply-based, 53 most significant bits, [0, 1). */
double or_rng_gen_f64(or_rng* r) {
  uint64_t v = or_rng_next_u64(r) >> 11;
  return (double)v * (1.0 / 9007199254740992.0);
}

void or_stream_u64(uint64_t seed, uint64_t n, uint64_t* out) {
  or_rng r;
  or_rng_seed_from_u64(&r, seed);
  for (uint64_t i = 0; i < n; i++) out[i] = or_rng_next_u64(&r);
}

/* randomness.rs:21-34 UnitDisk */
void or_sample_unit_disk(or_rng* r, double out[2]) {
  for (;;) {
    double x = 2.0 * or_rng_gen_f64(r) - 1.0;
    double y = 2.0 * or_rng_gen_f64(r) - 1.0;
    if (x * x + y * y < 1.0) { out[0] = x; out[1] = y; return; }
  }
}

/* randomness.rs:39-53 UnitBall */
void or_sample_unit_ball(or_rng* r, double out[3]) {
  for (;;) {
    double x = 2.0 * or_rng_gen_f64(r) - 1.0;
    double y = 2.0 * or_rng_gen_f64(r) - 1.0;
    double z = 2.0 * or_rng_gen_f64(r) - 1.0;
    if ((x * x + y * y) + z * z < 1.0) { out[0] = x; out[1] = y; out[2] = z; return; }
  }
}

/* randomness.rs:58-73 UnitSphere (Marsaglia) */
void or_sample_unit_sphere(or_rng* r, double out[3]) {
  for (;;) {
    double x = 2.0 * or_rng_gen_f64(r) - 1.0;
    double y = 2.0 * or_rng_gen_f64(r) - 1.0;
    double s = x * x + y * y;
    if (s < 1.0) {
      double n = 2.0 * sqrt(1.0 - s);
      out[0] = x * n; out[1] = y * n; out[2] = 1.0 - 2.0 * s;
      return;
    }
  }
}

/* randomness.rs:78-82 Bernoulli */
int or_sample_bernoulli(or_rng* r, double p) { return or_rng_gen_f64(r) < p; }

/* randomness.rs:91-105 noise::integer -- wrapping isize arithmetic, arithmetic >> 13 */
int64_t or_noise_integer(int64_t x, int64_t y, int64_t z, int64_t seed) {
  const uint64_t A = 0x369E6D3B899E43CFull, B = 0x53F89E7FFDA3B07Dull, C = 0x3B13C1CA4937E629ull,
                 D = 0x577C2C6E4019D645ull, E = 60493ull, F = 19990303ull, G = 1376312589ull;
  uint64_t h = A * (uint64_t)x + B * (uint64_t)y + C * (uint64_t)z + D * (uint64_t)seed;
  h = (uint64_t)((int64_t)h >> 13) ^ h;
  h = h * (h * h * E + F) + G;
  return (int64_t)h;
}

/* randomness.rs:108-110 noise::real */
double or_noise_real(int64_t x, int64_t y, int64_t z, int64_t seed) {
  return (double)or_noise_integer(x, y, z, seed) / (double)INT64_MAX;
}

/* ================================================================ math ======================= */

typedef struct { double x, y, z; } v3;

static inline v3 V(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return V(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mulc(v3 a, v3 b) { return V(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 smul(double s, v3 a) { return V(s * a.x, s * a.y, s * a.z); }
static inline v3 sdiv(v3 a, double s) { return V(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return V(-a.x, -a.y, -a.z); }
static inline double dot(v3 a, v3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }      /* nalgebra dot */
static inline double norm2(v3 a) { return (a.x * a.x + a.y * a.y) + a.z * a.z; }           /* norm_squared */
static inline v3 normalize(v3 a) { return sdiv(a, sqrt(norm2(a))); }                      /* a / |a| */
static inline v3 cross(v3 a, v3 b) {
  return V(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* nalgebra Matrix3 * Vector3 (gemv as column axpys): ((v0*c0) + v1*c1) + v2*c2 */
static inline v3 matvec(const double m[9], v3 v) {
  return V((v.x * m[0] + v.y * m[3]) + v.z * m[6], (v.x * m[1] + v.y * m[4]) + v.z * m[7],
           (v.x * m[2] + v.y * m[5]) + v.z * m[8]);
}

static const double RAY_EPSILON = 1e-3;  /* utility.rs:30 */
static const double SMOL = 1e-7;         /* utility.rs:31 */
static const double PI_ = 3.14159265358979323846;
static const double TAU_ = 6.28318530717958647692;

typedef struct { v3 o, d; double tmin, tmax; } ray_t;             /* utility.rs:52-57 */
typedef struct { ray_t r; v3 inv; } rayx_t;                       /* utility.rs:61-64 */
typedef struct { double t; v3 p, n; double u, v; } hit_t;          /* utility.rs:84-89 */

static inline v3 ray_at(const ray_t* r, double t) { return add(r->o, smul(t, r->d)); } /* utility.rs:67 */

/* utility.rs:93-100 Hit::at_infinity */
static hit_t hit_at_infinity(v3 d) {
  hit_t h;
  h.t = INFINITY;
  h.p = d;
  h.n = d;
  h.u = 0.5 - atan2(d.z, d.x) / TAU_;
  h.v = asin(d.y) / PI_ + 0.5;
  return h;
}

/* utility.rs:106-108 */
static inline v3 reflect(v3 i, v3 n) { return sub(i, smul(2.0 * dot(i, n), n)); }

/* utility.rs:111-119 */
static inline int refract(v3 i, v3 n, double eta, v3* out) {
  double cos_theta = dot(n, i);
  double k = 1.0 - eta * eta * (1.0 - cos_theta * cos_theta);
  if (k < 0.0) return 0;
  *out = sub(smul(eta, i), smul(eta * cos_theta + sqrt(k), n));
  return 1;
}

/* utility.rs:172-177 Transformation::lookat, column-major orientation */
void or_lookat(const double position[3], const double target[3], const double up[3], double orient[9]) {
  v3 p = V(position[0], position[1], position[2]);
  v3 t = V(target[0], target[1], target[2]);
  v3 u = V(up[0], up[1], up[2]);
  v3 z = normalize(sub(p, t));
  v3 x = cross(u, z);
  v3 y = cross(z, x);
  orient[0] = x.x; orient[1] = x.y; orient[2] = x.z;
  orient[3] = y.x; orient[4] = y.y; orient[5] = y.z;
  orient[6] = z.x; orient[7] = z.y; orient[8] = z.z;
}

typedef struct { double min[3], max[3]; } aabb_t;

/* utility.rs:137-154 AABB::collide; Rust f64::min/max ignore NaN like fmin/fmax */
static inline int aabb_collide(const aabb_t* b, const rayx_t* r) {
  double t0x = (b->min[0] - r->r.o.x) * r->inv.x, t0y = (b->min[1] - r->r.o.y) * r->inv.y,
         t0z = (b->min[2] - r->r.o.z) * r->inv.z;
  double t1x = (b->max[0] - r->r.o.x) * r->inv.x, t1y = (b->max[1] - r->r.o.y) * r->inv.y,
         t1z = (b->max[2] - r->r.o.z) * r->inv.z;
  double tmin = fmax(fmax(fmax(r->r.tmin, fmin(t0x, t1x)), fmin(t0y, t1y)), fmin(t0z, t1z));
  double tmax = fmin(fmin(fmin(r->r.tmax, fmax(t0x, t1x)), fmax(t0y, t1y)), fmax(t0z, t1z));
  return tmax >= tmin;
}

/* utility.rs:130-135 */
static inline aabb_t aabb_union(const aabb_t* a, const aabb_t* b) {
  aabb_t r;
  for (int k = 0; k < 3; k++) { r.min[k] = fmin(a->min[k], b->min[k]); r.max[k] = fmax(a->max[k], b->max[k]); }
  return r;
}

/* Rust `as` casts saturate and map NaN to 0 */
static inline uint32_t sat_u32(double x) {
  if (!(x > 0.0)) return 0;  /* NaN, negatives, -0 */
  if (x >= 4294967295.0) return 4294967295u;
  return (uint32_t)x;
}
static inline int64_t sat_i64(double x) {
  if (x != x) return 0;
  if (x >= 9223372036854775807.0) return INT64_MAX;
  if (x <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)x;
}
static inline uint8_t sat_u8(double x) {
  if (!(x > 0.0)) return 0;
  if (x >= 255.0) return 255;
  return (uint8_t)x;
}

/* ================================================================ scene ====================== */

typedef struct {
  uint32_t nv, ni, material;
  double *pos, *nrm, *uv;
  uint32_t* idx;
} mesh_t;

typedef struct {
  uint32_t kind, odd, even, w, h;
  int64_t seed;
  double color[3];
  uint8_t* rgba;
} tex_t;

typedef struct {
  int is_leaf;
  aabb_t box;
  uint32_t left, right, leaf;
} node_t;  /* bvh.rs:12-15 */

struct or_scene {
  uint32_t root_kind;
  uint32_t n_hit;
  rp_hittable* hit;  /* Bvh.leaves / List */
  uint32_t n_mesh;
  mesh_t* mesh;
  uint32_t n_mat;
  rp_material* mat;
  uint32_t n_tex;
  tex_t* tex;
  rp_emit background;
  uint32_t n_nodes, root, depth;
  node_t* nodes;
};

typedef struct { uint64_t c[OR_C_N]; } ctr_t;

/* mesh.rs:25-30 get_triangle (positions only for bounding boxes) */
static inline v3 vpos(const mesh_t* m, uint32_t vi) { return V(m->pos[3 * vi], m->pos[3 * vi + 1], m->pos[3 * vi + 2]); }
static inline v3 vnrm(const mesh_t* m, uint32_t vi) { return V(m->nrm[3 * vi], m->nrm[3 * vi + 1], m->nrm[3 * vi + 2]); }

/* hittable.rs:124-129, 131-140 */
static aabb_t hittable_bbox(const or_scene* s, const rp_hittable* h) {
  aabb_t b;
  if (h->kind == RP_HITTABLE_SPHERE) {
    for (int k = 0; k < 3; k++) { b.min[k] = h->center[k] - h->radius; b.max[k] = h->center[k] + h->radius; }
  } else {
    const mesh_t* m = &s->mesh[h->mesh];
    v3 a = vpos(m, m->idx[h->triangle]), bb = vpos(m, m->idx[h->triangle + 1]), c = vpos(m, m->idx[h->triangle + 2]);
    b.min[0] = fmin(fmin(a.x, bb.x), c.x); b.min[1] = fmin(fmin(a.y, bb.y), c.y); b.min[2] = fmin(fmin(a.z, bb.z), c.z);
    b.max[0] = fmax(fmax(a.x, bb.x), c.x); b.max[1] = fmax(fmax(a.y, bb.y), c.y); b.max[2] = fmax(fmax(a.z, bb.z), c.z);
  }
  return b;
}

typedef struct { uint32_t leaf; aabb_t box; } content_t;

/* bvh.rs:58-67 split: sort by centroid along the axis, split_at_mut(len / 2).  Rust's sort_unstable_by
 * orders equal centroids in an implementation-defined way; ties are broken by leaf id here (tree shape is
 * not part of the contract: SURVEY.md 8a A9), which makes the order total.  Under a total order the left
 * half is exactly the len/2 smallest elements and each half is sorted again on the next axis before it is
 * split, so the tree only depends on which elements go left, not on their order inside a half: a
 * selection (quickselect) of the len/2 smallest builds the identical tree in O(n) per level instead of
 * a full sort. */
static int less_centroid(const content_t* a, const content_t* b, int axis) {
  double ca = 0.5 * (a->box.min[axis] + a->box.max[axis]);
  double cb = 0.5 * (b->box.min[axis] + b->box.max[axis]);
  if (ca < cb) return 1;
  if (ca > cb) return 0;
  return a->leaf < b->leaf;
}

static void swap_content(content_t* a, content_t* b) {
  content_t t = *a; *a = *b; *b = t;
}

/* Afterwards c[0..k) are the k smallest of c[0..n) in the total order. */
static void select_smallest(content_t* c, uint32_t n, uint32_t k, int axis) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 16) {
    uint32_t m = lo + (hi - lo) / 2, e = hi - 1;
    /* median of three as the pivot, moved to e */
    if (less_centroid(&c[m], &c[lo], axis)) swap_content(&c[m], &c[lo]);
    if (less_centroid(&c[e], &c[lo], axis)) swap_content(&c[e], &c[lo]);
    if (less_centroid(&c[m], &c[e], axis)) swap_content(&c[m], &c[e]);
    uint32_t i = lo;
    for (uint32_t j = lo; j < e; j++)
      if (less_centroid(&c[j], &c[e], axis)) swap_content(&c[i++], &c[j]);
    swap_content(&c[i], &c[e]);
    if (i == k) return;
    if (k < i) hi = i;
    else lo = i + 1;
  }
  for (uint32_t i = lo + 1; i < hi; i++)  /* insertion sort of the last small range */
    for (uint32_t j = i; j > lo && less_centroid(&c[j], &c[j - 1], axis); j--) swap_content(&c[j], &c[j - 1]);
}

/* bvh.rs:36-56 make_bvh (post-order node array): the subtree of n leaves occupies nodes [base, base+2n-1),
 * left subtree first, then the right, the branch last -- so the two halves can be built concurrently. */
typedef struct {
  content_t* c;
  uint32_t n, base, depth, maxdepth;
  int axis;
  node_t* nodes;
} bvh_job_t;

static void* make_bvh_job(void* arg);

static void make_bvh(bvh_job_t* J) {
  if (J->depth > J->maxdepth) J->maxdepth = J->depth;
  node_t* nodes = J->nodes;
  if (J->n == 1) {
    node_t* nd = &nodes[J->base];
    nd->is_leaf = 1; nd->box = J->c[0].box; nd->leaf = J->c[0].leaf; nd->left = nd->right = 0;
    return;
  }
  uint32_t h = J->n / 2;
  select_smallest(J->c, J->n, h, J->axis);
  bvh_job_t L = {J->c, h, J->base, J->depth + 1, J->depth + 1, (J->axis + 1) % 3, nodes};
  bvh_job_t R = {J->c + h, J->n - h, J->base + 2 * h - 1, J->depth + 1, J->depth + 1, (J->axis + 1) % 3, nodes};
  pthread_t th;
  int spawned = J->depth < 5 && J->n >= (1u << 16) && pthread_create(&th, NULL, make_bvh_job, &L) == 0;
  if (!spawned) make_bvh(&L);
  make_bvh(&R);
  if (spawned) pthread_join(th, NULL);
  uint32_t l = L.base + 2 * L.n - 2, r = R.base + 2 * R.n - 2;
  node_t* nd = &nodes[J->base + 2 * J->n - 2];
  nd->is_leaf = 0; nd->left = l; nd->right = r; nd->leaf = 0;
  nd->box = aabb_union(&nodes[l].box, &nodes[r].box);
  if (L.maxdepth > J->maxdepth) J->maxdepth = L.maxdepth;
  if (R.maxdepth > J->maxdepth) J->maxdepth = R.maxdepth;
}

static void* make_bvh_job(void* arg) {
  make_bvh((bvh_job_t*)arg);
  return NULL;
}

static char g_err[256];

or_scene* or_scene_create(const rp_scene_desc* d) {
  if (!d || d->n_hittables == 0) return NULL;
  or_scene* s = (or_scene*)calloc(1, sizeof *s);
  s->root_kind = d->root_kind;
  s->n_hit = d->n_hittables;
  s->hit = (rp_hittable*)malloc(sizeof(rp_hittable) * d->n_hittables);
  memcpy(s->hit, d->hittables, sizeof(rp_hittable) * d->n_hittables);
  s->n_mesh = d->n_meshes;
  s->mesh = (mesh_t*)calloc(d->n_meshes ? d->n_meshes : 1, sizeof(mesh_t));
  for (uint32_t i = 0; i < d->n_meshes; i++) {
    const rp_mesh* m = &d->meshes[i];
    mesh_t* o = &s->mesh[i];
    o->nv = m->n_vertices; o->ni = m->n_indices; o->material = m->material;
    o->pos = (double*)malloc(sizeof(double) * 3 * (m->n_vertices + 1));
    o->nrm = (double*)malloc(sizeof(double) * 3 * (m->n_vertices + 1));
    o->uv = (double*)malloc(sizeof(double) * 2 * (m->n_vertices + 1));
    o->idx = (uint32_t*)malloc(sizeof(uint32_t) * (m->n_indices + 1));
    memcpy(o->pos, m->positions, sizeof(double) * 3 * m->n_vertices);
    memcpy(o->nrm, m->normals, sizeof(double) * 3 * m->n_vertices);
    memcpy(o->uv, m->uvs, sizeof(double) * 2 * m->n_vertices);
    memcpy(o->idx, m->indices, sizeof(uint32_t) * m->n_indices);
  }
  s->n_mat = d->n_materials;
  s->mat = (rp_material*)malloc(sizeof(rp_material) * (d->n_materials + 1));
  memcpy(s->mat, d->materials, sizeof(rp_material) * d->n_materials);
  s->n_tex = d->n_textures;
  s->tex = (tex_t*)calloc(d->n_textures + 1, sizeof(tex_t));
  for (uint32_t i = 0; i < d->n_textures; i++) {
    const rp_texture* t = &d->textures[i];
    tex_t* o = &s->tex[i];
    o->kind = t->kind; o->odd = t->odd; o->even = t->even; o->w = t->width; o->h = t->height;
    o->seed = t->seed;
    memcpy(o->color, t->color, sizeof o->color);
    if (t->kind == RP_TEXTURE_IMAGE) {
      size_t nb = (size_t)t->width * t->height * 4;
      o->rgba = (uint8_t*)malloc(nb ? nb : 1);
      memcpy(o->rgba, t->rgba, nb);
    }
  }
  s->background = d->background;
  if (s->root_kind == RP_ROOT_BVH) {
    /* bvh.rs:70-91 Bvh::new */
    content_t* c = (content_t*)malloc(sizeof(content_t) * s->n_hit);
    for (uint32_t i = 0; i < s->n_hit; i++) { c[i].leaf = i; c[i].box = hittable_bbox(s, &s->hit[i]); }
    s->nodes = (node_t*)malloc(sizeof(node_t) * (2 * s->n_hit));
    bvh_job_t J = {c, s->n_hit, 0, 0, 0, 0, s->nodes};
    make_bvh(&J);
    s->root = 2 * s->n_hit - 2;
    s->n_nodes = 2 * s->n_hit - 1;
    s->depth = J.maxdepth;
    free(c);
  }
  return s;
}

void or_scene_destroy(or_scene* s) {
  if (!s) return;
  for (uint32_t i = 0; i < s->n_mesh; i++) {
    free(s->mesh[i].pos); free(s->mesh[i].nrm); free(s->mesh[i].uv); free(s->mesh[i].idx);
  }
  for (uint32_t i = 0; i < s->n_tex; i++) free(s->tex[i].rgba);
  free(s->mesh); free(s->mat); free(s->tex); free(s->hit); free(s->nodes); free(s);
}

int or_scene_info(const or_scene* s, uint32_t* n_nodes, uint32_t* depth) {
  if (n_nodes) *n_nodes = s->n_nodes;
  if (depth) *depth = s->depth;
  return 0;
}

/* ---- intersection ---- */

typedef struct { int valid; hit_t h; uint32_t material; } hitm_t;

/* hittable.rs:39-63 */
static hitm_t hit_sphere(const rp_hittable* sp, const ray_t* r, ctr_t* C) {
  hitm_t res; res.valid = 0;
  OR_EVENT(C, OR_C_SPH);
  v3 center = V(sp->center[0], sp->center[1], sp->center[2]);
  double radius = sp->radius;
  v3 to_center = sub(r->o, center);
  double a = norm2(r->d);
  double half_b = dot(r->d, to_center);
  double c = norm2(to_center) - radius * radius;
  double delta = half_b * half_b - a * c;
  if (delta <= 0.0) return res;
  double sqrt_delta = sqrt(delta);
  double t = (-half_b - sqrt_delta) / a;
  if (t < r->tmin || t > r->tmax) {
    t = (-half_b + sqrt_delta) / a;
    if (t < r->tmin || t > r->tmax) return res;
  }
  res.valid = 1;
  res.h.t = t;
  res.h.p = ray_at(r, t);
  res.h.n = normalize(sub(res.h.p, center));
  res.h.u = 0.5 - atan2(res.h.n.z, res.h.n.x) / TAU_;
  res.h.v = asin(res.h.n.y) / PI_ + 0.5;
  res.material = sp->material;
  return res;
}

/* hittable.rs:65-108 (exact expression order) */
static hitm_t hit_triangle(const or_scene* s, const rp_hittable* tr, const ray_t* r, ctr_t* C) {
  hitm_t res; res.valid = 0;
  OR_EVENT(C, OR_C_TRI);
  const mesh_t* m = &s->mesh[tr->mesh];
  uint32_t i0 = m->idx[tr->triangle], i1 = m->idx[tr->triangle + 1], i2 = m->idx[tr->triangle + 2];
  v3 a = vpos(m, i0), b = vpos(m, i1), c = vpos(m, i2);
  v3 ba = sub(a, b), ca = sub(a, c), pa = sub(a, r->o), d = r->d;
  double det = ba.x * ca.y * d.z + ba.y * ca.z * d.x + ba.z * ca.x * d.y
             - ba.x * ca.z * d.y - ba.y * ca.x * d.z - ba.z * ca.y * d.x;
  if (fabs(det) < SMOL) return res;
  double inv_det = 1.0 / det;
  double t = (pa.x * (ba.y * ca.z - ba.z * ca.y)
            + pa.y * (ba.z * ca.x - ba.x * ca.z)
            + pa.z * (ba.x * ca.y - ba.y * ca.x)) * inv_det;
  double u = (pa.x * (ca.y * d.z - ca.z * d.y)
            + pa.y * (ca.z * d.x - ca.x * d.z)
            + pa.z * (ca.x * d.y - ca.y * d.x)) * inv_det;
  double v = (pa.x * (ba.z * d.y - ba.y * d.z)
            + pa.y * (ba.x * d.z - ba.z * d.x)
            + pa.z * (ba.y * d.x - ba.x * d.y)) * inv_det;
  double w = 1.0 - u - v;
  if (t < r->tmin || t > r->tmax || u < 0.0 || v < 0.0 || w < 0.0) return res;
  OR_EVENT(C, OR_C_TRI_HITS);
  res.valid = 1;
  res.h.t = t;
  res.h.p = ray_at(r, t);
  v3 n0 = vnrm(m, i0), n1 = vnrm(m, i1), n2 = vnrm(m, i2);
  res.h.n = add(add(smul(w, n0), smul(u, n1)), smul(v, n2));
  res.h.u = (w * m->uv[2 * i0] + u * m->uv[2 * i1]) + v * m->uv[2 * i2];
  res.h.v = (w * m->uv[2 * i0 + 1] + u * m->uv[2 * i1 + 1]) + v * m->uv[2 * i2 + 1];
  res.material = m->material;
  return res;
}

static hitm_t hittable_hit(const or_scene* s, const rp_hittable* h, const ray_t* r, ctr_t* C) {
  if (h->kind == RP_HITTABLE_SPHERE) return hit_sphere(h, r, C);
  return hit_triangle(s, h, r, C);
}

/* bvh.rs:93-119 hit_node (recursive DFS, box test on every node, left then right) */
static hitm_t hit_node(const or_scene* s, const rayx_t* ray, uint32_t node, ctr_t* C) {
  const node_t* nd = &s->nodes[node];
  hitm_t none; none.valid = 0;
  OR_EVENT(C, OR_C_BOX);
  if (nd->is_leaf) {
    if (aabb_collide(&nd->box, ray)) return hittable_hit(s, &s->hit[nd->leaf], &ray->r, C);
    return none;
  }
  if (!aabb_collide(&nd->box, ray)) return none;
  hitm_t hit; hit.valid = 0;
  rayx_t rr = *ray;
  hitm_t nh = hit_node(s, &rr, nd->left, C);
  if (nh.valid) { rr.r.tmax = nh.h.t; hit = nh; }
  nh = hit_node(s, &rr, nd->right, C);
  if (nh.valid) hit = nh;
  return hit;
}

/* hittable.rs:110-120 hit_list */
static hitm_t hit_list(const or_scene* s, const ray_t* ray, ctr_t* C) {
  hitm_t hit; hit.valid = 0;
  ray_t r = *ray;
  for (uint32_t i = 0; i < s->n_hit; i++) {
    hitm_t nh = hittable_hit(s, &s->hit[i], &r, C);
    if (nh.valid) { r.tmax = nh.h.t; hit = nh; }
  }
  return hit;
}

/* hittable.rs:18-25 on the root; bvh.rs:121-124 Bvh::hit */
static hitm_t scene_hit(const or_scene* s, const ray_t* r, ctr_t* C) {
  C->c[OR_C_RAYS]++;
  if (s->root_kind == RP_ROOT_LIST) return hit_list(s, r, C);
  rayx_t x;
  x.r = *r;
  x.inv = V(1.0 / r->d.x, 1.0 / r->d.y, 1.0 / r->d.z);  /* utility.rs:71-77 expand */
  return hit_node(s, &x, s->root, C);
}

int or_intersect(or_scene* s, const double* rays, uint64_t n, double* out_hit, uint32_t* out_material,
                 uint64_t* counters) {
  ctr_t C; memset(&C, 0, sizeof C);
  for (uint64_t i = 0; i < n; i++) {
    const double* q = rays + 8 * i;
    ray_t r; r.o = V(q[0], q[1], q[2]); r.d = V(q[3], q[4], q[5]); r.tmin = q[6]; r.tmax = q[7];
    hitm_t h = scene_hit(s, &r, &C);
    double* o = out_hit + 9 * i;
    if (h.valid) {
      o[0] = h.h.t; o[1] = h.h.p.x; o[2] = h.h.p.y; o[3] = h.h.p.z;
      o[4] = h.h.n.x; o[5] = h.h.n.y; o[6] = h.h.n.z; o[7] = h.h.u; o[8] = h.h.v;
      out_material[i] = h.material;
    } else {
      o[0] = INFINITY;
      for (int k = 1; k < 9; k++) o[k] = 0.0;
      out_material[i] = 0xffffffffu;
    }
  }
  if (counters) for (int k = 0; k < OR_C_N; k++) counters[k] += C.c[k];
  return 0;
}

/* ---- textures (texture.rs:21-118) ---- */

static v3 tex_sample(const or_scene* s, uint32_t tid, const hit_t* h, ctr_t* C);

static double grad_dot(v3 p, int64_t cx, int64_t cy, int64_t cz, int64_t seed) {  /* texture.rs:70-77 */
  v3 g = V(or_noise_real(cx, cy, cz, (int64_t)((uint64_t)seed + 1)),
           or_noise_real(cx, cy, cz, (int64_t)((uint64_t)seed + 2)),
           or_noise_real(cx, cy, cz, (int64_t)((uint64_t)seed + 3)));
  return dot(sub(p, V((double)cx, (double)cy, (double)cz)), g);
}
static inline double mix(double a, double b, double t) { return (b - a) * t + a; }  /* texture.rs:79-81 */

static v3 tex_sample(const or_scene* s, uint32_t tid, const hit_t* h, ctr_t* C) {
  const tex_t* t = &s->tex[tid];
  switch (t->kind) {
    case RP_TEXTURE_MISSING: return V(0.0, 0.0, 0.0);
    case RP_TEXTURE_DEBUG_UVS: return V(h->u, h->v, 0.0);
    case RP_TEXTURE_SOLID: return V(t->color[0], t->color[1], t->color[2]);
    case RP_TEXTURE_IMAGE: {  /* texture.rs:40-49 */
      double w = (double)t->w, hh = (double)t->h;
      double x = h->u * w, y = h->v * hh;
      /* f64::clamp: NaN passes through, then `as u32` saturates (NaN -> 0) */
      if (x < 0.0) x = 0.0;
      if (x > w - 1.0) x = w - 1.0;
      if (y < 0.0) y = 0.0;
      if (y > hh - 1.0) y = hh - 1.0;
      uint32_t i = sat_u32(x), j = sat_u32(y);
      const uint8_t* px = t->rgba + 4 * ((size_t)i + (size_t)j * t->w);
      OR_EVENT(C, OR_C_TEXELS);
      return V((double)px[0] / 255.0, (double)px[1] / 255.0, (double)px[2] / 255.0);
    }
    case RP_TEXTURE_CHECKER: {  /* texture.rs:51-60 */
      v3 p = h->p;
      if (fmod(floor(p.x) + floor(p.y) + floor(p.z), 2.0) == 0.0) return tex_sample(s, t->even, h, C);
      return tex_sample(s, t->odd, h, C);
    }
    case RP_TEXTURE_NOISE: {  /* texture.rs:62-68 */
      v3 p = h->p;
      double x = or_noise_real(sat_i64(floor(p.x)), sat_i64(floor(p.y)), sat_i64(floor(p.z)), t->seed);
      x = 0.5 * x + 0.5;
      return V(x, x, x);
    }
    case RP_TEXTURE_PERLIN: {  /* texture.rs:83-118 */
      v3 p = h->p;
      v3 fp = V(floor(p.x), floor(p.y), floor(p.z));
      int64_t flx = sat_i64(fp.x), fly = sat_i64(fp.y), flz = sat_i64(fp.z);
      int64_t clx = (int64_t)((uint64_t)flx + 1), cly = (int64_t)((uint64_t)fly + 1), clz = (int64_t)((uint64_t)flz + 1);
      double k1 = grad_dot(p, flx, fly, flz, t->seed), k2 = grad_dot(p, clx, fly, flz, t->seed);
      double k3 = grad_dot(p, flx, cly, flz, t->seed), k4 = grad_dot(p, clx, cly, flz, t->seed);
      double k5 = grad_dot(p, flx, fly, clz, t->seed), k6 = grad_dot(p, clx, fly, clz, t->seed);
      double k7 = grad_dot(p, flx, cly, clz, t->seed), k8 = grad_dot(p, clx, cly, clz, t->seed);
      v3 tt = sub(p, fp);
      tt.x = (tt.x * (tt.x * 6.0 - 15.0) + 10.0) * tt.x * tt.x * tt.x;
      tt.y = (tt.y * (tt.y * 6.0 - 15.0) + 10.0) * tt.y * tt.y * tt.y;
      tt.z = (tt.z * (tt.z * 6.0 - 15.0) + 10.0) * tt.z * tt.z * tt.z;
      double k12 = mix(k1, k2, tt.x), k34 = mix(k3, k4, tt.x), k56 = mix(k5, k6, tt.x), k78 = mix(k7, k8, tt.x);
      double k1234 = mix(k12, k34, tt.y), k5678 = mix(k56, k78, tt.y);
      double k = mix(k1234, k5678, tt.z);
      double x = 0.5 * k + 0.5;
      return V(x, x, x);
    }
  }
  return V(0.0, 0.0, 0.0);
}

/* ---- materials (material.rs) ---- */

/* material.rs:49-60 Emit::evaluate */
static v3 emit_eval(const or_scene* s, const rp_emit* e, const ray_t* in, const hit_t* h, ctr_t* C) {
  switch (e->kind) {
    case RP_EMIT_NONE: return V(0.0, 0.0, 0.0);
    case RP_EMIT_COLOR: return V(e->color[0], e->color[1], e->color[2]);
    case RP_EMIT_DEBUG_NORMALS: return h->n;
    case RP_EMIT_SKY_GRADIENT: {
      double t = 0.5 * (in->d.y / sqrt(norm2(in->d)) + 1.0);
      return add(smul(1.0 - t, V(1.0, 1.0, 1.0)), smul(t, V(0.5, 0.7, 1.0)));
    }
    case RP_EMIT_SKY_SPHERE: return tex_sample(s, e->texture, h, C);
  }
  return V(0.0, 0.0, 0.0);
}

/* material.rs:74-81 Absorb::evaluate */
static v3 absorb_eval(const or_scene* s, const rp_absorb* a, const hit_t* h, ctr_t* C) {
  switch (a->kind) {
    case RP_ABSORB_BLACK_BODY: return V(0.0, 0.0, 0.0);
    case RP_ABSORB_WHITE_BODY: return V(1.0, 1.0, 1.0);
    case RP_ABSORB_ALBEDO: return V(a->color[0], a->color[1], a->color[2]);
    case RP_ABSORB_ALBEDO_MAP: return tex_sample(s, a->texture, h, C);
  }
  return V(0.0, 0.0, 0.0);
}

/* material.rs:27-34 + 115-179 Scatter::evaluate; returns 1 and fills *out when a ray is scattered */
static int scatter_eval(const rp_scatter* sc, const ray_t* in, const hit_t* h, or_rng* rng, ray_t* out) {
  out->o = h->p; out->tmin = RAY_EPSILON; out->tmax = INFINITY;
  switch (sc->kind) {
    case RP_SCATTER_NONE: return 0;
    case RP_SCATTER_LAMBERT: {  /* material.rs:115-130 */
      if (dot(h->n, in->d) > 0.0) return 0;
      double us[3]; or_sample_unit_sphere(rng, us);
      out->d = normalize(add(h->n, V(us[0], us[1], us[2])));
      return 1;
    }
    case RP_SCATTER_METAL: {  /* material.rs:132-152 */
      if (dot(h->n, in->d) > 0.0) return 0;
      double ub[3]; or_sample_unit_ball(rng, ub);
      v3 rd = normalize(add(reflect(in->d, h->n), smul(sc->param, V(ub[0], ub[1], ub[2]))));
      if (dot(h->n, rd) < 0.0) return 0;
      out->d = rd;
      return 1;
    }
    case RP_SCATTER_DIELECTRIC: {  /* material.rs:154-179 */
      double eta; v3 n;
      if (dot(h->n, in->d) > 0.0) { eta = sc->param; n = neg(h->n); }
      else { eta = 1.0 / sc->param; n = h->n; }
      double r0 = (1.0 - eta) / (1.0 + eta);
      r0 = r0 * r0;                                  /* powi(2) */
      double x = 1.0 + dot(n, in->d);
      double x2 = x * x;
      double x5 = x * (x2 * x2);                     /* powi(5): LLVM binary expansion */
      double reflectance = r0 + (1.0 - r0) * x5;
      v3 dir;
      if (or_sample_bernoulli(rng, reflectance)) dir = reflect(in->d, n);
      else if (!refract(in->d, n, eta, &dir)) dir = reflect(in->d, n);
      out->d = dir;
      return 1;
    }
  }
  return 0;
}

/* ---- integrator (render.rs:94-146) ---- */

static v3 trace_continue(const or_scene* s, const ray_t* ray, uint32_t depth, or_rng* rng, ctr_t* C) {
  if (depth == 0) return V(0.0, 0.0, 0.0);
  hitm_t h = scene_hit(s, ray, C);
  if (h.valid) {
    const rp_material* m = &s->mat[h.material];
    ray_t sc;
    int scattered = scatter_eval(&m->scatter, ray, &h.h, rng, &sc);
    v3 absorb = absorb_eval(s, &m->absorb, &h.h, C);
    v3 emit = emit_eval(s, &m->emit, ray, &h.h, C);
    if (!scattered) return add(emit, V(0.0, 0.0, 0.0));
    return add(emit, mulc(absorb, trace_continue(s, &sc, depth - 1, rng, C)));
  }
  hit_t inf = hit_at_infinity(ray->d);
  return emit_eval(s, &s->background, ray, &inf, C);
}

static v3 trace_first(const or_scene* s, const ray_t* ray, uint32_t depth, or_rng* rng, ctr_t* C, int* hit_flag) {
  hitm_t h = scene_hit(s, ray, C);
  if (h.valid) {
    const rp_material* m = &s->mat[h.material];
    ray_t sc;
    int scattered = scatter_eval(&m->scatter, ray, &h.h, rng, &sc);
    v3 absorb = absorb_eval(s, &m->absorb, &h.h, C);
    v3 emit = emit_eval(s, &m->emit, ray, &h.h, C);
    *hit_flag = 1;
    if (!scattered) return add(emit, V(0.0, 0.0, 0.0));
    return add(emit, mulc(absorb, trace_continue(s, &sc, depth - 1, rng, C)));
  }
  *hit_flag = 0;
  hit_t inf = hit_at_infinity(ray->d);
  return emit_eval(s, &s->background, ray, &inf, C);
}

/* render.rs:32-52 Camera::shoot */
static ray_t shoot(const rp_camera* cam, double u, double v, or_rng* rng) {
  double tan_fov = tan(0.5 * cam->fov);
  double disk[2]; or_sample_unit_disk(rng, disk);
  v3 origin = V(cam->lens_radius * disk[0], cam->lens_radius * disk[1], 0.0);
  v3 dir = normalize(sub(V((2.0 * u - 1.0) * tan_fov * cam->focal_dist * cam->aspect_ratio,
                           (2.0 * v - 1.0) * tan_fov * cam->focal_dist, -cam->focal_dist), origin));
  ray_t r;
  r.d = matvec(cam->orientation, dir);
  r.o = add(matvec(cam->orientation, origin), V(cam->position[0], cam->position[1], cam->position[2]));
  r.tmin = RAY_EPSILON;
  r.tmax = INFINITY;
  return r;
}

/* main.rs:70-85 per-pixel body over `spp` samples with the caller's rng: the colour sum (main.rs:80)
 * and the number of samples whose first ray hit (main.rs:81); the caller divides (main.rs:86-87). */
static void render_pixel(const or_scene* s, const rp_camera* cam, uint32_t i, uint32_t j, uint32_t W, uint32_t H,
                         uint32_t spp, uint32_t max_bounce, or_rng* rng, ctr_t* C, double out[3], double* fg) {
  or_rng jit = *rng;  /* render.rs:75 make_uv_jitter clones the rng */
  v3 fc = V(0.0, 0.0, 0.0);
  double foreground = 0.0;
  for (uint32_t k = 0; k < spp; k++) {
    double ju = ((double)i + or_rng_gen_f64(&jit)) / (double)W;  /* render.rs:77-80 */
    double jv = ((double)j + or_rng_gen_f64(&jit)) / (double)H;
    ray_t r = shoot(cam, ju, jv, rng);
    int hit = 0;
    v3 c = trace_first(s, &r, max_bounce, rng, C, &hit);
    C->c[OR_C_SAMPLES]++;
    fc = add(fc, c);
    if (hit) foreground += 1.0;
  }
  out[0] = fc.x; out[1] = fc.y; out[2] = fc.z;
  *fg = foreground;
}

/* ---- per-pixel-seeded render (RNG contract) ---- */

typedef struct {
  or_scene* s;
  const rp_camera* cam;
  const rp_render_params* p;
  double* out;
  float* fg;
  uint32_t tiles_x, n_tiles, tw, th, shards, shard;
  uint32_t next_tile;
  pthread_mutex_t mu;
  ctr_t total;
} job_t;

static void* render_worker(void* arg) {
  job_t* J = (job_t*)arg;
  ctr_t C; memset(&C, 0, sizeof C);
  for (;;) {
    pthread_mutex_lock(&J->mu);
    uint32_t t = J->next_tile;
    while (t < J->n_tiles && (t % J->shards) != J->shard) t++;
    J->next_tile = t + 1;
    pthread_mutex_unlock(&J->mu);
    if (t >= J->n_tiles) break;
    uint32_t ox = (t % J->tiles_x) * J->tw, oy = (t / J->tiles_x) * J->th;
    uint32_t w = J->p->width - ox < J->tw ? J->p->width - ox : J->tw;
    uint32_t h = J->p->height - oy < J->th ? J->p->height - oy : J->th;
    for (uint32_t tj = 0; tj < h; tj++)
      for (uint32_t ti = 0; ti < w; ti++) {
        uint32_t i = ox + ti, j = oy + tj;
        /* RNG contract (include/rp.h): batch b (samples N*b .. N*b+N-1, N = samples_per_stream, 0 -> 32) of
         * pixel (i, j) has its own stream seed_from_u64(seed + b*W*H + j*W + i) and runs the unchanged
         * per-pixel body over its samples; the batch sums are added in batch order, then divided by spp
         * (main.rs:86-87).  N >= spp: one stream per pixel. */
        const uint64_t WH = (uint64_t)J->p->width * J->p->height;
        const uint64_t N = J->p->samples_per_stream ? J->p->samples_per_stream : OR_SAMPLES_PER_STREAM;
        double c[3] = {0.0, 0.0, 0.0}, fg = 0.0;
        for (uint64_t b = 0; b * N < J->p->spp; b++) {
          uint64_t n = J->p->spp - b * N;
          if (n > N) n = N;
          or_rng rng;
          or_rng_seed_from_u64(&rng, J->p->seed + b * WH + (uint64_t)j * J->p->width + i);
          double cb[3], fb;
          render_pixel(J->s, J->cam, i, j, J->p->width, J->p->height, (uint32_t)n, J->p->max_bounce, &rng, &C, cb, &fb);
          c[0] = c[0] + cb[0]; c[1] = c[1] + cb[1]; c[2] = c[2] + cb[2];
          fg += fb;
        }
        const double spp = (double)J->p->spp;
        size_t px = (size_t)j * J->p->width + i;
        J->out[3 * px] = c[0] / spp; J->out[3 * px + 1] = c[1] / spp; J->out[3 * px + 2] = c[2] / spp;
        if (J->fg) J->fg[px] = (float)(fg / spp);
      }
  }
  pthread_mutex_lock(&J->mu);
  for (int k = 0; k < OR_C_N; k++) J->total.c[k] += C.c[k];
  pthread_mutex_unlock(&J->mu);
  return NULL;
}

int or_render(or_scene* s, const rp_camera* cam, const rp_render_params* p, double* out_rgb, float* out_fg,
              uint64_t* counters, int threads) {
  if (!s || !cam || !p || !out_rgb || p->max_bounce < 1 || p->width == 0 || p->height == 0) return -1;
  job_t J;
  memset(&J, 0, sizeof J);
  J.s = s; J.cam = cam; J.p = p; J.out = out_rgb; J.fg = out_fg;
  J.tw = p->tile_w ? p->tile_w : 32; J.th = p->tile_h ? p->tile_h : 32;
  J.tiles_x = (p->width + J.tw - 1) / J.tw;
  J.n_tiles = J.tiles_x * ((p->height + J.th - 1) / J.th);
  J.shards = p->num_shards ? p->num_shards : 1;
  J.shard = p->shard;
  pthread_mutex_init(&J.mu, NULL);
  if (threads < 1) threads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
  for (int t = 0; t < threads; t++) pthread_create(&th[t], NULL, render_worker, &J);
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
  free(th);
  pthread_mutex_destroy(&J.mu);
  if (counters) for (int k = 0; k < OR_C_N; k++) counters[k] += J.total.c[k];
  return 0;
}

/* ---- the reference driver for the CPU baseline (main.rs:36-106) ---- */

typedef struct { uint32_t oi, oj, w, h; } tile_t;  /* image.rs:143-148 */

typedef struct {
  or_scene* s;
  const rp_camera* cam;
  uint32_t W, H, spp, max_bounce;
  double* out;
  tile_t* q;
  int32_t qn;
  pthread_mutex_t mu;
  ctr_t total;
  uint64_t seed;
  uint32_t next_worker;
} base_t;

static void* base_worker(void* arg) {
  base_t* B = (base_t*)arg;
  pthread_mutex_lock(&B->mu);
  uint32_t wid = B->next_worker++;
  pthread_mutex_unlock(&B->mu);
  or_rng rng;
  or_rng_seed_from_u64(&rng, B->seed + wid);  /* main.rs:52 from_entropy -> deterministic per worker */
  ctr_t C; memset(&C, 0, sizeof C);
  for (;;) {
    tile_t tile;
    pthread_mutex_lock(&B->mu);  /* main.rs:56-59 job_queue.lock().pop() (LIFO) */
    int have = B->qn > 0;
    if (have) tile = B->q[--B->qn];
    pthread_mutex_unlock(&B->mu);
    if (!have) break;
    double* cb = (double*)malloc(sizeof(double) * 3 * tile.w * tile.h);  /* main.rs:63 color_buffer */
    for (uint32_t tj = 0; tj < tile.h; tj++)
      for (uint32_t ti = 0; ti < tile.w; ti++) {
        double c[3], fg;
        render_pixel(B->s, B->cam, ti + tile.oi, tj + tile.oj, B->W, B->H, B->spp, B->max_bounce, &rng, &C, c, &fg);
        const double spp = (double)B->spp;  /* main.rs:86 */
        cb[3 * (ti + tj * tile.w)] = c[0] / spp; cb[3 * (ti + tj * tile.w) + 1] = c[1] / spp;
        cb[3 * (ti + tj * tile.w) + 2] = c[2] / spp;
      }
    if (B->out)
      for (uint32_t tj = 0; tj < tile.h; tj++)
        for (uint32_t ti = 0; ti < tile.w; ti++)
          for (int k = 0; k < 3; k++)
            B->out[3 * ((size_t)(tj + tile.oj) * B->W + ti + tile.oi) + k] = cb[3 * (ti + tj * tile.w) + k];
    free(cb);
  }
  pthread_mutex_lock(&B->mu);
  for (int k = 0; k < OR_C_N; k++) B->total.c[k] += C.c[k];
  pthread_mutex_unlock(&B->mu);
  return NULL;
}

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

double or_render_baseline(or_scene* s, const rp_camera* cam, uint32_t width, uint32_t height, uint32_t spp,
                          uint32_t max_bounce, uint32_t tile, uint32_t workers, uint64_t seed, double* out_rgb,
                          uint64_t* counters) {
  base_t B;
  memset(&B, 0, sizeof B);
  B.s = s; B.cam = cam; B.W = width; B.H = height; B.spp = spp; B.max_bounce = max_bounce; B.out = out_rgb;
  B.seed = seed;
  /* image.rs:151-167 Tile::split_in_tiles */
  uint32_t nx = (width + tile - 1) / tile, ny = (height + tile - 1) / tile;
  B.q = (tile_t*)malloc(sizeof(tile_t) * nx * ny);
  for (uint32_t tj = 0; tj < ny; tj++)
    for (uint32_t ti = 0; ti < nx; ti++) {
      tile_t* t = &B.q[B.qn++];
      t->oi = ti * tile; t->oj = tj * tile;
      t->w = tile < width - t->oi ? tile : width - t->oi;
      t->h = tile < height - t->oj ? tile : height - t->oj;
    }
  pthread_mutex_init(&B.mu, NULL);
  if (workers < 1) workers = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * workers);
  double t0 = now_s();  /* main.rs:45 */
  for (uint32_t w = 0; w < workers; w++) pthread_create(&th[w], NULL, base_worker, &B);
  for (uint32_t w = 0; w < workers; w++) pthread_join(th[w], NULL);
  double el = now_s() - t0;  /* main.rs:106 */
  free(th);
  free(B.q);
  pthread_mutex_destroy(&B.mu);
  if (counters) for (int k = 0; k < OR_C_N; k++) counters[k] += B.total.c[k];
  return el;
}

/* ================================================================ host I/O =================== */

void or_free(void* p) { free(p); }

void or_mesh_free(or_mesh_data* m) {
  if (!m) return;
  free(m->positions); free(m->normals); free(m->uvs); free(m->indices);
  memset(m, 0, sizeof *m);
}

/* nom 7 `double`: [+-] digits [. digits] [(e|E) [+-] digits] (at least one digit), or inf/nan words */
static int parse_double(const char** sp, double* out) {
  const char* s = *sp;
  const char* q = s;
  if (*q == '+' || *q == '-') q++;
  if (!strncasecmp(q, "infinity", 8) || !strncasecmp(q, "inf", 3) || !strncasecmp(q, "nan", 3)) {
    char* end;
    *out = strtod(s, &end);
    *sp = end;
    return 1;
  }
  int digits = 0;
  while (*q >= '0' && *q <= '9') { q++; digits++; }
  if (*q == '.') { q++; while (*q >= '0' && *q <= '9') { q++; digits++; } }
  if (!digits) return 0;
  if (*q == 'e' || *q == 'E') {
    const char* e = q + 1;
    if (*e == '+' || *e == '-') e++;
    if (*e >= '0' && *e <= '9') { while (*e >= '0' && *e <= '9') e++; q = e; }
  }
  char buf[128];
  size_t n = (size_t)(q - s);
  if (n >= sizeof buf) return 0;
  memcpy(buf, s, n); buf[n] = 0;
  *out = strtod(buf, NULL);
  *sp = q;
  return 1;
}

static int space1(const char** sp) {
  const char* s = *sp;
  if (*s != ' ' && *s != '\t') return 0;
  while (*s == ' ' || *s == '\t') s++;
  *sp = s;
  return 1;
}

typedef struct { uint32_t p; int64_t n, t; } objidx_t;  /* -1 = None */

/* mesh.rs:59-71 parse_index: separated_list1(tag("/"), opt(integer)) */
static int parse_index(const char** sp, objidx_t* out) {
  const char* s = *sp;
  int64_t vals[16]; int nv = 0;
  for (;;) {
    const char* d = s;
    uint64_t v = 0; int nd = 0, ovf = 0;
    while (*d >= '0' && *d <= '9') { v = v * 10 + (uint64_t)(*d - '0'); if (v > 0xffffffffull) ovf = 1; d++; nd++; }
    if (nv < 16) vals[nv++] = (nd && !ovf) ? (int64_t)v : -1;
    s = d;
    if (*s == '/') { s++; continue; }
    break;
  }
  if (vals[0] < 0) return 0;  /* "Position index not provided" */
  if (vals[0] == 0) return -1; /* 0 - 1 underflows: the reference panics */
  out->p = (uint32_t)(vals[0] - 1);
  out->t = nv > 1 && vals[1] > 0 ? vals[1] - 1 : (nv > 1 && vals[1] == 0 ? -2 : -1);
  out->n = nv > 2 && vals[2] > 0 ? vals[2] - 1 : (nv > 2 && vals[2] == 0 ? -2 : -1);
  if (out->t == -2 || out->n == -2) return -1;
  *sp = s;
  return 1;
}

typedef struct { objidx_t key; uint32_t value; int used; } hslot_t;

static uint64_t hash_idx(const objidx_t* k) {
  uint64_t h = (uint64_t)k->p * 0x9E3779B97F4A7C15ull ^ (uint64_t)(k->n + 7) * 0xC2B2AE3D27D4EB4Full ^
               (uint64_t)(k->t + 13) * 0x165667B19E3779F9ull;
  return h ^ (h >> 29);
}

/* mesh.rs:145-183 obj::load (parser mesh.rs:112-135) */
int or_obj_load(const char* path, or_mesh_data* out) {
  memset(out, 0, sizeof *out);
  FILE* f = fopen(path, "rb");
  if (!f) { snprintf(g_err, sizeof g_err, "cannot open %s", path); return -1; }
  size_t cp = 1024, cn = 1024, ct = 1024, cv = 4096, cf = 1024;
  size_t np = 0, nn = 0, nt = 0, nvx = 0, nf = 0;
  double* P = (double*)malloc(sizeof(double) * 3 * cp);
  double* N = (double*)malloc(sizeof(double) * 3 * cn);
  double* T = (double*)malloc(sizeof(double) * 2 * ct);
  objidx_t* VX = (objidx_t*)malloc(sizeof(objidx_t) * cv);
  uint32_t* FF = (uint32_t*)malloc(sizeof(uint32_t) * 2 * cf);  /* first, count */
  char* line = NULL; size_t lcap = 0; ssize_t len;
  int rc = 0;
  while ((len = getline(&line, &lcap, f)) >= 0) {
    while (len > 0 && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
    const char* s = line;
    double v[3];
    if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
      s += 1;
      if (!space1(&s) || !parse_double(&s, &v[0]) || !space1(&s) || !parse_double(&s, &v[1]) || !space1(&s) ||
          !parse_double(&s, &v[2])) continue;
      if (np == cp) { cp *= 2; P = (double*)realloc(P, sizeof(double) * 3 * cp); }
      memcpy(P + 3 * np++, v, sizeof v);
    } else if (s[0] == 'v' && s[1] == 'n') {
      s += 2;
      if (!space1(&s) || !parse_double(&s, &v[0]) || !space1(&s) || !parse_double(&s, &v[1]) || !space1(&s) ||
          !parse_double(&s, &v[2])) continue;
      if (nn == cn) { cn *= 2; N = (double*)realloc(N, sizeof(double) * 3 * cn); }
      memcpy(N + 3 * nn++, v, sizeof v);
    } else if (s[0] == 'v' && s[1] == 't') {
      s += 2;
      if (!space1(&s) || !parse_double(&s, &v[0]) || !space1(&s) || !parse_double(&s, &v[1])) continue;
      if (nt == ct) { ct *= 2; T = (double*)realloc(T, sizeof(double) * 2 * ct); }
      memcpy(T + 2 * nt++, v, sizeof(double) * 2);
    } else if (s[0] == 'f') {
      s += 1;
      if (!space1(&s)) continue;
      objidx_t idx; uint32_t cnt = 0, first = (uint32_t)nvx;
      int r = parse_index(&s, &idx);
      if (r < 0) { rc = -3; break; }
      if (r == 0) continue;
      for (;;) {
        if (nvx == cv) { cv *= 2; VX = (objidx_t*)realloc(VX, sizeof(objidx_t) * cv); }
        VX[nvx++] = idx; cnt++;
        const char* save = s;
        if (!space1(&s)) break;
        r = parse_index(&s, &idx);
        if (r < 0) { rc = -3; break; }
        if (r == 0) { s = save; break; }
      }
      if (rc) break;
      if (nf == cf) { cf *= 2; FF = (uint32_t*)realloc(FF, sizeof(uint32_t) * 2 * cf); }
      FF[2 * nf] = first; FF[2 * nf + 1] = cnt; nf++;
    }
  }
  free(line);
  fclose(f);
  if (!rc) {
    /* dedup (p, n, t) in first-use order */
    size_t hcap = 16;
    while (hcap < 2 * nvx + 16) hcap *= 2;
    hslot_t* H = (hslot_t*)calloc(hcap, sizeof(hslot_t));
    uint32_t* remap = (uint32_t*)malloc(sizeof(uint32_t) * (nvx + 1));
    uint32_t nu = 0;
    out->positions = (double*)malloc(sizeof(double) * 3 * (nvx + 1));
    out->normals = (double*)malloc(sizeof(double) * 3 * (nvx + 1));
    out->uvs = (double*)malloc(sizeof(double) * 2 * (nvx + 1));
    for (size_t k = 0; k < nvx && !rc; k++) {
      objidx_t* key = &VX[k];
      size_t hsh = hash_idx(key) & (hcap - 1);
      while (H[hsh].used && !(H[hsh].key.p == key->p && H[hsh].key.n == key->n && H[hsh].key.t == key->t))
        hsh = (hsh + 1) & (hcap - 1);
      if (!H[hsh].used) {
        if (key->p >= np || (key->n >= 0 && (size_t)key->n >= nn) || (key->t >= 0 && (size_t)key->t >= nt)) {
          rc = -4;  /* index out of bounds: the reference panics */
          break;
        }
        H[hsh].used = 1; H[hsh].key = *key; H[hsh].value = nu;
        memcpy(out->positions + 3 * nu, P + 3 * key->p, sizeof(double) * 3);
        if (key->n >= 0) memcpy(out->normals + 3 * nu, N + 3 * key->n, sizeof(double) * 3);
        else out->normals[3 * nu] = out->normals[3 * nu + 1] = out->normals[3 * nu + 2] = 0.0;
        if (key->t >= 0) memcpy(out->uvs + 2 * nu, T + 2 * key->t, sizeof(double) * 2);
        else out->uvs[2 * nu] = out->uvs[2 * nu + 1] = 0.0;
        nu++;
      }
      remap[k] = H[hsh].value;
    }
    if (!rc) {
      out->indices = (uint32_t*)malloc(sizeof(uint32_t) * (3 * nf + 1));
      for (size_t k = 0; k < nf; k++) {
        if (FF[2 * k + 1] != 3) { rc = -5; break; }  /* "Non-triangular face are not supported" */
        for (int c = 0; c < 3; c++) out->indices[3 * k + c] = remap[FF[2 * k] + c];
      }
      out->n_vertices = nu;
      out->n_indices = (uint32_t)(3 * nf);
    }
    free(H); free(remap);
  }
  free(P); free(N); free(T); free(VX); free(FF);
  if (rc) or_mesh_free(out);
  return rc;
}

/* image.rs:73-114 tga::load */
int or_tga_load(const char* path, uint32_t* w, uint32_t* h, uint8_t** rgba) {
  FILE* f = fopen(path, "rb");
  if (!f) return -1;
  uint8_t hd[18];
  if (fread(hd, 1, 18, f) != 18) { fclose(f); return -2; }
  uint32_t width = hd[12] | (hd[13] << 8), height = hd[14] | (hd[15] << 8);
  uint8_t bpp = hd[16], desc = hd[17];
  if (hd[0] != 0 || hd[1] != 0 || hd[2] != 2 || (bpp != 24 && bpp != 32)) { fclose(f); return -3; }
  uint8_t* img = (uint8_t*)malloc((size_t)width * height * 4 + 1);
  for (uint32_t y0 = 0; y0 < height; y0++) {
    uint32_t y = (desc & (1 << 5)) ? height - 1 - y0 : y0;
    for (uint32_t x = 0; x < width; x++) {
      uint8_t px[4];
      if (fread(px, 1, bpp / 8, f) != (size_t)(bpp / 8)) { free(img); fclose(f); return -4; }
      uint8_t* o = img + 4 * ((size_t)x + (size_t)y * width);
      o[0] = px[2]; o[1] = px[1]; o[2] = px[0]; o[3] = bpp == 32 ? px[3] : 0xff;
    }
  }
  fclose(f);
  *w = width; *h = height; *rgba = img;
  return 0;
}

/* image.rs:116-137 tga::save */
int or_tga_save(const char* path, uint32_t w, uint32_t h, const uint8_t* rgba) {
  if (w > 65535 || h > 65535) return -2;
  FILE* f = fopen(path, "wb");
  if (!f) return -1;
  uint8_t hd[18] = {0};
  hd[2] = 2; hd[16] = 32;
  hd[12] = (uint8_t)w; hd[13] = (uint8_t)(w >> 8); hd[14] = (uint8_t)h; hd[15] = (uint8_t)(h >> 8);
  fwrite(hd, 1, 18, f);
  for (uint32_t y = 0; y < h; y++)
    for (uint32_t x = 0; x < w; x++) {
      const uint8_t* p = rgba + 4 * ((size_t)x + (size_t)y * w);
      uint8_t o[4] = {p[2], p[1], p[0], p[3]};
      fwrite(o, 1, 4, f);
    }
  fclose(f);
  return 0;
}

/* utility.rs:212-220 to_srgb_u8 */
void or_to_srgb_u8(const double* rgb, uint64_t n, uint8_t* rgba) {
  for (uint64_t i = 0; i < n; i++) {
    for (int c = 0; c < 3; c++) {
      double x = rgb[3 * i + c];
      if (x < 0.0) x = 0.0;
      if (x > 1.0) x = 1.0;
      rgba[4 * i + c] = sat_u8(255.0 * pow(x, 1.0 / 2.2));
    }
    rgba[4 * i + 3] = 0xff;
  }
}
