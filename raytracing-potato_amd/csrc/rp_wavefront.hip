// rp_wavefront.hip -- the stage-split ("wavefront") engine: the same paths as the megakernel
// (rp_kernel.hip), with traversal and shading in separate kernels over a pool of path slots.
//
// The megakernel runs traversal and shading on the same lanes: a wave traverses until few of its lanes
// still traverse, then shades the finished ones -- every material, texture and sample-start branch with
// the lanes that happen to need it (~30 % of the wave), and the lanes that finished early idle in the
// traversal loop meanwhile.  Here a slot pool of P paths (P >> resident lanes) lives in HBM / the
// Infinity Cache, structure-of-arrays, and each iteration is two launches:
//   trace: persistent; a lane whose ray is done fetches the next slot of the ray queue (compacted by the
//          shade pass), so traversal lanes stay busy without waiting for shading;
//   shade: one lane per queued slot: the hit or miss is shaded (rp_device.h shade_ray, the megakernel's
//          code), the path continues, or its sample ends and the slot starts the unit's next sample (or
//          fetches the next unit); rays to trace next are appended to the other queue (wave-aggregated).
// The RNG stream is the contract's (one StdRng per (pixel, sample batch)): the shade lane derives the key
// from the unit seed and generates the keystream blocks it reads into a two-block window in LDS, so
// nothing but the stream position is stored per slot.  Results are those of the megakernel bit for bit
// (same arithmetic, same per-unit accumulation order).  References as rp_device.h.
#include "rp_device.h"

#pragma clang fp contract(off)

namespace rpk {

// ---- keystream window of a shading lane: blocks end-2, end-1 of its stream in LDS ([word][lane]) -------
struct WRng {
  lds_u32* ring;    // this lane's column: ring word i at ring[i * BLOCK] (32 words: 2 blocks)
  uint32_t key[8];  // StdRng::seed_from_u64(unit seed) (rp_device.h seed_key)
  uint32_t pos;     // next keystream word (even)
  uint32_t end;     // one past the newest block held
};

// Out of line: every draw site would otherwise inline a 2.5 KB ChaCha12 (instruction-cache pressure).
static __device__ __attribute__((noinline)) void wr_block(const uint32_t* key, uint32_t b, lds_u32* ring) {
  uint32_t k[8], w[16];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = key[i];
  chacha12(k, b, w);
  lds_u32* dst = ring + (b & 1u) * 16u * BLOCK;
#pragma unroll
  for (int i = 0; i < 16; i++) dst[i * BLOCK] = w[i];
}
RPK_INLINE void wr_gen(WRng& r, uint32_t b) { wr_block(r.key, b, r.ring); }
// every block up to last_blk is made (the draw sites ensure the blocks of the words they read; a try
// spans at most two consecutive blocks, the window)
RPK_INLINE void ring_ensure(WRng& r, uint32_t last_blk) {
  if (r.end + 1u < last_blk) r.end = last_blk - 1u;  // skipped blocks are never read (the window slides)
  while (last_blk >= r.end) {
    wr_gen(r, r.end);
    r.end++;
  }
}
RPK_INLINE uint2 ring_u64(const WRng& r, uint32_t a) {
  const lds_u32* p = r.ring + (a & 31u) * BLOCK;
  return make_uint2(p[0], p[BLOCK]);
}
RPK_INLINE double ring_f64(const WRng& r, uint32_t a) {
  const uint2 v = ring_u64(r, a);
  return words_f64(v.x, v.y);
}
RPK_INLINE double ring_sym(const WRng& r, uint32_t a) {
  const uint2 v = ring_u64(r, a);
  return words_sym(v.x, v.y);
}
RPK_INLINE double gen_f64(WRng& r) {
  ring_ensure(r, r.pos >> 4);
  const double x = ring_f64(r, r.pos);
  r.pos += 2;
  return x;
}
// make_uv_jitter's words 4s..4s+3 of the stream (block s/4, render.rs:74-82): generated in registers
RPK_INLINE uint4 rng_jitter(WRng& r, uint32_t s) {
  uint32_t w[16];
  chacha12(r.key, s >> 2, w);
  const uint32_t q = s & 3u;
  uint4 v = make_uint4(w[0], w[1], w[2], w[3]);
  if (q == 1u) v = make_uint4(w[4], w[5], w[6], w[7]);
  if (q == 2u) v = make_uint4(w[8], w[9], w[10], w[11]);
  if (q == 3u) v = make_uint4(w[12], w[13], w[14], w[15]);
  return v;
}

// ---- path state ---------------------------------------------------------------------------------------
// The paths in flight are kept in QUEUE ORDER: a shade pass reads entry i of the input state and appends
// the paths that go on to the output state at consecutive positions (wave-aggregated atomic), so every
// state access of both passes is coalesced; the trace pass reads the ray of entry q and writes its hit at
// q.  Two state buffers alternate.  st words (SoA, P entries each): ST_S sample index in the unit |
// FIRST_BIT, ST_DEPTH bounces left, ST_POS keystream word (POS_NEW: the entry holds no unit yet), ST_PIPJ
// pixel i | j << 16, ST_BATCH, ST_SLOT the unit's output slot, ST_HITS samples whose first ray hit.
enum { ST_S = 0, ST_DEPTH, ST_POS, ST_PIPJ, ST_BATCH, ST_SLOT, ST_HITS, ST_N };
static constexpr uint32_t FIRST_BIT = 0x80000000u, POS_NEW = 0xFFFFFFFFu;
enum { WC_N0 = 0, WC_N1 = 1, WC_FETCH = 2, WC_N = 4 };

struct WfState {
  double* ray;  // 6 x P: o.x o.y o.z d.x d.y d.z
  double* tp;   // 3 x P: path throughput
  double* sum;  // 3 x P: the unit's sample sum
  uint32_t* st; // ST_N x P
};
struct WfArgs {
  WfState in, out;  // the pass reads `in`, a shade pass appends to `out`
  double* hit;      // 3 x P: t, u, v of the closest hit of input entry q
  int32_t* prim;    // P: its primitive (-1 = miss)
  uint32_t* wc;     // WC_N counters: the two state buffers' lengths, the trace pass's fetch index
  uint32_t P;
  uint32_t nin;     // WC_N0 / WC_N1: the counter of `in` (the other one counts `out`)
};

__global__ void __launch_bounds__(256) wf_init_kernel(const WfArgs w) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < w.P) w.in.st[ST_POS * (uint64_t)w.P + i] = POS_NEW;
  if (i == 0) {
    w.wc[w.nin] = w.P;
    w.wc[w.nin ^ 1u] = 0;
    w.wc[WC_FETCH] = 0;
  }
}

// ---- shade pass ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(BLOCK) wf_shade_kernel(const KArgs args, const WfArgs w) {
  __shared__ uint32_t ring[32 * BLOCK];
  const uint32_t tid = threadIdx.x;
  const uint32_t i = blockIdx.x * BLOCK + tid;
  if (blockIdx.x == 0 && tid == 0) w.wc[WC_FETCH] = 0;  // the next trace pass fetches from its start
  const uint32_t n = w.wc[w.nin];
  const bool live = i < n;
  const uint64_t P = w.P;
  uint32_t s = 0, depth = 0, pos = POS_NEW, pipj = 0, batch = 0, oslot = 0, hits = 0;
  if (live) {
    s = w.in.st[ST_S * P + i];
    depth = w.in.st[ST_DEPTH * P + i];
    pos = w.in.st[ST_POS * P + i];
    pipj = w.in.st[ST_PIPJ * P + i];
    batch = w.in.st[ST_BATCH * P + i];
    oslot = w.in.st[ST_SLOT * P + i];
    hits = w.in.st[ST_HITS * P + i];
  }
  KArgsPtr A = kargs();
  WRng rng;
  rng.ring = (lds_u32*)(ring + tid);
  bool traced = live && pos != POS_NEW, start = false, fetch = live && pos == POS_NEW;
  bool ended_sample = false, ended_pixel = false, append = false;
  double sx = 0.0, sy = 0.0, sz = 0.0, tx = 1.0, ty = 1.0, tz = 1.0;
  V3 o = v3(0.0, 0.0, 0.0), d = v3(0.0, 0.0, 1.0);
  if (traced) {
    seed_key(unit_seed(A, pipj & 0xFFFFu, pipj >> 16, batch), rng.key);
    rng.pos = pos;
    rng.end = pos >> 4;
    o = v3(w.in.ray[i], w.in.ray[P + i], w.in.ray[2 * P + i]);
    d = v3(w.in.ray[3 * P + i], w.in.ray[4 * P + i], w.in.ray[5 * P + i]);
    tx = w.in.tp[i];
    ty = w.in.tp[P + i];
    tz = w.in.tp[2 * P + i];
    sx = w.in.sum[i];
    sy = w.in.sum[P + i];
    sz = w.in.sum[2 * P + i];
    HitRec hr;
    hr.t = w.hit[i];
    hr.u = w.hit[P + i];
    hr.v = w.hit[2 * P + i];
    hr.prim = w.prim[i];
    const bool first = (s & FIRST_BIT) != 0u;
    s &= ~FIRST_BIT;
    const KScene S = load_scene(A);
    const bool scattered = shade_ray(S, hr, o, d, rng, tx, ty, tz, sx, sy, sz, first, hits);
    bool end_sample = true;
    if (scattered) {
      depth--;
      end_sample = depth == 0;  // trace_path_continue(depth 0) is black (render.rs:128-131)
    }
    append = !end_sample;
    if (end_sample) {
      s++;
      ended_sample = true;
      A = kargs();
      if (s == unit_spp(A, batch)) {  // main.rs:86-87 (for this unit's batch of samples)
        if (A->P.nbatch == 1) {
          const double spp = (double)A->P.spp;
          double* outp = A->out;
          outp[3 * (uint64_t)oslot + 0] = sx / spp;
          outp[3 * (uint64_t)oslot + 1] = sy / spp;
          outp[3 * (uint64_t)oslot + 2] = sz / spp;
          if (A->out_fg) A->out_fg[oslot] = (float)((double)hits / spp);
        } else {  // one batch of several: its sum, reduced in batch order by reduce_batches
          const uint64_t u = (uint64_t)oslot * A->P.nbatch + batch;
          double* part = A->P.partial;
          part[3 * u + 0] = sx;
          part[3 * u + 1] = sy;
          part[3 * u + 2] = sz;
          A->P.partial_hits[u] = hits;
        }
        ended_pixel = batch == 0;
        fetch = true;
      } else {
        start = true;
      }
    }
  }
  if (fetch) {  // the path's next unit (pixel, sample batch) from the frame's queue; none left: it ends
    uint32_t pi = 0, pj = 0;
    if (fetch_pixel<false>(oslot, pi, pj, batch)) {
      pipj = pi | (pj << 16);
      s = 0;
      hits = 0;
      sx = sy = sz = 0.0;
      A = kargs();
      seed_key(unit_seed(A, pi, pj, batch), rng.key);
      rng.pos = 0;
      rng.end = 0;
      start = true;
    }
  }
  if (start) {  // camera sample s of the unit (main.rs:75-76): jitter + Camera::shoot
    start_sample(rng, s, pipj & 0xFFFFu, pipj >> 16, o, d);
    depth = kargs()->P.max_bounce;
    tx = ty = tz = 1.0;
    s |= FIRST_BIT;
    append = true;
  }
  if (append) {
    const uint32_t k = atomicAdd(&w.wc[w.nin ^ 1u], 1u);
    w.out.ray[k] = o.x;
    w.out.ray[P + k] = o.y;
    w.out.ray[2 * P + k] = o.z;
    w.out.ray[3 * P + k] = d.x;
    w.out.ray[4 * P + k] = d.y;
    w.out.ray[5 * P + k] = d.z;
    w.out.tp[k] = tx;
    w.out.tp[P + k] = ty;
    w.out.tp[2 * P + k] = tz;
    w.out.sum[k] = sx;
    w.out.sum[P + k] = sy;
    w.out.sum[2 * P + k] = sz;
    w.out.st[ST_S * P + k] = s;
    w.out.st[ST_DEPTH * P + k] = depth;
    w.out.st[ST_POS * P + k] = rng.pos;
    w.out.st[ST_PIPJ * P + k] = pipj;
    w.out.st[ST_BATCH * P + k] = batch;
    w.out.st[ST_SLOT * P + k] = oslot;
    w.out.st[ST_HITS * P + k] = hits;
  }
  // per-wave counts (ballot popcounts) into the frame's counters
  const uint64_t n_rays = (uint64_t)__popcll(__ballot(traced));
  const uint64_t n_samples = (uint64_t)__popcll(__ballot(ended_sample));
  const uint64_t n_pixels = (uint64_t)__popcll(__ballot(ended_pixel));
  if ((tid & 63u) == 0u && (n_rays | n_samples | n_pixels)) {
    unsigned long long* ctr = kargs()->ctr;
    atomicAdd(&ctr[CTR_RAYS], (unsigned long long)n_rays);
    atomicAdd(&ctr[CTR_SAMPLES], (unsigned long long)n_samples);
    atomicAdd(&ctr[CTR_PIXELS], (unsigned long long)n_pixels);
  }
}

// ---- trace pass ---------------------------------------------------------------------------------------
// Persistent: every lane takes the next queued ray as soon as its ray is done.  A wave refills its idle
// lanes when at least WF_REFILL of them wait (the ray setup runs with many lanes) or when none
// traverse; the refilling lanes get consecutive entries (wave-aggregated atomic), so the ray loads coalesce.
static constexpr uint32_t WF_REFILL = 16;
template <bool SPILL, uint32_t NF>
__global__ void __launch_bounds__(BLOCK) wf_trace_kernel(const KArgs args, const WfArgs w) {
  extern __shared__ uint32_t lds_stack[];
  lds_u32* stk = (lds_u32*)(lds_stack + threadIdx.x);
  const uint32_t tid = threadIdx.x;
  if (blockIdx.x == 0 && tid == 0) w.wc[w.nin ^ 1u] = 0;  // the next shade pass appends from 0
  const uint32_t n = w.wc[w.nin];
  const uint64_t P = w.P;
  bool have = false, drained = false, overflow = false;
  uint32_t q = 0;
  V3 o = v3(0.0, 0.0, 0.0), d = v3(0.0, 0.0, 1.0);
  Ray32 r;
  TravState ts;
  ts.cur = rpl::ENTRY_EMPTY;
  ts.leaf = 0u;
  ts.sp = 0u;
  ts.best = 0.0;
  ts.bestp = -1;
  ts.bestm = KM_UNKNOWN;
  ts.bu = ts.bv = 0.0;
  ts.gy = ts.py = 0u;
  for (;;) {
    const uint64_t idle = __ballot(!have);
    if (!drained && idle != 0 && ((uint32_t)__popcll(idle) >= WF_REFILL || __ballot(have) == 0)) {
      if (!have) {
        q = atomicAdd(&w.wc[WC_FETCH], 1u);
        if (q < n) {
          o = v3(w.in.ray[q], w.in.ray[P + q], w.in.ray[2 * P + q]);
          d = v3(w.in.ray[3 * P + q], w.in.ray[4 * P + q], w.in.ray[5 * P + q]);
          const KScene S = load_scene(kargs());
          setup_ray32<NF>(o, d, RAY_EPSILON, S.qbound, r);
          trav_init<NF>(S, INF, ts, d);
          double best = ts.best;
          for (uint32_t k = S.always_first; k < S.always_first + S.n_always; k++)
            prim_test(S, k, o, d, RAY_EPSILON, best, ts);
          ts.best = best;
          have = true;
        }
      }
      // a lane that fetched and got nothing: the queue is exhausted for every later fetch as well
      if (__ballot(!have) != 0) drained = true;
    }
    if (__ballot(have) == 0) break;  // drained and every ray of this wave done
    if (have) {
      const KScene S = load_scene(kargs());
      const uint32_t spl = SPILL ? (blockIdx.x * BLOCK + tid) * (S.stack_depth - S.lds_depth) : 0u;
      trav_step<SPILL, NF>(S, stk, BLOCK, spl, r, o, d, RAY_EPSILON, ts, overflow);
      if (trav_done(ts)) {
        w.hit[q] = ts.best;
        w.hit[P + q] = ts.bu;
        w.hit[2 * P + q] = ts.bv;
        w.prim[q] = ts.bestp;
        have = false;
      }
    }
  }
  if (overflow) atomicOr(&kargs()->ctr[CTR_STATUS], (unsigned long long)STATUS_STACK_OVERFLOW);
}

// ---- host side ----------------------------------------------------------------------------------------
int launch_wavefront(const KScene& s, const KParams& p, double* out_rgb, float* out_fg, uint64_t* counters,
                     uint32_t* queue, const WfBuffers& b, int trace_grid, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  KArgs a;
  a.S = s;
  a.P = p;
  a.out = out_rgb;
  a.out_fg = out_fg;
  a.ctr = reinterpret_cast<unsigned long long*>(counters);
  a.queue = queue;
  a.diag = reinterpret_cast<unsigned long long*>(s.diag);
  WfState sb[2];
  for (int k = 0; k < 2; k++) {
    sb[k].ray = b.ray + (uint64_t)k * 6 * b.P;
    sb[k].tp = b.tp + (uint64_t)k * 3 * b.P;
    sb[k].sum = b.sum + (uint64_t)k * 3 * b.P;
    sb[k].st = b.st + (uint64_t)k * ST_N * b.P;
  }
  WfArgs w;
  w.hit = b.hit;
  w.prim = b.prim;
  w.wc = b.wc;
  w.P = b.P;
  uint32_t cur = 0;  // the state buffer holding the paths to shade / trace next
  auto set = [&](uint32_t c) {
    w.in = sb[c];
    w.out = sb[c ^ 1u];
    w.nin = c;
  };
  set(cur);
  const unsigned sgrid = (unsigned)((b.P + BLOCK - 1) / BLOCK);
  hipLaunchKernelGGL(wf_init_kernel, dim3(sgrid), dim3(256), 0, st, w);
  hipLaunchKernelGGL(wf_shade_kernel, dim3(sgrid), dim3(BLOCK), 0, st, a, w);  // paths fetch their first units
  cur ^= 1u;
  const size_t lds = (size_t)s.lds_depth * BLOCK * sizeof(uint32_t);
  const bool spill = s.lds_depth < s.stack_depth;
  uint32_t* h_n = b.host_count;
  // every iteration advances each queued path by one ray, and a path's units run back to back: a frame
  // needs at most (units per path + 2) x samples per unit x (max_bounce + 1) iterations (a safety bound)
  const uint64_t bound = (p.n_queue / b.P + 2) * (uint64_t)p.spp_batch * (p.max_bounce + 1) + 64;
  for (uint32_t it = 1;; it++) {
    if (it > bound) return (int)hipErrorUnknown;
    set(cur);
    if (s.node_format == rpl::NODES_W8) {
      if (spill) hipLaunchKernelGGL((wf_trace_kernel<true, rpl::NODES_W8>), dim3(trace_grid), dim3(BLOCK), lds, st, a, w);
      else hipLaunchKernelGGL((wf_trace_kernel<false, rpl::NODES_W8>), dim3(trace_grid), dim3(BLOCK), lds, st, a, w);
    } else if (s.node_format == rpl::NODES_Q8) {
      if (spill) hipLaunchKernelGGL((wf_trace_kernel<true, rpl::NODES_Q8>), dim3(trace_grid), dim3(BLOCK), lds, st, a, w);
      else hipLaunchKernelGGL((wf_trace_kernel<false, rpl::NODES_Q8>), dim3(trace_grid), dim3(BLOCK), lds, st, a, w);
    } else {
      if (spill) hipLaunchKernelGGL((wf_trace_kernel<true, rpl::NODES_F32>), dim3(trace_grid), dim3(BLOCK), lds, st, a, w);
      else hipLaunchKernelGGL((wf_trace_kernel<false, rpl::NODES_F32>), dim3(trace_grid), dim3(BLOCK), lds, st, a, w);
    }
    hipLaunchKernelGGL(wf_shade_kernel, dim3(sgrid), dim3(BLOCK), 0, st, a, w);
    cur ^= 1u;
    if (it % b.poll == 0) {  // host poll: stop once no ray is queued
      hipError_t e = hipMemcpyAsync(h_n, b.wc + cur, sizeof(uint32_t), hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e != hipSuccess) return (int)e;
      if (*h_n == 0) break;
    }
  }
  return (int)hipGetLastError();
}

int wavefront_trace_blocks_per_cu(uint32_t lds_depth, bool spill, uint32_t nf, int* blocks) {
  const size_t lds = (size_t)lds_depth * BLOCK * sizeof(uint32_t);
  if (nf == rpl::NODES_W8) {
    if (spill) return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wf_trace_kernel<true, rpl::NODES_W8>, BLOCK, lds);
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wf_trace_kernel<false, rpl::NODES_W8>, BLOCK, lds);
  }
  if (nf == rpl::NODES_Q8) {
    if (spill) return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wf_trace_kernel<true, rpl::NODES_Q8>, BLOCK, lds);
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wf_trace_kernel<false, rpl::NODES_Q8>, BLOCK, lds);
  }
  if (spill) return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wf_trace_kernel<true, rpl::NODES_F32>, BLOCK, lds);
  return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, wf_trace_kernel<false, rpl::NODES_F32>, BLOCK, lds);
}

}  // namespace rpk
