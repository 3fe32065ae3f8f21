// rp_kernel.hip -- gfx950 path-tracing megakernel (the hot path of alucas2/raytracing-potato).
//
// One lane = one pixel's path state.  Each lane loops
//     [fetch pixel] -> [new sample: jitter + Camera::shoot] -> traverse -> shade -> ...
// as a single flat loop (path regeneration), so every live lane of a wave executes the SAME traversal
// code each iteration whatever bounce or sample it is on; lanes that finish a pixel refetch from the
// atomic unit queue of their XCD group (persistent threads; the compiler folds the per-lane atomicAdd into
// one wave atomic via ballot + mbcnt).  Traversal stacks live in LDS, lane-major ([depth][lane]) so a
// wave's push/pop is bank-conflict-free whatever depth each lane is at.
//
// Arithmetic is IEEE binary64 in the reference's exact operation order (no contraction: this file is
// compiled with -ffp-contract=off and the pragma below), so paths -- and the RNG draws they consume --
// are the reference's.  References: render.rs:32-146, bvh.rs:93-124, hittable.rs:39-108,
// material.rs:27-179, texture.rs:21-118, randomness.rs:9-110, utility.rs:67-154.
#include "rp_device.h"

#pragma clang fp contract(off)

namespace rpk {

// 4 waves per SIMD (128 VGPRs): measured 3.7 % faster on C3 than 3 waves/SIMD with the whole traversal stack in
// LDS; 5 waves (96 VGPRs) spills and loses 4-13 %.
#define RPK_RENDER_ATTR __attribute__((amdgpu_waves_per_eu(4)))
// Wave issue priority by phase (s_setprio): traversal 2 > shading 1 > keystream refill 0 -- a traversing
// wave's next node fetch goes out sooner while VALU-heavy work fills the gaps (C3 234.7 -> 230.1 ms, C5
// 2,039 -> 2,015 ms; traversal-only priority 231.5, priority to shading 237.6, refill at 1: +1.7 %)
static constexpr int PRIO_TRAV = 2, PRIO_SHADE = 1, PRIO_REFILL = 0;
// Keystream blocks a lane keeps ahead (rp_device.h RngT): 8, or 4 in the quantized-node kernel that large
// scenes use -- C5 -1.7 % (its smaller slab footprint leaves L2 and the Infinity Cache to the 1.1 GB scene;
// 2 blocks: -0.9 %), while C3 wants 8 (4: +0.6 %, 2: +16 %), ab38.  A run-time ring size cost C3 +0.3 % (ab39).
template <uint32_t NF>
constexpr uint32_t RingFor = NF == rpl::NODES_Q8 ? 4u : RING;

// Tile costs are measured on one unit in eight (pixel and batch hashed: every tile's sample spreads over its pixels
// and batches) -- timing all units cost 0.9 %
RPK_INLINE bool meas_unit(uint32_t pipj, uint32_t batch) { return ((pipj ^ (pipj >> 16) ^ batch ^ (pipj >> 3)) & 7u) == 0u; }

// PROBE = the cost-probe launch (rp_kernel.h, cost-ordered tile scheduling): a separate symbol so profiles
// and timings of the frame kernel never mix with it.
template <bool PROBE, bool SPILL, uint32_t NF>
__global__ void __launch_bounds__(BLOCK) RPK_RENDER_ATTR render_kernel(const KArgs args) {
  extern __shared__ uint32_t lds_stack[];
  __shared__ unsigned long long blk_ctr[3];
  DIAG(__shared__ unsigned long long wmax[BLOCK / 64][8];
       if (threadIdx.x < BLOCK / 64 * 8) wmax[threadIdx.x / 8][threadIdx.x % 8] = 0;)
  if (threadIdx.x < 3) blk_ctr[threadIdx.x] = 0;
  DIAG(if (threadIdx.x < 2 * DREG_N) g_dreg[threadIdx.x] = 0;)
  DIAG(if (threadIdx.x < DCYC_N) g_dcyc[threadIdx.x] = 0;)
  // frame timeline (100 MHz real-time clock, comparable across XCDs): first block start, first failed
  // pixel fetch (queue drained), last wave exit -- minima stored bit-inverted so atomicMax serves both
  DIAG(if (!PROBE && threadIdx.x == 0) atomicMax(&kargs()->diag[10], ~(unsigned long long)__builtin_amdgcn_s_memrealtime());)
  __syncthreads();
  lds_u32* stk = (lds_u32*)(lds_stack + threadIdx.x);

  // per-WAVE totals (ballot popcounts: scalar registers, not three VGPRs through the shading code)
  uint64_t n_rays = 0, n_samples = 0, n_pixels = 0;
  DIAG(uint32_t lane_rays = 0;)
  bool overflow = false;
  DIAG(uint64_t ph[5] = {0, 0, 0, 0, 0}; uint64_t iters = 0, active = 0; TravDiag td; uint64_t t_prev = stamp();)
  DIAG(const uint64_t t_blk = __builtin_amdgcn_s_memrealtime(); uint64_t t_pix = t_blk, t_retire = t_blk; uint32_t rays_pix = 0;
       auto tbin = [&](uint64_t t) { return (uint32_t)min<uint64_t>((t - t_blk) / DIAG_BIN_TICKS, DIAG_HIST - 1); };)

  // ---- lane state: one pixel's path at a time.  Hot state (ray, throughput, radiance, traversal)
  // in registers; cold per-pixel state (pixel sum, slot/pixel/sample counters, keystream cursors) in
  // LDS, structure-of-arrays so every access is bank-conflict-free; keystream blocks in the slab.
  __shared__ double c_sum[3 * BLOCK];
  __shared__ double c_T[3 * BLOCK];
  // (8 words per lane: one more would push the block past 40 KB of LDS and cost a block per CU)
  __shared__ uint32_t c_u[8 * BLOCK];
  const uint32_t tid = threadIdx.x;
  uint32_t& slot = c_u[tid];
  uint32_t& pipj = c_u[BLOCK + tid];  // pixel i | j << 16 (make_tiling caps width and height at 65535)
  uint32_t& s = c_u[3 * BLOCK + tid];
  uint32_t& hits = c_u[4 * BLOCK + tid];
  uint32_t& batch = c_u[2 * BLOCK + tid];
  double& sum_x = c_sum[tid];
  double& sum_y = c_sum[BLOCK + tid];
  double& sum_z = c_sum[2 * BLOCK + tid];
  double& T_x = c_T[tid];  // path throughput (read and written once per shade)
  double& T_y = c_T[BLOCK + tid];
  double& T_z = c_T[2 * BLOCK + tid];
  uint32_t depth = 0;
  uint32_t work = 0;  // PROBE: the probed sample's traversal work (rp_device.h WORK_*)
  bool first = true;
  RngT<RingFor<NF>> rng;
  rng.slab = reinterpret_cast<uint4*>(kargs()->S.rng_slab) + ((uint64_t)blockIdx.x * BLOCK + tid) * RngT<RingFor<NF>>::lane_n;
  rng.end = c_u + 5 * BLOCK + tid;
  rng.jtag = c_u + 6 * BLOCK + tid;
  rng.pos = 0;
  V3 o = v3(0, 0, 0), d = v3(0, 0, 1);
  T_x = T_y = T_z = 1.0;
  s = 0;
  hits = 0;
  sum_x = sum_y = sum_z = 0.0;
  TravState ts;
  ts.cur = rpl::ENTRY_EMPTY;  // no ray: done
  ts.leaf = 0u;
  ts.sp = 0u;
  ts.best = 0.0;
  ts.bestp = -1;
  ts.bestm = KM_UNKNOWN;
  ts.bu = ts.bv = 0.0;
  ts.gy = ts.py = 0u;
  uint32_t pi = 0, pj = 0;
  bool alive = fetch_pixel<PROBE>(slot, pi, pj, batch);
  pipj = pi | (pj << 16);
  bool tdone = true;  // traversal of the current ray finished (or no ray)
  bool newray = false;  // a ray started since the last traversal round (always-tested prims pending)
  // Camera samples start at the top of the next round, after the refill pass: `start` = sample s is due,
  // `fresh` = and it is the first of a unit whose key and block 0 the refill pass makes.
  bool start = alive, fresh = alive;
  DIAG({ uint64_t t = stamp(); ph[0] += t - t_prev; t_prev = t; })

  // Every lane of the wave stays in this loop until the whole wave has retired, so the ballots below
  // see all 64 lanes.  Each round: step the traversal of the lanes that are still traversing until
  // fewer than trav_threshold of them remain (and some finished lane is waiting), then shade the
  // finished lanes and give them their next ray; unfinished lanes resume where they stopped (their
  // node, LDS stack and closest hit so far are kept).
  for (;;) {
    DIAG(iters++;)
    DREG(DREG_ROUND)
    __builtin_amdgcn_s_setprio(PRIO_REFILL);
    {
      KArgsPtr A = kargs();
      const uint64_t seed = unit_seed(A, pipj & 0xFFFFu, pipj >> 16, batch);  // RNG contract
      DCYC_BEGIN(cr)
      rng_refill(rng, alive, fresh, seed, start ? s - 1 : s, unit_spp(A, batch));
      DCYC_END(DCYC_REFILL, cr)
      // a measured unit's start (100 MHz real-time clock, the same on every XCD): its duration is its tile's cost
      if (!PROBE && fresh && ((A->P.tile_meas && meas_unit(pipj, batch)) || A->P.unit_cost))
        A->S.unit_t0[blockIdx.x * BLOCK + tid] = (uint32_t)__builtin_amdgcn_s_memrealtime();
    }
    if (start) {
      KArgsPtr A = kargs();
      DCYC_BEGIN(cs)
      start_sample(rng, s, pipj & 0xFFFFu, pipj >> 16, o, d);
      DCYC_END(DCYC_START_SAMPLE, cs)
      depth = A->P.max_bounce;
      T_x = T_y = T_z = 1.0;
      first = true;
      trav_init<NF>(load_scene(A), INF, ts, d);
      tdone = false;
      newray = true;
      start = fresh = false;
    }
    DIAG({ uint64_t t = stamp(); ph[1] += t - t_prev; t_prev = t; })
    {
      KArgsPtr A = kargs();
      const KScene S = load_scene(A);
      const uint32_t thr = A->P.trav_threshold;
      // the lane's spill run (SPILL kernels): lane index x spill entries per lane
      const uint32_t spl = SPILL ? (blockIdx.x * BLOCK + tid) * (S.stack_depth - S.lds_depth) : 0u;
      // camera rays and scattered rays started since the last round: the always-tested primitives (trav_begin),
      // at one site for both
      if (newray) {
        DCYC_BEGIN(cn)
        double best = ts.best;
        for (uint32_t k = S.always_first; k < S.always_first + S.n_always; k++)
          prim_test(S, k, o, d, RAY_EPSILON, best, ts);
        ts.best = best;
        newray = false;
        DCYC_END(DCYC_NEWRAY, cn)
      }
      Ray32 r;
      setup_ray32<NF>(o, d, RAY_EPSILON, S.qbound, r);
      __builtin_amdgcn_s_setprio(PRIO_TRAV);  // (PRIO_* above)
      for (;;) {
        if (alive && !tdone) {
          DREG(DREG_STEP)
#ifdef RPK_DIAG
          trav_step<SPILL, NF, PROBE>(S, stk, BLOCK, spl, r, o, d, RAY_EPSILON, ts, overflow, &td, &work);
#else
          trav_step<SPILL, NF, PROBE>(S, stk, BLOCK, spl, r, o, d, RAY_EPSILON, ts, overflow, nullptr, &work);
#endif
          tdone = trav_done(ts);
        }
        // the threshold scales with the wave's live lanes: a wave whose units are retiring (the frame's tail, or the long
        // units of one stream per pixel) keeps stepping its traversals instead of pausing them for every shading round
        // (C3 one stream per pixel -2.2 %, C3 and C5 unchanged: profiles/r5/c3_c5_sparse_wave_ab.json)
        const uint64_t act = __ballot(alive && !tdone);
        const uint64_t waiting = __ballot(alive && tdone);
        if (act == 0 || (waiting != 0 && 64u * (uint32_t)__popcll(act) < thr * (uint32_t)__popcll(__ballot(alive)))) break;
      }
    }
    __builtin_amdgcn_s_setprio(PRIO_SHADE);
    DIAG({ uint64_t t = stamp(); ph[2] += t - t_prev; t_prev = t; })
    if (__ballot(alive) == 0) break;

    n_rays += (uint64_t)__popcll(__ballot(alive && tdone));
    bool ended_sample = false, ended_pixel = false;
    uint32_t meas_k = 0xFFFFFFFFu, meas_dur = 0u;  // a unit ended: its shard tile and duration
    if (alive && tdone) {
      DIAG(active++;)
      DREG(DREG_SHADE)
      DIAG(lane_rays++;)
      HitRec hr;
      hr.t = ts.best;
      hr.u = ts.bu;
      hr.v = ts.bv;
      hr.prim = ts.bestp;
      // the f32-node (cache-resident scene) kernel carries the hit's kind and material out of the traversal
      // (C3 -0.5 %); the q8 kernel of large scenes re-reads them (carrying them cost C5 +0.9 %: its traversal,
      // 2/3 of the wave-cycles, pays the register)
      hr.km = NF == rpl::NODES_Q8 ? KM_UNKNOWN : ts.bestm;

      // ---- shade.  Hits and misses share one spherical-uv site and one texture-sampling site, so a wave
      // with both pays for each f64 atan2/asin and texture walk once.
      bool end_sample = true, scattered_any = false;
      {
        const KScene S = load_scene(kargs());
        scattered_any = shade_ray(S, hr, o, d, rng, T_x, T_y, T_z, sum_x, sum_y, sum_z, first, hits);
        if (scattered_any) {
          depth--;
          end_sample = depth == 0;  // trace_path_continue(depth 0) is black (render.rs:128-131)
        }
      }
      first = false;

      // ---- end of a camera sample: accumulate (main.rs:80), maybe finish the pixel, start the next
      if (end_sample) {
        DREG(DREG_END_SAMPLE)
        DCYC_BEGIN(ce)
        KArgsPtr A = kargs();
        s++;
        ended_sample = true;
        if (s == unit_spp(A, batch)) {  // main.rs:86-87 (for this unit's batch of samples)
          DREG(DREG_END_PIXEL)
          if (PROBE) {
            // spp is 1 here: the sample traced max_bounce - depth scattered rays plus its last one; its cost
            // is their shading plus the traversal work counted in trav_step (node visits and primitive
            // tests: C5's rays differ far more in traversal than in path length)
            const uint32_t k = slot / A->P.probe_px, rays = A->P.max_bounce - depth + (scattered_any ? 0u : 1u);
            const uint32_t r = work + WORK_RAY * rays;
            work = 0;
            atomicAdd(&A->P.tile_cost[k], r);
            atomicMax(&A->P.tile_cost[TILE_SORT_MAX + k], r);
          } else if (A->P.nbatch == 1) {
            // (the unit's frame: its global batch, nbatch being 1)
            const double spp = (double)A->P.spp;
            double* out = A->out + (uint64_t)batch * A->P.out_stride;
            out[3 * (uint64_t)slot + 0] = sum_x / spp;
            out[3 * (uint64_t)slot + 1] = sum_y / spp;
            out[3 * (uint64_t)slot + 2] = sum_z / spp;
            if (A->out_fg) A->out_fg[(uint64_t)batch * A->P.n_slots + slot] = (float)((double)hits / spp);
          } else {  // one batch of several: its sum, reduced in batch order by reduce_batches
            // (frame f's sums follow frame f - 1's: index (f n_slots + slot) nbatch + b = slot nbatch + global batch
            // + f (n_slots - 1) nbatch)
            const uint64_t u = (uint64_t)slot * A->P.nbatch + batch +
                               (uint64_t)unit_frame(A, batch) * (A->P.n_slots - 1) * A->P.nbatch;
            double* part = A->P.partial;
            part[3 * u + 0] = sum_x;
            part[3 * u + 1] = sum_y;
            part[3 * u + 2] = sum_z;
            A->P.partial_hits[u] = hits;
          }
          // the unit's duration: its tile's measured cost (rp_kernel.h tile_meas), from one unit in eight (pixel and
          // batch hashed: every tile's sample spread over its pixels and batches) -- timing all units cost 0.9 % --
          // and every unit's duration for the next frame's per-unit order (unit_cost, rp_sched.hip)
          const bool mt = !PROBE && A->P.tile_meas && meas_unit(pipj, batch);
          if (!PROBE && (mt || A->P.unit_cost)) {
            const uint32_t dur = (uint32_t)__builtin_amdgcn_s_memrealtime() - A->S.unit_t0[blockIdx.x * BLOCK + tid];
            if (A->P.unit_cost)  // (every frame of a launch writes its unit's slot: any of them is the pixel's cost)
              A->P.unit_cost[(uint64_t)slot * A->P.nbatch + (batch - unit_frame(A, batch) * A->P.nbatch)] = dur;
            if (mt) {
              meas_dur = dur >> MEAS_SHIFT;
              meas_k = slot / (A->P.tw * A->P.th);
            }
          }
          ended_pixel = batch == unit_frame(A, batch) * A->P.nbatch;  // the pixel's first batch of its frame
          DIAG(if (!PROBE) {
            const uint32_t b = tbin(t_pix);
            atomicAdd(&A->diag[128 + b], (unsigned long long)(lane_rays - rays_pix));
            atomicAdd(&A->diag[192 + b], 1ull);
            atomicMax(&A->diag[256 + b], (unsigned long long)(lane_rays - rays_pix));
            {  // the slowest unit of the frame: duration (100 MHz ticks), its pixel and batch, and its rays
              const uint64_t now = __builtin_amdgcn_s_memrealtime();
              atomicMax(&A->diag[13], ((now - t_pix) << 32) | ((uint64_t)batch << 28) | (uint64_t)(pipj & 0x0FFFFFFFu));
              atomicMax(&A->diag[14], ((now - t_pix) << 32) | (uint64_t)(lane_rays - rays_pix));
              // the distribution of unit durations (log2 bins) and the rays those units traced
              const int lb = min(max(63 - __builtin_clzll((now - t_pix) | 1ull) - (int)DIAG_DUR_LOG0, 0), (int)DIAG_DUR_N - 1);
              atomicAdd(&A->diag[DIAG_DUR + lb], 1ull);
              atomicAdd(&A->diag[DIAG_DUR + DIAG_DUR_N + lb], (unsigned long long)(lane_rays - rays_pix));
            }
            t_pix = __builtin_amdgcn_s_memrealtime();
            rays_pix = lane_rays;
          })
          uint32_t pi = 0, pj = 0;
          alive = fetch_pixel<PROBE>(slot, pi, pj, batch);
          pipj = pi | (pj << 16);
          DIAG(if (!alive) t_retire = __builtin_amdgcn_s_memrealtime();)
          DIAG(if (!PROBE && !alive) atomicMax(&A->diag[11], ~(unsigned long long)__builtin_amdgcn_s_memrealtime());)
          if (alive) {
            fresh = true;
            s = 0;
            hits = 0;
            sum_x = sum_y = sum_z = 0.0;
          }
        }
        start = alive;  // next round, after the refill pass
        DCYC_END(DCYC_END_SAMPLE, ce)
      } else {
        DCYC_BEGIN(cb)
        trav_init<NF>(load_scene(kargs()), INF, ts, d);
        tdone = false;
        newray = true;
        DCYC_END(DCYC_NEXT_BOUNCE, cb)
      }
    }
    n_samples += (uint64_t)__popcll(__ballot(ended_sample));
    n_pixels += (uint64_t)__popcll(__ballot(ended_pixel));
    if (!PROBE) {
      // Tile costs: the wave's units that ended this round mostly belong to one tile (a wave fetches consecutive
      // units), so the wave sums and maxes their durations for the first ending lane's tile and adds them with one
      // atomic each -- 64 lanes' atomics on one word serialise in L2 -- and the rare lanes of other tiles add their own.
      const uint64_t em = __ballot(meas_k != 0xFFFFFFFFu);
      if (em != 0) {
        const uint32_t lead = (uint32_t)__builtin_ctzll(em);
        const uint32_t k0 = __builtin_amdgcn_readlane(meas_k, lead);
        const bool mine = meas_k == k0;
        uint32_t sum = mine ? meas_dur : 0u, mx = sum;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
          sum += __shfl_xor(sum, off);
          mx = max(mx, (uint32_t)__shfl_xor(mx, off));
        }
        uint32_t* meas = kargs()->P.tile_meas;
        if ((threadIdx.x & 63u) == lead) {
          atomicAdd(&meas[k0], sum);
          atomicMax(&meas[TILE_SORT_MAX + k0], mx);
        }
        if (meas_k != 0xFFFFFFFFu && !mine) {
          atomicAdd(&meas[meas_k], meas_dur);
          atomicMax(&meas[TILE_SORT_MAX + meas_k], meas_dur);
        }
      }
    }
    DIAG({ uint64_t t = stamp(); ph[3] += t - t_prev; t_prev = t; })
  }

#ifdef RPK_DIAG
  {
    // per-wave maxima over lanes (a lane stops counting when it retires), then summed over waves
    unsigned long long* dg = kargs()->diag;
    const uint64_t t = stamp();
    ph[4] += t - t_prev;
    const int w = threadIdx.x >> 6;
    for (int q = 0; q < 5; q++) atomicMax(&wmax[w][q], (unsigned long long)ph[q]);
    atomicMax(&wmax[w][5], (unsigned long long)iters);
    atomicMax(&wmax[w][6], (unsigned long long)td.trips);
    atomicAdd(&dg[8], (unsigned long long)td.visits);
    atomicAdd(&dg[9], (unsigned long long)td.tests);
    atomicAdd(&dg[6], (unsigned long long)active);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
      for (int q = 0; q < 6; q++) atomicAdd(&dg[q], wmax[w][q]);
      atomicAdd(&dg[7], wmax[w][6]);
    }
    if (threadIdx.x < 2 * DREG_N) atomicAdd(&dg[16 + threadIdx.x], g_dreg[threadIdx.x]);
    if (threadIdx.x < DCYC_N) atomicAdd(&dg[DIAG_CYC + threadIdx.x], g_dcyc[threadIdx.x]);
    if (!PROBE && (threadIdx.x & 63) == 0) atomicMax(&dg[12], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    if (!PROBE) atomicAdd(&dg[64 + tbin(t_retire)], 1ull);
  }
#endif
  if ((threadIdx.x & 63u) == 0) {
    atomicAdd(&blk_ctr[0], (unsigned long long)n_rays);
    atomicAdd(&blk_ctr[1], (unsigned long long)n_samples);
    atomicAdd(&blk_ctr[2], (unsigned long long)n_pixels);
  }
  unsigned long long* ctr = kargs()->ctr;
  if (overflow) atomicOr(&ctr[CTR_STATUS], (unsigned long long)STATUS_STACK_OVERFLOW);
  __syncthreads();
  if (threadIdx.x < 3) atomicAdd(&ctr[CTR_RAYS + threadIdx.x], blk_ctr[threadIdx.x]);
}

template <uint32_t NF>
__global__ void __launch_bounds__(BLOCK) intersect_kernel(const KScene S, const double* __restrict__ rays, uint64_t n,
                                                         double* __restrict__ out_hit, uint32_t* __restrict__ out_mat,
                                                         unsigned long long* __restrict__ ctr) {
  extern __shared__ uint32_t lds_stack[];
  const uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (i >= n) return;
  const double* q = rays + 8 * i;
  const V3 o = v3(q[0], q[1], q[2]), d = v3(q[3], q[4], q[5]);
  const double tmin = q[6], tmax = q[7];
  HitRec hr;
  bool overflow = false;
  traverse<NF>(S, (lds_u32*)(lds_stack + threadIdx.x), BLOCK, o, d, tmin, tmax, hr, overflow);
  double* oh = out_hit + 9 * i;
  if (hr.prim >= 0) {
    Surf h;
    if (surface(S, hr, o, d, h, true)) {  // Hittable::hit returns the full Hit record
      h.u = 0.5 - atan2(h.n.z, h.n.x) / TAU_;
      h.v = asin(h.n.y) / PI_ + 0.5;
    }
    oh[0] = hr.t; oh[1] = h.p.x; oh[2] = h.p.y; oh[3] = h.p.z;
    oh[4] = h.n.x; oh[5] = h.n.y; oh[6] = h.n.z; oh[7] = h.u; oh[8] = h.v;
    out_mat[i] = h.material;
  } else {
    oh[0] = INF;
    for (int k = 1; k < 9; k++) oh[k] = 0.0;
    out_mat[i] = 0xffffffffu;
  }
  if (overflow) atomicOr(&ctr[CTR_STATUS], (unsigned long long)STATUS_STACK_OVERFLOW);
}

int launch_render(const KScene& s, const KParams& p, double* out_rgb, float* out_fg, uint64_t* counters,
                  uint32_t* queue, int grid, void* stream) {
  const size_t lds = (size_t)s.lds_depth * BLOCK * sizeof(uint32_t);
  const bool spill = s.lds_depth < s.stack_depth;
  KArgs a;
  a.S = s;
  a.P = p;
  a.out = out_rgb;
  a.out_fg = out_fg;
  a.ctr = reinterpret_cast<unsigned long long*>(counters);
  a.queue = queue;
  a.diag = reinterpret_cast<unsigned long long*>(s.diag);
  const hipStream_t st = (hipStream_t)stream;
#define RPK_LAUNCH(P_, S_)                                                                                   \
  do {                                                                                                   \
    if (s.node_format == rpl::NODES_W8)                                                                  \
      hipLaunchKernelGGL((render_kernel<P_, S_, rpl::NODES_W8>), dim3(grid), dim3(BLOCK), lds, st, a);   \
    else if (s.node_format == rpl::NODES_Q8)                                                             \
      hipLaunchKernelGGL((render_kernel<P_, S_, rpl::NODES_Q8>), dim3(grid), dim3(BLOCK), lds, st, a);   \
    else                                                                                                 \
      hipLaunchKernelGGL((render_kernel<P_, S_, rpl::NODES_F32>), dim3(grid), dim3(BLOCK), lds, st, a);  \
  } while (0)
  if (p.probe && spill) RPK_LAUNCH(true, true);
  else if (p.probe) RPK_LAUNCH(true, false);
  else if (spill) RPK_LAUNCH(false, true);
  else RPK_LAUNCH(false, false);
#undef RPK_LAUNCH
  return (int)hipGetLastError();
}

// Multi-batch frames: pixel value = (S_0 + S_1 + ... + S_{nb-1}) / spp, added in batch order (the oracle's
// order), foreground likewise.  One thread per shard slot; slots of edge tiles outside the frame skipped.
__global__ void __launch_bounds__(256) reduce_batches_kernel(const KParams P, double* __restrict__ out,
                                                            float* __restrict__ out_fg) {
  const uint64_t slot = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (slot >= P.n_slots) return;
  const uint32_t tile_px = P.tw * P.th, k = (uint32_t)(slot / tile_px), local = (uint32_t)(slot % tile_px);
  const uint32_t dk = P.shard + k * P.nshards, t = P.tile_map ? P.tile_map[dk] : dk;
  if ((t % P.tiles_x) * P.tw + local % P.tw >= P.W || (t / P.tiles_x) * P.th + local / P.tw >= P.H) return;
  const double* part = P.partial + 3 * slot * P.nbatch;
  const uint32_t* ph = P.partial_hits + slot * P.nbatch;
  double x = 0.0, y = 0.0, z = 0.0;
  uint32_t h = 0;
  for (uint32_t b = 0; b < P.nbatch; b++) {
    x = x + part[3 * b];
    y = y + part[3 * b + 1];
    z = z + part[3 * b + 2];
    h += ph[b];
  }
  const double spp = (double)P.spp;
  out[3 * slot + 0] = x / spp;
  out[3 * slot + 1] = y / spp;
  out[3 * slot + 2] = z / spp;
  if (out_fg) out_fg[slot] = (float)((double)h / spp);
}

int launch_reduce_batches(const KParams& p, double* out_rgb, float* out_fg, void* stream) {
  if (p.n_slots == 0) return 0;
  hipLaunchKernelGGL(reduce_batches_kernel, dim3((unsigned)((p.n_slots + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, p, out_rgb, out_fg);
  return (int)hipGetLastError();
}

// Output stage (utility.rs:212-220 to_srgb_u8, image.rs:116-137 tga::save pixel order): per shard slot,
// linear f64 RGB -> B, G, R, 255 bytes.  `(255 * clamp(x, 0, 1).powf(1/2.2)) as u8` is a monotone step
// function of x, so the byte is the number of its 255 thresholds (the smallest x reaching 1, 2, ..., 255,
// found on the host with the host libm's pow -- the reference's own arithmetic) that x reaches: an 8-step
// binary search in an LDS copy of the table, no device pow, bit-identical by construction.  NaN reaches
// no threshold (Rust's saturating `as u8` maps NaN to 0), values above 1 reach all 255.
__global__ void __launch_bounds__(256) srgb_bgra_kernel(const SrgbTable tab, const double* __restrict__ rgb,
                                                       uint64_t n, uint32_t* __restrict__ bgra) {
  // the thresholds straight from the kernel-argument segment (constant memory, L1/K$-resident), not an LDS copy: a frame
  // gather runs while other frames' persistent render kernels hold every CU's LDS (see SORT_BLOCK)
  const double* thr = tab.thr;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    uint32_t px = 0xff000000u;
#pragma unroll
    for (int c = 0; c < 3; c++) {
      const double x = rgb[3 * i + c];
      uint32_t k = 0;
#pragma unroll
      for (uint32_t step = 128; step; step >>= 1)
        if (x >= thr[k + step]) k += step;
      px |= k << (8 * (2 - c));  // byte 0 = B, 1 = G, 2 = R, 3 = A
    }
    bgra[i] = px;
  }
}

int launch_srgb_bgra(const SrgbTable& tab, const double* rgb, uint64_t n, uint8_t* bgra, void* stream) {
  if (n == 0) return 0;
  const uint64_t blocks = (n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536;
  hipLaunchKernelGGL(srgb_bgra_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, tab, rgb, n,
                     reinterpret_cast<uint32_t*>(bgra));
  return (int)hipGetLastError();
}

// Multi-GPU frame assembly (rp_frame_gather): frame pixel (i, j) <- the slot of the rank owning its tile.
// Consecutive threads take consecutive pixels of a row, so the frame writes are coalesced; the reads are
// runs of tw slots.
__global__ void __launch_bounds__(256) frame_assemble_kernel(const FrameGeom g, const uint32_t* __restrict__ src,
                                                            uint32_t words, uint32_t* __restrict__ frame) {
  const uint64_t n = (uint64_t)g.W * g.H;
  for (uint64_t px = (uint64_t)blockIdx.x * 256 + threadIdx.x; px < n; px += (uint64_t)gridDim.x * 256) {
    const uint32_t j = (uint32_t)(px / g.W), i = (uint32_t)(px - (uint64_t)j * g.W);
    const uint32_t t = (j / g.th) * g.tiles_x + i / g.tw;
    const uint32_t pos = g.tile_pos ? g.tile_pos[t] : t;
    const uint32_t r = pos % g.nranks, k = pos / g.nranks;
    const uint64_t slot = (uint64_t)k * g.tw * g.th + (uint64_t)(j % g.th) * g.tw + i % g.tw;
    const uint64_t rw = g.rank_words ? g.rank_words : g.stride * words;
    const uint32_t* s = src + (uint64_t)r * rw + slot * words;
    for (uint32_t w = 0; w < words; w++) frame[px * words + w] = s[w];
  }
}

int launch_frame_assemble(const FrameGeom& g, const uint32_t* gathered, uint32_t words, uint32_t* frame, void* stream) {
  const uint64_t n = (uint64_t)g.W * g.H;
  if (n == 0) return 0;
  const uint64_t blocks = (n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536;
  hipLaunchKernelGGL(frame_assemble_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, g, gathered,
                     words, frame);
  return (int)hipGetLastError();
}

// The tile sorts below are one-block bitonic sorts over a workspace scratch array in GLOBAL memory (L2-resident, at
// most 128 KB), with no LDS and few registers.  They run in front of a frame's render, and with frames in flight
// another frame's persistent render kernel holds every CU's LDS: a block that needs LDS (the first form sorted in
// 64-128 KB of it) waited 20-78 ms for a CU to drain (profiles/r3 shard trace), so the next frame could not start
// filling the CUs the previous one released.  A 256-thread block without LDS fits beside the render waves at once.
// __syncthreads() orders the block's global accesses (workgroup-scope fence: the waves share one CU's L1).
static constexpr int SORT_BLOCK = 256;
template <class T>
__device__ __forceinline__ void bitonic_global(T* __restrict__ key, uint32_t np2) {
  for (uint32_t size = 2; size <= np2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = threadIdx.x; i < np2; i += SORT_BLOCK) {
        const uint32_t j = i ^ stride;
        if (j > i) {
          const T a = key[i], b = key[j];
          const bool up = (i & size) == 0;
          if ((a > b) == up) { key[i] = b; key[j] = a; }
        }
      }
      __syncthreads();
    }
  }
}

static_assert(TILE_SORT_MAX <= (1 << 14), "tile index field is 14 bits");
// Buckets per octave of cost.  Inside a bucket the tiles keep their Z-order, so coarser buckets trade cost order for
// locality: octave buckets C5 -1.7 % against quarter-octave ones (C3 -0.1 %); two octaves per bucket C5 -2.0 % but C3
// +0.5 % (profiles/r4/c3_c5_sort_buckets*_ab.json, learned costs and per-XCD queues; the probe-era C3 sweep preferred 4)
static constexpr float SORT_Q = 1.0f;
__device__ __forceinline__ uint32_t spread8(uint32_t v) {  // 8 bits -> every other bit of 16
  v = (v | (v << 4)) & 0x0F0Fu;
  v = (v | (v << 2)) & 0x3333u;
  return (v | (v << 1)) & 0x5555u;
}
__device__ __forceinline__ uint32_t compact8(uint32_t v) {  // inverse of spread8
  v &= 0x5555u;
  v = (v | (v >> 1)) & 0x3333u;
  v = (v | (v >> 2)) & 0x0F0Fu;
  return (v | (v >> 4)) & 0x00FFu;
}

// Keys: [31:28] 0 | [27:22] 63 - costliest-sample bucket | [21:16] 63 - mean-cost bucket | [15:0] Z-order code of
// the tile's frame coordinates (both < 256), which also identifies the tile.  Ascending order = costliest
// buckets first, Z-order inside a bucket (row-major inside a bucket measured the same on C3: 247.4 vs 247.5
// ms); without costs (cost == NULL) plain Z-order.
__global__ void __launch_bounds__(SORT_BLOCK) tile_sort_kernel(const uint32_t* __restrict__ cost, uint32_t n,
                                                               uint32_t probe_px, uint32_t np2, TileGeom g,
                                                               uint32_t* __restrict__ order, uint32_t* __restrict__ key) {
  for (uint32_t i = threadIdx.x; i < np2; i += SORT_BLOCK) {
    uint32_t kk = 0xFFFFFFFFu;
    if (i < n) {
      const uint32_t dk = g.shard + i * g.nshards, t = g.map ? g.map[dk] : dk, tx = t % g.tiles_x, ty = t / g.tiles_x;
      uint32_t ql = 0, qm = 0;
      if (cost) {
        // SORT_Q buckets per octave of the costliest probed (or measured) sample's cost and of the mean cost
        const uint32_t c = g.cost_by_tile ? t : i;
        const float mean = (float)cost[c] / (float)probe_px;
        ql = min((uint32_t)(log2f((float)cost[TILE_SORT_MAX + c] + 1.0f) * SORT_Q), 63u);
        qm = min((uint32_t)(log2f(mean + 1.0f) * SORT_Q), 63u);
      }
      kk = ((63u - ql) << 22) | ((63u - qm) << 16) | (spread8(ty) << 1) | spread8(tx);
    }
    key[i] = kk;
  }
  __syncthreads();
  bitonic_global(key, np2);
  // back from the frame tile to its shard tile index: the inverse deal order (plan[n_tiles + t], laid out by
  // launch_tile_plan right behind the order) or the interleave's (t - shard) / nshards
  const uint32_t n_tiles = g.map ? g.map_tiles : 0u;
  for (uint32_t i = threadIdx.x; i < n; i += SORT_BLOCK) {
    const uint32_t m = key[i] & 0xFFFFu, tx = compact8(m), ty = compact8(m >> 1), t = ty * g.tiles_x + tx;
    order[i] = g.map ? g.map[n_tiles + t] / g.nshards : (t - g.shard) / g.nshards;
  }
}

int launch_tile_sort(const uint32_t* cost, uint32_t n, uint32_t probe_px, const TileGeom& g, uint32_t* order,
                     uint64_t* scratch, void* stream) {
  if (n == 0 || n > TILE_SORT_MAX) return (int)hipErrorInvalidValue;
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  hipLaunchKernelGGL(tile_sort_kernel, dim3(1), dim3(SORT_BLOCK), 0, (hipStream_t)stream, cost, n, probe_px, np2, g,
                     order, reinterpret_cast<uint32_t*>(scratch));
  return (int)hipGetLastError();
}

// Balanced tile plan (rp_kernel.h launch_tile_plan).  One block: the n frame tiles sorted by 64-bit key
// (~block cost << 32 | block << 14 | tile: descending block cost, a block's tiles together; 16384 tiles = 128 KB of
// global scratch), then dealt in units of block x block sorted positions, rounds of nranks units alternating direction
// ("snake": round k gives its units to ranks 0..N-1 when k is even, N-1..0 when odd, so each pair of rounds gives
// every rank one unit from the costly and one from the cheap end of the pair's 2N-unit range), and the positions past
// the last whole round tile by tile the same way, the last partial round forward -- every rank gets exactly the
// interleave's tile count, so shard sizes and gather strides do not change.  With block = 1 this is the per-tile deal
// (block index = tile index).  The deal is parallel (position p of the sorted order -> rank and shard tile), its
// imbalance is second order in the cost curve (a greedy LPT step per tile would be a serial loop of n wave
// reductions).  Deterministic: integer keys and sums, no atomics but order-free integer adds.
static constexpr int PLAN_BLOCK = SORT_BLOCK;
__device__ __forceinline__ uint64_t mix64(uint64_t z) {  // splitmix64 finaliser
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ void __launch_bounds__(PLAN_BLOCK) tile_plan_kernel(const uint32_t* __restrict__ cost, uint32_t n,
                                                               uint32_t np2, uint32_t N, uint32_t tiles_x, uint32_t bs,
                                                               uint32_t* __restrict__ plan,
                                                               unsigned long long* __restrict__ key) {
  // scratch: key[0, np2) the sort keys, key[TILE_SORT_MAX] the plan hash's accumulator, key[TILE_SORT_MAX + 1 + b] block
  // b's summed cost (global, like the keys: no LDS, see SORT_BLOCK)
  unsigned long long* hash = key + TILE_SORT_MAX;
  unsigned long long* bcost = key + TILE_SORT_MAX + 1;
  const uint32_t bx_n = (tiles_x + bs - 1) / bs;
  auto block_of = [&](uint32_t t) { return (t / tiles_x / bs) * bx_n + (t % tiles_x) / bs; };
  if (threadIdx.x == 0) *hash = 0;
  for (uint32_t i = threadIdx.x; i < n; i += PLAN_BLOCK) bcost[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += PLAN_BLOCK) atomicAdd(&bcost[block_of(i)], (unsigned long long)cost[i]);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < np2; i += PLAN_BLOCK) {
    if (i < n) {
      const uint32_t b = block_of(i);
      const uint64_t c = min(bcost[b], 0xFFFFFFFFull);
      key[i] = ((0xFFFFFFFFull - c) << 32) | ((uint64_t)b << 14) | i;
    } else {
      key[i] = ~0ull;
    }
  }
  __syncthreads();
  bitonic_global(key, np2);
  const uint32_t U = bs * bs, R = n / (U * N), head = R * U * N;  // whole rounds of N units
  const uint32_t tail_full = (n - head) / N;                        // whole tile rounds past them
  uint64_t h = 0;
  for (uint32_t p = threadIdx.x; p < n; p += PLAN_BLOCK) {
    const uint32_t t = (uint32_t)key[p] & 0x3FFFu;
    uint32_t rank, j;
    if (p < head) {
      const uint32_t u = p / U, k = u / N, i = u - k * N;
      rank = (k & 1u) ? N - 1u - i : i;
      j = k * U + (p - u * U);
    } else {
      const uint32_t q = p - head, k = q / N, i = q - k * N;
      rank = (k < tail_full && (k & 1u)) ? N - 1u - i : i;
      j = R * U + k;
    }
    const uint32_t pos = j * N + rank;
    plan[pos] = t;
    plan[n + t] = pos;
    h += mix64(((uint64_t)pos << 32) | t);
  }
  atomicAdd(hash, (unsigned long long)h);
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t v = mix64(atomicAdd(hash, 0ull) ^ ((uint64_t)n << 32 | N)) | 1ull;  // never 0 (0 = the interleave)
    plan[2 * n] = (uint32_t)v;
    plan[2 * n + 1] = (uint32_t)(v >> 32);
  }
}

int launch_tile_plan(const uint32_t* cost, uint32_t n, uint32_t nranks, uint32_t tiles_x, uint32_t block, uint32_t* plan,
                     uint64_t* scratch, void* stream) {
  if (n == 0 || n > TILE_SORT_MAX || nranks == 0 || tiles_x == 0 || block == 0) return (int)hipErrorInvalidValue;
  uint32_t np2 = 1;
  while (np2 < n) np2 <<= 1;
  hipLaunchKernelGGL(tile_plan_kernel, dim3(1), dim3(PLAN_BLOCK), 0, (hipStream_t)stream, cost, n, np2, nranks, tiles_x,
                     block, plan, reinterpret_cast<unsigned long long*>(scratch));
  return (int)hipGetLastError();
}

// The packed block of a frame gather (rp_kernel.h launch_gather_pack) and the counter reduction.  Small kernels
// without LDS that fit beside in-flight render waves.
__global__ void __launch_bounds__(256) gather_pack_kernel(const uint64_t* __restrict__ ctr, const uint32_t* __restrict__ hash,
                                                          const uint32_t* __restrict__ meas, uint32_t st,
                                                          uint32_t* __restrict__ send) {
  const uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < GATHER_CTR) {
    uint64_t v = 0;
    if (i < CTR_N) v = ctr ? ctr[i] : 0ull;
    else if (i == GATHER_CTR_HASH) v = hash ? ((uint64_t)hash[1] << 32 | hash[0]) : 0ull;
    reinterpret_cast<uint64_t*>(send)[i] = v;
  }
  if (i < 2 * st) {  // sums [0, st), maxima [st, 2 st): the measured table holds TILE_SORT_MAX of each
    const uint32_t half = i < st ? 0u : 1u, k = i - half * st;
    send[2 * GATHER_CTR + i] = meas && k < (uint32_t)TILE_SORT_MAX ? meas[half * TILE_SORT_MAX + k] : 0u;
  }
}
__global__ void counters_reduce_kernel(const uint64_t* __restrict__ g, uint32_t nranks, uint64_t rank_u64,
                                       uint64_t* __restrict__ out) {
  if (threadIdx.x != 0) return;
  uint64_t rays = 0, samples = 0, pixels = 0, status = 0;
  for (uint32_t r = 0; r < nranks; r++) {
    const uint64_t* b = g + (uint64_t)r * rank_u64;
    rays += b[CTR_RAYS];
    samples += b[CTR_SAMPLES];
    pixels += b[CTR_PIXELS];
    status |= b[CTR_STATUS];
    if (b[GATHER_CTR_HASH] != g[GATHER_CTR_HASH]) status |= STATUS_PLAN_MISMATCH;
  }
  out[CTR_RAYS] = rays;
  out[CTR_SAMPLES] = samples;
  out[CTR_PIXELS] = pixels;
  out[CTR_STATUS] = status;
}
int launch_gather_pack(const uint64_t* ctr, const uint32_t* hash, const uint32_t* meas, uint32_t stride_tiles,
                       uint32_t* send, void* stream) {
  const uint32_t n = 2 * stride_tiles > GATHER_CTR ? 2 * stride_tiles : GATHER_CTR;
  hipLaunchKernelGGL(gather_pack_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, ctr, hash, meas,
                     stride_tiles, send);
  return (int)hipGetLastError();
}
int launch_counters_reduce(const uint64_t* gathered, uint32_t nranks, uint64_t rank_words, uint64_t* out, void* stream) {
  hipLaunchKernelGGL(counters_reduce_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, gathered, nranks, rank_words / 2,
                     out);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(256) learn_costs_kernel(const uint32_t* __restrict__ sum, const uint32_t* __restrict__ mx,
                                                         uint32_t rank_stride, uint32_t N, uint32_t n,
                                                         const uint32_t* __restrict__ plan, uint32_t* __restrict__ fcost) {
  const uint32_t pos = blockIdx.x * 256 + threadIdx.x;
  if (pos >= n) return;
  const uint32_t r = pos % N, k = pos / N, t = plan ? plan[pos] : pos;
  fcost[t] = sum[r * rank_stride + k];
  fcost[TILE_SORT_MAX + t] = mx[r * rank_stride + k];
}

int launch_learn_costs(const uint32_t* sum, const uint32_t* max, uint32_t rank_stride, uint32_t nranks, uint32_t n_tiles,
                       const uint32_t* plan, uint32_t* fcost, void* stream) {
  if (n_tiles == 0 || n_tiles > TILE_SORT_MAX || nranks == 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(learn_costs_kernel, dim3((n_tiles + 255) / 256), dim3(256), 0, (hipStream_t)stream, sum, max,
                     rank_stride, nranks, n_tiles, plan, fcost);
  return (int)hipGetLastError();
}

uint64_t rng_slab_bytes_per_lane() { return (uint64_t)SLAB_N * sizeof(uint4); }

int render_blocks_per_cu(uint32_t lds_depth, bool spill, uint32_t nf, int* blocks) {
  const size_t lds = (size_t)lds_depth * BLOCK * sizeof(uint32_t);
  if (nf == rpl::NODES_W8) {
    if (spill) return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, render_kernel<false, true, rpl::NODES_W8>, BLOCK, lds);
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, render_kernel<false, false, rpl::NODES_W8>, BLOCK, lds);
  }
  if (nf == rpl::NODES_Q8) {
    if (spill) return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, render_kernel<false, true, rpl::NODES_Q8>, BLOCK, lds);
    return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, render_kernel<false, false, rpl::NODES_Q8>, BLOCK, lds);
  }
  if (spill) return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, render_kernel<false, true, rpl::NODES_F32>, BLOCK, lds);
  return (int)hipOccupancyMaxActiveBlocksPerMultiprocessor(blocks, render_kernel<false, false, rpl::NODES_F32>, BLOCK, lds);
}

int launch_intersect(const KScene& s, const double* rays, uint64_t n, double* out_hit, uint32_t* out_mat,
                     uint64_t* counters, void* stream) {
  if (n == 0) return 0;
  const size_t lds = (size_t)s.stack_depth * BLOCK * sizeof(uint32_t);
  const uint64_t grid = (n + BLOCK - 1) / BLOCK;
  if (s.node_format == rpl::NODES_W8)
    hipLaunchKernelGGL(intersect_kernel<rpl::NODES_W8>, dim3((unsigned)grid), dim3(BLOCK), lds, (hipStream_t)stream, s,
                       rays, n, out_hit, out_mat, reinterpret_cast<unsigned long long*>(counters));
  else if (s.node_format == rpl::NODES_Q8)
    hipLaunchKernelGGL(intersect_kernel<rpl::NODES_Q8>, dim3((unsigned)grid), dim3(BLOCK), lds, (hipStream_t)stream, s,
                       rays, n, out_hit, out_mat, reinterpret_cast<unsigned long long*>(counters));
  else
    hipLaunchKernelGGL(intersect_kernel<rpl::NODES_F32>, dim3((unsigned)grid), dim3(BLOCK), lds, (hipStream_t)stream, s,
                       rays, n, out_hit, out_mat, reinterpret_cast<unsigned long long*>(counters));
  return (int)hipGetLastError();
}

}  // namespace rpk
