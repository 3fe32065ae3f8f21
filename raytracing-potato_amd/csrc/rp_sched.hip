// rp_sched.hip -- the learned per-unit dispatch order of the render kernel (rp_kernel.h launch_unit_order).
//
// A frame ends when its longest unit ends: a unit (pixel, sample stream) is a chain of dependent rays on one lane, so
// a long unit handed out late is a latency-bound tail by itself.  Under SURVEY.md 8c's one stream per pixel a C3 unit
// is a whole 256-sample pixel -- up to ~2,000 rays (a glass-bunny pixel), 100-290 ms -- and the per-tile cost order
// leaves those pixels wherever their tile's row-major order puts them.  Every render stores each unit's duration
// (rp_kernel.h KParams::unit_cost); the next frame of the same shape sorts its units by it, longest first
// (longest-processing-time first), in log-spaced buckets (UNIT_ORDER_Q per octave) inside which the units keep their
// shard order (tile-major: neighbouring pixels stay together for the caches).  Results never depend on the order.
// Measured (round 6, bucket fix below): a lone C3 frame under the one-stream contract 220.1 ms against 260.8 ms in tile
// order (-15.6 %); in 32-sample streams 213.8 vs 204.8 ms (+4.4 %): AUTO = LEARNED for lone one-stream frames only.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "rp_kernel.h"

namespace rpk {

// key = (255 - bucket) << 32 | unit: ascending = longest buckets first, shard order inside a bucket.  Units that never
// ran (edge-tile slots outside the frame: cost 0) sort last.  A duration is in 100 MHz ticks, so its bucket
// log2(c) * UNIT_ORDER_Q + 1 reaches ~130 for a 300 ms unit: the bucket field has 8 bits.  (Round 5 clamped it to 63,
// ~0.46 ms: nearly every unit shared the top bucket and the "learned" order was shard order -- ADVICE r5.)
// the sort bucket of a unit of duration c (100 MHz ticks): 0 for a unit that never ran, else log2(c) * Q + 1 (<= 254)
__device__ __forceinline__ uint32_t unit_bucket(uint32_t c) {
  if (c == 0u) return 0u;
  return min((uint32_t)(log2f((float)c) * (float)UNIT_ORDER_Q) + 1u, 254u);
}

__global__ void __launch_bounds__(256) unit_keys_kernel(const uint32_t* __restrict__ cost, uint64_t n,
                                                        unsigned long long* __restrict__ key) {
  const uint64_t u = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= n) return;
  const uint32_t c = cost[u];
  key[u] = ((unsigned long long)(255u - unit_bucket(c)) << 32) | u;
}

__global__ void __launch_bounds__(256) unit_order_kernel(const unsigned long long* __restrict__ key, uint64_t n,
                                                         uint32_t* __restrict__ order) {
  const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (p < n) order[p] = (uint32_t)key[p];
}

size_t unit_order_scratch_bytes(uint64_t n) {
  size_t bytes = 0;
  if (n == 0 || n >= (1ull << 31)) return 0;
  if (hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                        (int)n, 0, UNIT_KEY_BITS) != hipSuccess)
    return 0;
  return bytes;
}

int launch_unit_order(const uint32_t* cost, uint64_t n, uint64_t* keys, uint64_t* keys2, void* scratch,
                      size_t scratch_bytes, uint32_t* order, void* stream) {
  if (n == 0 || n >= (1ull << 31)) return (int)hipErrorInvalidValue;
  const hipStream_t st = (hipStream_t)stream;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(unit_keys_kernel, dim3(blocks), dim3(256), 0, st, cost, n,
                     reinterpret_cast<unsigned long long*>(keys));
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  size_t bytes = scratch_bytes;
  // bits 0-30 the unit, 32-39 the bucket
  e = hipcub::DeviceRadixSort::SortKeys(scratch, bytes, reinterpret_cast<unsigned long long*>(keys),
                                        reinterpret_cast<unsigned long long*>(keys2), (int)n, 0, UNIT_KEY_BITS, st);
  if (e != hipSuccess) return (int)e;
  hipLaunchKernelGGL(unit_order_kernel, dim3(blocks), dim3(256), 0, st,
                     reinterpret_cast<const unsigned long long*>(keys2), n, order);
  return (int)hipGetLastError();
}

}  // namespace rpk
