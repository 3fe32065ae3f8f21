// Cost of lane selects on gfx950 (measurement tool, not product code).  tools/valu_rates.hip measured a VOP2
// v_cndmask_b32 (lane mask in VCC) at ~23 SIMD cycles per wave-instruction against ~4 for the VOP3 form with the mask
// in another SGPR pair; this probe times the render kernel's own pattern -- the 5-exchange sorting network of the 4-wide
// node visit (rp_device.h trav_step: (t_near, entry) pairs, compare + 4 selects per exchange) -- compiled from C as the
// kernel is, against the same network with branch-free integer swaps (non-negative f32 keys order as integers), and a
// baseline that only perturbs the keys.  Reports SIMD cycles per network at 4 and 8 waves per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -o raytracing-potato_amd/lib/select_probe tools/select_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

enum Variant { BASE, SELECT, XORSWAP, SELECT_E64, SELECT_E64_VCC, N_VAR };
static const char* kNames[N_VAR] = {"perturb only", "C selects (compiler's choice)", "integer xor swaps",
                                    "asm v_cmp_e64 + v_cndmask_b32_e64", "asm v_cmp_e32 vcc + v_cndmask_b32_e64 (vcc)"};

__device__ __forceinline__ uint64_t cmp_lt_f32(float a, float b) {
  uint64_t m;
  asm volatile("v_cmp_lt_f32_e64 %0, %1, %2\n\ts_nop 1" : "=s"(m) : "v"(a), "v"(b));
  return m;
}
__device__ __forceinline__ uint32_t sel(uint64_t m, uint32_t f, uint32_t t) {  // m ? t : f per lane
  uint32_t r;
  asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(f), "v"(t), "s"(m));
  return r;
}

template <int V>
__global__ __launch_bounds__(64) void net_kernel(uint32_t* out, int trips) {
  float tn[4];
  uint32_t cc[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    tn[i] = (float)((threadIdx.x * 7 + i * 13) & 31) + 0.5f;
    cc[i] = threadIdx.x * 4 + i;
  }
  uint32_t acc = 0;
  for (int t = 0; t < trips; t++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
#pragma unroll
      for (int i = 0; i < 4; i++) tn[i] = fmaf(tn[i], 0.75f, (float)(i + 1));  // keys stay positive and reshuffle
      if constexpr (V == SELECT) {
#define CSWAP(a, b) { const bool sw = tn[b] < tn[a]; const float t_ = sw ? tn[b] : tn[a]; tn[b] = sw ? tn[a] : tn[b]; \
                      tn[a] = t_; const uint32_t c_ = sw ? cc[b] : cc[a]; cc[b] = sw ? cc[a] : cc[b]; cc[a] = c_; }
        CSWAP(0, 1) CSWAP(2, 3) CSWAP(0, 2) CSWAP(1, 3) CSWAP(1, 2)
#undef CSWAP
      }
      if constexpr (V == XORSWAP) {
        uint32_t k[4];
#pragma unroll
        for (int i = 0; i < 4; i++) k[i] = __float_as_uint(tn[i]);
#define XSWAP(a, b) { const uint32_t m = (uint32_t)((int32_t)(k[b] - k[a]) >> 31); \
                      const uint32_t dk = (k[a] ^ k[b]) & m; k[a] ^= dk; k[b] ^= dk; \
                      const uint32_t dc = (cc[a] ^ cc[b]) & m; cc[a] ^= dc; cc[b] ^= dc; }
        XSWAP(0, 1) XSWAP(2, 3) XSWAP(0, 2) XSWAP(1, 3) XSWAP(1, 2)
#undef XSWAP
#pragma unroll
        for (int i = 0; i < 4; i++) tn[i] = __uint_as_float(k[i]);
      }
      if constexpr (V == SELECT_E64) {
#define ESWAP(a, b) { const uint64_t m = cmp_lt_f32(tn[b], tn[a]); \
                      const uint32_t ta = sel(m, __float_as_uint(tn[a]), __float_as_uint(tn[b])); \
                      const uint32_t tb = sel(m, __float_as_uint(tn[b]), __float_as_uint(tn[a])); \
                      tn[a] = __uint_as_float(ta); tn[b] = __uint_as_float(tb); \
                      const uint32_t ca = sel(m, cc[a], cc[b]), cb = sel(m, cc[b], cc[a]); cc[a] = ca; cc[b] = cb; }
        ESWAP(0, 1) ESWAP(2, 3) ESWAP(0, 2) ESWAP(1, 3) ESWAP(1, 2)
#undef ESWAP
      }
      if constexpr (V == SELECT_E64_VCC) {
#define VSWAP(a, b) { uint32_t ta, tb, ca, cb; \
        asm volatile("v_cmp_lt_f32_e32 vcc, %4, %5\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, %6, %7, vcc\n\t" \
                     "v_cndmask_b32_e64 %1, %7, %6, vcc\n\tv_cndmask_b32_e64 %2, %8, %9, vcc\n\tv_cndmask_b32_e64 %3, %9, %8, vcc" \
                     : "=&v"(ta), "=&v"(tb), "=&v"(ca), "=&v"(cb) \
                     : "v"(tn[b]), "v"(tn[a]), "v"(__float_as_uint(tn[a])), "v"(__float_as_uint(tn[b])), "v"(cc[a]), "v"(cc[b]) \
                     : "vcc"); \
        tn[a] = __uint_as_float(ta); tn[b] = __uint_as_float(tb); cc[a] = ca; cc[b] = cb; }
        VSWAP(0, 1) VSWAP(2, 3) VSWAP(0, 2) VSWAP(1, 3) VSWAP(1, 2)
#undef VSWAP
      }
      acc += cc[0] ^ cc[3];
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc + __float_as_uint(tn[0] + tn[1] + tn[2] + tn[3]);
}

template <int V>
static float run(uint32_t* out, int blocks, int trips) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  net_kernel<V><<<blocks, 64>>>(out, 1);
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e0));
  net_kernel<V><<<blocks, 64>>>(out, trips);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return ms;
}

int main(int argc, char** argv) {
  const double mhz = argc > 1 ? std::atof(argv[1]) : 2400.0;
  const int trips = argc > 2 ? std::atoi(argv[2]) : 200000;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int simds = p.multiProcessorCount * 4;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&out, sizeof(uint32_t) * 64 * simds * 8));
  // the sorted output must agree between the variants (same keys, same network)
  std::printf("{\"device\": \"%s\", \"clock_mhz_assumed\": %.0f, \"networks_per_wave\": %d, \"variants\": {", p.gcnArchName,
              mhz, trips * 8);
  for (int v = 0; v < N_VAR; v++) {
    std::printf("%s\"%s\": {", v ? ", " : "", kNames[v]);
    for (int w : {4, 8}) {
      const int blocks = simds * w;
      float ms = 0;
      switch (v) {
        case BASE: ms = run<BASE>(out, blocks, trips); break;
        case SELECT: ms = run<SELECT>(out, blocks, trips); break;
        case XORSWAP: ms = run<XORSWAP>(out, blocks, trips); break;
        case SELECT_E64: ms = run<SELECT_E64>(out, blocks, trips); break;
        case SELECT_E64_VCC: ms = run<SELECT_E64_VCC>(out, blocks, trips); break;
      }
      std::printf("%s\"waves_per_simd_%d\": {\"ms\": %.3f, \"simd_cycles_per_network\": %.2f}", w == 4 ? "" : ", ", w, ms,
                  ms * 1e-3 * mhz * 1e6 / ((double)trips * 8 * w));
    }
    std::printf("}");
  }
  std::printf("}}\n");
  CHECK(hipFree(out));
  return 0;
}
