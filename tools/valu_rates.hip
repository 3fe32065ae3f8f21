// VALU throughput of the instructions the Node4Q decode could use (measurement tool, not product code): each kernel
// runs a long unrolled stream of ONE instruction (inline asm, 8 independent destinations per round) on every resident
// wave, and the host reports the SIMD cycles per wave-instruction from the wall time at the clock given on the command
// line (and from each wave's own clock64), for 2, 4 and 8 waves per SIMD.  The candidates: v_cvt_f32_ubyte0 + v_pk_fma_f32 (the decode of v58) against
// v_perm_b32 + v_fma_mix_f32 (byte codes as f16 subnormals).
//
//   hipcc --offload-arch=gfx950 -O3 -o raytracing-potato_amd/lib/valu_rates tools/valu_rates.hip
//   raytracing-potato_amd/lib/valu_rates [clock_mhz]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

enum Op { FMA_F32, FMAC_F32, ADD_F32, MUL_F32, MAX_F32, MAX3_F32, MED3_F32, PK_FMA_F32, PK_ADD_F32, PK_MUL_F32, FMA_MIX_F32, CVT_UBYTE0, CVT_F32_U32, CVT_F64_U32, CVT_F32_F64, FMA_F64, ADD_F64, MUL_F64, CMP_LT_F64, ADD_U32, XOR_B32, AND_B32, LSHLREV_B32, ALIGNBIT_B32, PERM_B32, ADD3_U32, XAD_U32, LSHL_OR_B32, BFE_U32, MUL_LO_U32, MOV_B32, CNDMASK_B32, CMP_LT_F32, CMP_LT_U32_E64, CNDMASK_E64_SGPR, CNDMASK_VCC_INDEP, CNDMASK_E64_INDEP, CMP_CNDMASK_PAIR, CMP_NOP_4CND, SMOV_4CND, CMP_ONCE_CND, CMP_E64_4CND_E64, MAX_I32, MIN_U32, MAX3_I32, MIN3_U32, SUB_U32, OR_B32, LSHRREV_B32, OR3_B32, AND_OR_B32, BFI_B32, MUL_U32_U24, SUBREV_U32, NOT_B32, ADD_CO_U32, LSHL_ADD_U32, CMP_EQ_U32_E32, N_OPS };
static const char* kNames[N_OPS] = {"v_fma_f32", "v_fmac_f32", "v_add_f32", "v_mul_f32", "v_max_f32", "v_max3_f32", "v_med3_f32", "v_pk_fma_f32", "v_pk_add_f32", "v_pk_mul_f32", "v_fma_mix_f32", "v_cvt_f32_ubyte0", "v_cvt_f32_u32", "v_cvt_f64_u32", "v_cvt_f32_f64", "v_fma_f64", "v_add_f64", "v_mul_f64", "v_cmp_lt_f64", "v_add_u32", "v_xor_b32", "v_and_b32", "v_lshlrev_b32", "v_alignbit_b32", "v_perm_b32", "v_add3_u32", "v_xad_u32", "v_lshl_or_b32", "v_bfe_u32", "v_mul_lo_u32", "v_mov_b32", "v_cndmask_b32", "v_cmp_lt_f32", "v_cmp_lt_u32_e64", "v_cndmask_b32_e64 (sgpr mask)", "v_cndmask_b32 (vcc, independent)", "v_cndmask_b32_e64 (sgpr, independent)", "v_cmp_lt_f32 + v_cndmask_b32 pair", "v_cmp vcc + s_nop 1 + 4 v_cndmask (vcc)", "s_mov_b64 vcc + 4 v_cndmask (vcc)", "v_cndmask (vcc set by v_cmp before the loop)", "v_cmp_e64 sgpr + 4 v_cndmask_e64 (sgpr)", "v_max_i32", "v_min_u32", "v_max3_i32", "v_min3_u32", "v_sub_u32", "v_or_b32", "v_lshrrev_b32", "v_or3_b32", "v_and_or_b32", "v_bfi_b32", "v_mul_u32_u24", "v_subrev_u32", "v_not_b32", "v_add_co_u32", "v_lshl_add_u32", "v_cmp_eq_u32_e32"};
constexpr int kRounds = 64;  // unrolled rounds of 8 instructions per loop trip

template <int OP>
__global__ __launch_bounds__(64) void stream_kernel(float* out, unsigned long long* clk, int trips) {
  const unsigned long long c0 = clock64(), r0 = wall_clock64();
  float a[8];
  double d[8];
  uint32_t u[8];
  unsigned long long m[8] = {};
  const unsigned long long msk = 0xAAAAAAAAAAAAAAAAull ^ (unsigned long long)blockIdx.x;
  const float x = (float)threadIdx.x * 1e-3f;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    a[j] = x + (float)j;
    d[j] = (double)a[j];
    u[j] = threadIdx.x * 0x01010101u + (uint32_t)j;
  }
  const float b = 0.999f, c = 1e-6f;
  const double db = 0.999, dc = 1e-6;
  const uint32_t sel = 0x0c010c00u;
  if constexpr (OP == CMP_ONCE_CND) asm volatile("v_cmp_lt_u32 vcc, %0, %1\n\ts_nop 4" : : "v"(u[0]), "v"(sel) : "vcc");
  for (int t = 0; t < trips; t++) {
#pragma unroll
    for (int r = 0; r < kRounds; r++) {
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if constexpr (OP == FMA_F32) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
        if constexpr (OP == FMAC_F32) asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
        if constexpr (OP == ADD_F32) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b), "v"(c));
        if constexpr (OP == MUL_F32) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b), "v"(c));
        if constexpr (OP == MAX_F32) asm volatile("v_max_f32 %0, %0, %1" : "+v"(a[j]) : "v"(b), "v"(c));
        if constexpr (OP == MAX3_F32) asm volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
        if constexpr (OP == MED3_F32) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[j]) : "v"(b), "v"(c));
        if constexpr (OP == PK_FMA_F32) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(d[j]) : "v"(db), "v"(dc));
        if constexpr (OP == PK_ADD_F32) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(d[j]) : "v"(db), "v"(dc));
        if constexpr (OP == PK_MUL_F32) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(d[j]) : "v"(db), "v"(dc));
        if constexpr (OP == FMA_MIX_F32) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(a[j]) : "v"(u[j]), "v"(b));
        if constexpr (OP == CVT_UBYTE0) asm volatile("v_cvt_f32_ubyte0 %0, %1" : "=v"(a[j]) : "v"(u[j]));
        if constexpr (OP == CVT_F32_U32) asm volatile("v_cvt_f32_u32 %0, %1" : "=v"(a[j]) : "v"(u[j]));
        if constexpr (OP == CVT_F64_U32) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(d[j]) : "v"(u[j]));
        if constexpr (OP == CVT_F32_F64) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(a[j]) : "v"(d[j]));
        if constexpr (OP == FMA_F64) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(d[j]) : "v"(db), "v"(dc));
        if constexpr (OP == ADD_F64) asm volatile("v_add_f64 %0, %0, %1" : "+v"(d[j]) : "v"(db), "v"(dc));
        if constexpr (OP == MUL_F64) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(d[j]) : "v"(db), "v"(dc));
        if constexpr (OP == CMP_LT_F64) asm volatile("v_cmp_lt_f64 vcc, %1, %2" : "=v"(a[j]) : "v"(d[j]), "v"(db) : "vcc");
        if constexpr (OP == ADD_U32) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == XOR_B32) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == AND_B32) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == LSHLREV_B32) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == ALIGNBIT_B32) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == PERM_B32) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == ADD3_U32) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == XAD_U32) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == LSHL_OR_B32) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == BFE_U32) asm volatile("v_bfe_u32 %0, %0, 3, 5" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == MUL_LO_U32) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == MOV_B32) asm volatile("v_mov_b32 %0, %1" : "=v"(a[j]) : "v"(u[j]));
        if constexpr (OP == CNDMASK_B32) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(u[j]) : "v"(u[(j + 1) & 7]) : "vcc");
        if constexpr (OP == CMP_LT_F32) asm volatile("v_cmp_lt_f32 vcc, %1, %2" : "=v"(a[j]) : "v"(a[j]), "v"(b) : "vcc");
        if constexpr (OP == CMP_LT_U32_E64) asm volatile("v_cmp_lt_u32 %0, %1, %2" : "=s"(m[j]) : "v"(u[j]), "v"(sel));
        if constexpr (OP == CNDMASK_E64_SGPR) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "s"(msk));
        if constexpr (OP == CNDMASK_VCC_INDEP) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(a[j]) : "v"(u[j]), "v"(sel) : "vcc");
        if constexpr (OP == CNDMASK_E64_INDEP) asm volatile("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(a[j]) : "v"(u[j]), "v"(sel), "s"(msk));
        if constexpr (OP == CMP_CNDMASK_PAIR)
          asm volatile("v_cmp_lt_u32 vcc, %1, %2\n\tv_cndmask_b32 %0, %1, %2, vcc" : "=v"(a[j]) : "v"(u[j]), "v"(sel) : "vcc");
        if constexpr (OP == CMP_NOP_4CND)
          asm volatile("v_cmp_lt_u32 vcc, %4, %5\n\ts_nop 1\n\tv_cndmask_b32 %0, %4, %5, vcc\n\tv_cndmask_b32 %1, %5, %4, vcc\n\t"
                       "v_cndmask_b32 %2, %4, %5, vcc\n\tv_cndmask_b32 %3, %5, %4, vcc"
                       : "=v"(a[j]), "=v"(a[(j + 1) & 7]), "=v"(a[(j + 2) & 7]), "=v"(a[(j + 3) & 7]) : "v"(u[j]), "v"(sel) : "vcc");
        if constexpr (OP == SMOV_4CND)
          asm volatile("s_mov_b64 vcc, %6\n\tv_cndmask_b32 %0, %4, %5, vcc\n\tv_cndmask_b32 %1, %5, %4, vcc\n\t"
                       "v_cndmask_b32 %2, %4, %5, vcc\n\tv_cndmask_b32 %3, %5, %4, vcc"
                       : "=v"(a[j]), "=v"(a[(j + 1) & 7]), "=v"(a[(j + 2) & 7]), "=v"(a[(j + 3) & 7]) : "v"(u[j]), "v"(sel), "s"(msk) : "vcc");
        if constexpr (OP == CMP_ONCE_CND) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(a[j]) : "v"(u[j]), "v"(sel));
        if constexpr (OP == CMP_E64_4CND_E64)
          asm volatile("v_cmp_lt_u32_e64 %6, %4, %5\n\ts_nop 1\n\tv_cndmask_b32_e64 %0, %4, %5, %6\n\tv_cndmask_b32_e64 %1, %5, %4, %6\n\t"
                       "v_cndmask_b32_e64 %2, %4, %5, %6\n\tv_cndmask_b32_e64 %3, %5, %4, %6"
                       : "=v"(a[j]), "=v"(a[(j + 1) & 7]), "=v"(a[(j + 2) & 7]), "=v"(a[(j + 3) & 7]) : "v"(u[j]), "v"(sel), "s"(m[j]));
        if constexpr (OP == MAX_I32) asm volatile("v_max_i32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]));
        if constexpr (OP == MIN_U32) asm volatile("v_min_u32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]));
        if constexpr (OP == MAX3_I32) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == MIN3_U32) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == SUB_U32) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]));
        if constexpr (OP == OR_B32) asm volatile("v_or_b32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]));
        if constexpr (OP == LSHRREV_B32) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(u[j]));
        if constexpr (OP == OR3_B32) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == AND_OR_B32) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == BFI_B32) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(u[j]) : "v"(u[(j + 1) & 7]), "v"(sel));
        if constexpr (OP == MUL_U32_U24) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]));
        if constexpr (OP == SUBREV_U32) asm volatile("v_subrev_u32 %0, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]));
        if constexpr (OP == NOT_B32) asm volatile("v_not_b32 %0, %0" : "+v"(u[j]));
        if constexpr (OP == ADD_CO_U32) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]) : "vcc");
        if constexpr (OP == LSHL_ADD_U32) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]));
        if constexpr (OP == CMP_EQ_U32_E32) asm volatile("v_cmp_eq_u32 vcc, %0, %1" : "+v"(u[j]) : "v"(u[(j + 1) & 7]) : "vcc");
      }
    }
  }
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; j++) s += a[j] + (float)d[j] + (float)u[j] + (float)m[j];
  out[blockIdx.x * 64 + threadIdx.x] = s;
  const unsigned long long c1 = clock64(), r1 = wall_clock64();
  if (threadIdx.x == 0) {  // this wave's shader-clock cycles and 100 MHz real-time ticks
    clk[2 * blockIdx.x] = c1 - c0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

struct Res { double ms, cycles, mhz; };
template <int OP>
static Res run(float* out, unsigned long long* clk, int blocks, int trips) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  stream_kernel<OP><<<blocks, 64>>>(out, clk, 1);  // warm
  CHECK(hipGetLastError());
  CHECK(hipEventRecord(e0));
  stream_kernel<OP><<<blocks, 64>>>(out, clk, trips);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  std::vector<unsigned long long> h(2 * (size_t)blocks);
  CHECK(hipMemcpy(h.data(), clk, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
  double cyc = 0, ticks = 0;
  for (int b = 0; b < blocks; b++) { cyc += (double)h[2 * b]; ticks += (double)h[2 * b + 1]; }
  return {ms, cyc / blocks, ticks > 0 ? cyc / ticks * 100.0 : 0.0};
}

static Res (*const kRun[N_OPS])(float*, unsigned long long*, int, int) = {run<FMA_F32>, run<FMAC_F32>, run<ADD_F32>, run<MUL_F32>, run<MAX_F32>, run<MAX3_F32>, run<MED3_F32>, run<PK_FMA_F32>, run<PK_ADD_F32>, run<PK_MUL_F32>, run<FMA_MIX_F32>, run<CVT_UBYTE0>, run<CVT_F32_U32>, run<CVT_F64_U32>, run<CVT_F32_F64>, run<FMA_F64>, run<ADD_F64>, run<MUL_F64>, run<CMP_LT_F64>, run<ADD_U32>, run<XOR_B32>, run<AND_B32>, run<LSHLREV_B32>, run<ALIGNBIT_B32>, run<PERM_B32>, run<ADD3_U32>, run<XAD_U32>, run<LSHL_OR_B32>, run<BFE_U32>, run<MUL_LO_U32>, run<MOV_B32>, run<CNDMASK_B32>, run<CMP_LT_F32>, run<CMP_LT_U32_E64>, run<CNDMASK_E64_SGPR>, run<CNDMASK_VCC_INDEP>, run<CNDMASK_E64_INDEP>, run<CMP_CNDMASK_PAIR>, run<CMP_NOP_4CND>, run<SMOV_4CND>, run<CMP_ONCE_CND>, run<CMP_E64_4CND_E64>, run<MAX_I32>, run<MIN_U32>, run<MAX3_I32>, run<MIN3_U32>, run<SUB_U32>, run<OR_B32>, run<LSHRREV_B32>, run<OR3_B32>, run<AND_OR_B32>, run<BFI_B32>, run<MUL_U32_U24>, run<SUBREV_U32>, run<NOT_B32>, run<ADD_CO_U32>, run<LSHL_ADD_U32>, run<CMP_EQ_U32_E32>};

int main(int argc, char** argv) {
  const double mhz = argc > 1 ? std::atof(argv[1]) : 2400.0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int simds = p.multiProcessorCount * 4;
  float* out = nullptr;
  unsigned long long* clk = nullptr;
  const int trips = argc > 2 ? std::atoi(argv[2]) : 20000;
  CHECK(hipMalloc(&out, sizeof(float) * 64 * simds * 8));
  CHECK(hipMalloc(&clk, sizeof(unsigned long long) * 2 * simds * 8));
  std::printf("{\"device\": \"%s\", \"cus\": %d, \"clock_mhz_assumed\": %.0f, \"instructions_per_wave\": %d, \"rates\": {",
              p.gcnArchName, p.multiProcessorCount, mhz, trips * kRounds * 8);
  for (int op = 0; op < N_OPS; op++) {
    std::printf("%s\"%s\": {", op ? ", " : "", kNames[op]);
    for (int w : {2, 4, 8}) {
      const int blocks = simds * w;  // one-wave blocks: w waves per SIMD once every SIMD holds w
      const Res r = kRun[op](out, clk, blocks, trips);
      // SIMD cycles per wave-instruction: a wave's own shader-clock cycles over the stream / (its instructions / the
      // waves sharing its SIMD); and the same from the wall time at the assumed clock
      const double n = (double)trips * kRounds * 8;
      std::printf("%s\"waves_per_simd_%d\": {\"ms\": %.3f, \"clock_mhz\": %.0f, \"simd_cycles_per_instr\": %.3f, "
                  "\"simd_cycles_per_instr_wall\": %.3f}", w == 2 ? "" : ", ", w, r.ms, r.mhz, r.cycles / (n * w),
                  r.ms * 1e-3 * mhz * 1e6 / (n * w));
    }
    std::printf("}");
  }
  std::printf("}}\n");
  CHECK(hipFree(out));
  CHECK(hipFree(clk));
  return 0;
}
