// lds_probe.hip -- DIAGNOSTIC ONLY (tools/gather_lds_wait.py): a kernel with the footprint of RCCL's
// all-gather kernel on gfx950 -- ncclDevKernel_Generic_{1,2,4} in /opt/rocm/lib/librccl.so.1's gfx950 code object:
// 37,664 B of LDS per block, 248-256 VGPRs per lane, blocks of up to 512 threads (llvm-readelf --notes) -- enqueued on
// the gather's stream behind frames in flight, to time how long a collective's kernel waits for a CU that the
// persistent render blocks (16 per CU, ~10 KB of LDS and 120 VGPRs each) would have to release.  Not part of librp.
#include <hip/hip_runtime.h>

extern "C" {

__global__ void __launch_bounds__(64) probe_stamp_kernel(unsigned long long* out) {
  if (threadIdx.x == 0) out[0] = __builtin_amdgcn_s_memrealtime();
}

__global__ void __launch_bounds__(512) probe_rccl_sized_kernel(unsigned long long* out) {
  extern __shared__ unsigned int lds[];
  asm volatile("v_mov_b32 v255, 0" ::: "v255");  // 256 VGPRs per lane, as ncclDevKernel_Generic
  if (threadIdx.x == 0) out[1 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = threadIdx.x;
  __syncthreads();
  if (lds[(threadIdx.x + 1) % blockDim.x] == 0xFFFFFFFFu) out[0] = 0;  // never: keeps the LDS use
}

// out: 1 + blocks words (100 MHz real-time ticks): [0] when the stream reached the probe, [1 + b] block b's start.
int lds_probe_launch(unsigned long long* out, int blocks, int threads, int lds_bytes, void* stream) {
  hipLaunchKernelGGL(probe_stamp_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, out);
  hipLaunchKernelGGL(probe_rccl_sized_kernel, dim3(blocks), dim3(threads), (size_t)lds_bytes, (hipStream_t)stream, out);
  return (int)hipGetLastError();
}

}
