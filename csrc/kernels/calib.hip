// Calibration kernels for launch/boundary measurements (tools/mlp_microbench.py).
#include "common.h"

namespace dtfx {

// mode 0: nothing; 1: read ctr (dependent scalar load); 2: read ctr + one
// dependent load per lane from `data` (the latency chain of a real kernel).
__global__ void calib_kernel(int mode, const int* __restrict__ ctr, const float* __restrict__ data,
                             float* __restrict__ out) {
  if (mode == 0) return;
  const int s = ctr[0];
  if (mode == 1) {
    if (s == -12345) out[0] = 1.f;
    return;
  }
  const float v = data[(size_t)(s & 1023) * 64 + threadIdx.x + blockIdx.x * 64];
  if (v == -12345.f) out[0] = v;
}

// Clock probe: out2[block] = {memtime delta, realtime delta} around a chain of
// `iters` dependent FMAs (shader clock = memtime / (realtime / 100 MHz)).
__global__ void clock_probe_kernel(int iters, unsigned long long* out2, float* sink) {
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  float v = threadIdx.x * 1e-3f;
  for (int i = 0; i < iters; ++i) v = fmaf(v, 0.999f, 1e-4f);
  asm volatile("" ::"v"(v));
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out2[2 * blockIdx.x] = t1 - t0;
    out2[2 * blockIdx.x + 1] = r1 - r0;
  }
  if (v == -1.f) sink[0] = v;
}

void clock_probe_launch(int iters, int grid, unsigned long long* out2, float* sink, hipStream_t s) {
  hipLaunchKernelGGL(clock_probe_kernel, dim3(grid), dim3(64), 0, s, iters, out2, sink);
  DTFX_HIP_CHECK(hipGetLastError());
}

void calib_launch(int mode, int grid, int block, const int* ctr, const float* data, float* out,
                  hipStream_t s) {
  hipLaunchKernelGGL(calib_kernel, dim3(grid), dim3(block), 0, s, mode, ctr, data, out);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
