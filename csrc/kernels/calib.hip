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

void calib_launch(int mode, int grid, int block, const int* ctr, const float* data, float* out,
                  hipStream_t s) {
  hipLaunchKernelGGL(calib_kernel, dim3(grid), dim3(block), 0, s, mode, ctr, data, out);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
