// Vectorised elementwise kernels for the generic layer path.
//
//   act_bwd : dz = dy * act'(s)   s = saved forward output (sigmoid, relu) or
//             pre-activation (gelu), the TF SigmoidGrad/ReluGrad ops
//   act_fwd : y = act(x)          standalone activation (when not fused)
// float4 grid-stride loops; scalar tail.
#include "common.h"

namespace dtfx {

__device__ __forceinline__ float gelu_t(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}
__device__ __forceinline__ float gelu_tg(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float th = tanhf(k0 * (x + k1 * x * x * x));
  return 0.5f * (1.f + th) + 0.5f * x * (1.f - th * th) * k0 * (1.f + 3.f * k1 * x * x);
}

__device__ __forceinline__ float actb(int act, float dy, float s) {
  if (act == 1) return dy * s * (1.f - s);
  if (act == 2) return s > 0.f ? dy : 0.f;
  if (act == 3) return dy * gelu_tg(s);
  return dy;
}
__device__ __forceinline__ float actf(int act, float x) {
  if (act == 1) return sigmoidf_(x);
  if (act == 2) return fmaxf(x, 0.f);
  if (act == 3) return gelu_t(x);
  return x;
}

__global__ __launch_bounds__(256) void act_bwd_kernel(long long n, int act,
                                                      const float* __restrict__ dy,
                                                      const float* __restrict__ s,
                                                      float* __restrict__ dz) {
  const long long n4 = n >> 2, stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(dy)[i];
    const float4 b = reinterpret_cast<const float4*>(s)[i];
    reinterpret_cast<float4*>(dz)[i] =
        make_float4(actb(act, a.x, b.x), actb(act, a.y, b.y), actb(act, a.z, b.z), actb(act, a.w, b.w));
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    dz[i] = actb(act, dy[i], s[i]);
  }
}

__global__ __launch_bounds__(256) void act_fwd_kernel(long long n, int act,
                                                      const float* __restrict__ x,
                                                      float* __restrict__ y) {
  const long long n4 = n >> 2, stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 a = reinterpret_cast<const float4*>(x)[i];
    reinterpret_cast<float4*>(y)[i] = make_float4(actf(act, a.x), actf(act, a.y), actf(act, a.z), actf(act, a.w));
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    y[i] = actf(act, x[i]);
  }
}

static dim3 ew_grid(long long n) {
  long long b = ((n >> 2) + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

void act_bwd_launch(long long n, int act, const float* dy, const float* s, float* dz,
                    hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(act_bwd_kernel, ew_grid(n), dim3(256), 0, st, n, act, dy, s, dz);
  DTFX_HIP_CHECK(hipGetLastError());
}

void act_fwd_launch(long long n, int act, const float* x, float* y, hipStream_t st) {
  if (n <= 0) return;
  hipLaunchKernelGGL(act_fwd_kernel, ew_grid(n), dim3(256), 0, st, n, act, x, y);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
