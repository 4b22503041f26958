// Multi-tensor optimizers over ONE flat f32 parameter buffer (every model
// parameter is a view into it), so a single launch updates all tensors.
//
//   sgd      : p -= lr * (g + wd * p)            (GradientDescentOptimizer,
//                                                 worker.py:71, ApplyGradientDescent)
//   momentum : v = mu * v + g' ; p -= lr * (nesterov ? g' + mu * v : v)
//   adam(w)  : bias-corrected Adam; decoupled weight decay when adamw
//   scale    : x *= alpha                        (gradient averaging)
//
// All loops are grid-stride over float4 (dwordx4) with a scalar tail.
// `lr_ptr` / `step_ptr` (optional) let a captured hipGraph pick up a device-side
// learning-rate schedule / step count instead of a frozen kernel argument.
#include "common.h"

#include <stdexcept>

namespace dtfx {

static inline dim3 stream_grid(long long n4) {
  long long b = (n4 + 255) / 256;
  if (b > 2048) b = 2048;
  if (b < 1) b = 1;
  return dim3((unsigned)b);
}

__global__ __launch_bounds__(256) void sgd_kernel(long long n, float* __restrict__ p,
                                                  const float* __restrict__ g, float lr,
                                                  const float* __restrict__ lr_ptr, float wd) {
  const float l = lr_ptr ? *lr_ptr : lr;
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    pv.x -= l * (gv.x + wd * pv.x);
    pv.y -= l * (gv.y + wd * pv.y);
    pv.z -= l * (gv.z + wd * pv.z);
    pv.w -= l * (gv.w + wd * pv.w);
    reinterpret_cast<float4*>(p)[i] = pv;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    p[i] -= l * (g[i] + wd * p[i]);
  }
}

__global__ __launch_bounds__(256) void momentum_kernel(long long n, float* __restrict__ p,
                                                       const float* __restrict__ g,
                                                       float* __restrict__ v, float lr,
                                                       const float* __restrict__ lr_ptr,
                                                       float mu, float wd, int nesterov) {
  const float l = lr_ptr ? *lr_ptr : lr;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const float gg = g[i] + wd * p[i];
    const float vv = mu * v[i] + gg;
    v[i] = vv;
    p[i] -= l * (nesterov ? gg + mu * vv : vv);
  }
}

__global__ __launch_bounds__(256) void adam_kernel(long long n, float* __restrict__ p,
                                                   const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v,
                                                   float lr, const float* __restrict__ lr_ptr,
                                                   float b1, float b2, float eps, float wd,
                                                   int adamw, int step,
                                                   const int* __restrict__ step_ptr) {
  const float l = lr_ptr ? *lr_ptr : lr;
  const int t = (step_ptr ? *step_ptr : step);
  const float bc1 = 1.f - powf(b1, (float)t);
  const float bc2 = 1.f - powf(b2, (float)t);
  const float step_size = l / bc1;
  const float rbc2 = rsqrtf(bc2);
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  auto upd = [&](float& pp, float gg, float& mm, float& vv) {
    if (!adamw) gg += wd * pp;
    mm = b1 * mm + (1.f - b1) * gg;
    vv = b2 * vv + (1.f - b2) * gg * gg;
    const float denom = sqrtf(vv) * rbc2 + eps;
    if (adamw) pp -= l * wd * pp;
    pp -= step_size * mm / denom;
  };
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 mv = reinterpret_cast<float4*>(m)[i];
    float4 vv = reinterpret_cast<float4*>(v)[i];
    upd(pv.x, gv.x, mv.x, vv.x);
    upd(pv.y, gv.y, mv.y, vv.y);
    upd(pv.z, gv.z, mv.z, vv.z);
    upd(pv.w, gv.w, mv.w, vv.w);
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(m)[i] = mv;
    reinterpret_cast<float4*>(v)[i] = vv;
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    upd(p[i], g[i], m[i], v[i]);
  }
}

__global__ __launch_bounds__(256) void scale_kernel(long long n, float* __restrict__ x, float a) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) x[i] *= a;
}

__global__ void counter_add_kernel(int* c, int d) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *c += d;
}

static void check_align(const void* p, const char* what) {
  if (reinterpret_cast<uintptr_t>(p) & 15)
    throw std::runtime_error(std::string(what) + ": buffer must be 16-byte aligned");
}

void sgd_launch(long long n, float* p, const float* g, float lr, const float* lr_ptr, float wd,
                hipStream_t s) {
  if (n <= 0) return;
  check_align(p, "sgd");
  check_align(g, "sgd");
  hipLaunchKernelGGL(sgd_kernel, stream_grid(n >> 2), dim3(256), 0, s, n, p, g, lr, lr_ptr, wd);
  DTFX_HIP_CHECK(hipGetLastError());
}

void momentum_launch(long long n, float* p, const float* g, float* v, float lr,
                     const float* lr_ptr, float mu, float wd, bool nesterov, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(momentum_kernel, stream_grid(n), dim3(256), 0, s, n, p, g, v, lr, lr_ptr, mu,
                     wd, nesterov ? 1 : 0);
  DTFX_HIP_CHECK(hipGetLastError());
}

void adam_launch(long long n, float* p, const float* g, float* m, float* v, float lr,
                 const float* lr_ptr, float b1, float b2, float eps, float wd, bool adamw,
                 int step, const int* step_ptr, hipStream_t s) {
  if (n <= 0) return;
  check_align(p, "adam");
  check_align(g, "adam");
  check_align(m, "adam");
  check_align(v, "adam");
  hipLaunchKernelGGL(adam_kernel, stream_grid(n >> 2), dim3(256), 0, s, n, p, g, m, v, lr, lr_ptr,
                     b1, b2, eps, wd, adamw ? 1 : 0, step, step_ptr);
  DTFX_HIP_CHECK(hipGetLastError());
}

void scale_launch(long long n, float* x, float a, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(scale_kernel, stream_grid(n), dim3(256), 0, s, n, x, a);
  DTFX_HIP_CHECK(hipGetLastError());
}

void counter_add_launch(int* c, int d, hipStream_t s) {
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, s, c, d);
  DTFX_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG init (tf.random_normal_initializer,
// worker.py:51,53; truncated normal / uniform for the extension models).
// mode 0: normal(a = mean, b = std)   1: uniform[a, b)
// mode 2: truncated normal (|z| <= 2, redrawn), mean a, std b
// ---------------------------------------------------------------------------
struct U4 { unsigned x, y, z, w; };

__device__ __forceinline__ U4 philox10(U4 c, unsigned k0, unsigned k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c.x;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c.z;
    const unsigned hi0 = (unsigned)(p0 >> 32), lo0 = (unsigned)p0;
    const unsigned hi1 = (unsigned)(p1 >> 32), lo1 = (unsigned)p1;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float u01(unsigned x) {  // (0, 1]
  return ((float)(x >> 8) + 1.f) * (1.f / 16777216.f);
}

__global__ __launch_bounds__(256) void philox_init_kernel(long long n, float* __restrict__ out,
                                                          unsigned long long seed,
                                                          unsigned long long offset, int mode,
                                                          float a, float b) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  const unsigned k0 = (unsigned)seed, k1 = (unsigned)(seed >> 32);
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i * 4 < n; i += stride) {
    float v[4];
    bool done[4] = {false, false, false, false};
    for (int round = 0; round < (mode == 2 ? 16 : 1); ++round) {
      const unsigned long long ctr = (unsigned long long)i;
      const U4 r = philox10(U4{(unsigned)ctr, (unsigned)(ctr >> 32),
                               (unsigned)offset + (unsigned)round, (unsigned)(offset >> 32)},
                            k0, k1);
      float z[4];
      if (mode == 1) {
        z[0] = u01(r.x); z[1] = u01(r.y); z[2] = u01(r.z); z[3] = u01(r.w);
      } else {
        const float r0 = sqrtf(-2.f * __logf(u01(r.x))), t0 = 6.283185307179586f * u01(r.y);
        const float r1 = sqrtf(-2.f * __logf(u01(r.z))), t1 = 6.283185307179586f * u01(r.w);
        z[0] = r0 * __cosf(t0); z[1] = r0 * __sinf(t0);
        z[2] = r1 * __cosf(t1); z[3] = r1 * __sinf(t1);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (done[e]) continue;
        if (mode == 2 && fabsf(z[e]) > 2.f && round < 15) continue;
        if (mode == 2 && fabsf(z[e]) > 2.f) z[e] = copysignf(2.f, z[e]);
        v[e] = (mode == 1) ? (a + (b - a) * (1.f - z[e])) : (a + b * z[e]);
        done[e] = true;
      }
      if (done[0] && done[1] && done[2] && done[3]) break;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (i * 4 + e < n) out[i * 4 + e] = v[e];
  }
}

void philox_init_launch(long long n, float* out, unsigned long long seed,
                        unsigned long long offset, int mode, float a, float b, hipStream_t s) {
  if (n <= 0) return;
  if (mode < 0 || mode > 2) throw std::runtime_error("philox_init: mode must be 0, 1 or 2");
  hipLaunchKernelGGL(philox_init_kernel, stream_grid((n + 3) >> 2), dim3(256), 0, s, n, out, seed,
                     offset, mode, a, b);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
