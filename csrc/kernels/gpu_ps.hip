// Kernels of the GPU-resident parameter store (async-PS mode with the variables in GPU memory;
// SURVEY.md §2.4 (2), the "GPU-PS variant" of the reference's ps task, main.py:66-70, whose
// variables TF's replica_device_setter places on /job:ps, worker.py:24-32).
//
// The store is ONE uncached (MTYPE UC) allocation on the owning GPU: the flat f32 parameters
// followed by a control block of 64-bit words (global_step, initialised flag).  Workers on
// other GPUs map it over IPC, so every access below is a direct xGMI read / write of the
// owner's HBM; workers on the owner's GPU access it locally.  UC accesses bypass every GPU
// cache: a pull always sees the latest applied values, an apply lands in memory without any
// cache write-back, and no fence is needed between processes.
//
//   gps_pull_kernel   local replica <- store              (worker.py:81-85 sync_op)
//   gps_apply_kernel  store -= lr * local gradient        (worker.py:79 ApplyGradientDescent:
//                     use_locking=False -> plain read-modify-write, lock-free / Hogwild like
//                     TF's default; use_locking=True -> one f32 atomic add per element)
//   gps_fetch_add     store.global_step += delta, old value returned (worker.py:32,141)
#include "common.h"

#include <stdexcept>

namespace dtfx {
namespace gps {

__global__ __launch_bounds__(256) void gps_pull_kernel(float* __restrict__ dst,
                                                       const float* __restrict__ src,
                                                       long long n) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i + 3 < n) {
    *reinterpret_cast<float4*>(dst + i) = *reinterpret_cast<const float4*>(src + i);
  } else {
    for (long long k = i; k < n; ++k) dst[k] = src[k];
  }
}

template <bool LOCKING>
__global__ __launch_bounds__(256) void gps_apply_kernel(float* __restrict__ p,
                                                        const float* __restrict__ g, float lr,
                                                        long long n) {
  const long long i = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
  if (LOCKING) {
    for (long long k = i; k < i + 4 && k < n; ++k)
      __hip_atomic_fetch_add(p + k, -lr * g[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else if (i + 3 < n) {
    const float4 gv = *reinterpret_cast<const float4*>(g + i);
    float4 pv = *reinterpret_cast<const float4*>(p + i);
    pv.x -= lr * gv.x;
    pv.y -= lr * gv.y;
    pv.z -= lr * gv.z;
    pv.w -= lr * gv.w;
    *reinterpret_cast<float4*>(p + i) = pv;
  } else {
    for (long long k = i; k < n; ++k) p[k] -= lr * g[k];
  }
}

// out[0] = old counter value; out[1 ..] = `nextra` f32 words copied from `extra` (the
// worker's loss / accuracy record of the step), so one read-back serves both
__global__ void gps_fetch_add_kernel(unsigned long long* ctr, long long delta,
                                     unsigned long long* out, const float* extra, int nextra) {
  if (threadIdx.x == 0)
    *out = __hip_atomic_fetch_add(ctr, (unsigned long long)delta, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_SYSTEM);
  if ((int)threadIdx.x < nextra)
    reinterpret_cast<float*>(out + 1)[threadIdx.x] = extra[threadIdx.x];
}

}  // namespace gps

void gps_pull_launch(float* dst, const float* src, long long n, hipStream_t s) {
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15)
    throw std::runtime_error("gpu_ps: buffers must be 16-byte aligned");
  const long long blocks = (n + 1023) / 1024;
  hipLaunchKernelGGL(gps::gps_pull_kernel, dim3((unsigned)blocks), dim3(256), 0, s, dst, src, n);
  DTFX_HIP_CHECK(hipGetLastError());
}

void gps_apply_launch(float* p, const float* g, float lr, long long n, bool locking,
                      hipStream_t s) {
  if ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g)) & 15)
    throw std::runtime_error("gpu_ps: buffers must be 16-byte aligned");
  const long long blocks = (n + 1023) / 1024;
  if (locking)
    hipLaunchKernelGGL(gps::gps_apply_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, p, g,
                       lr, n);
  else
    hipLaunchKernelGGL(gps::gps_apply_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, p,
                       g, lr, n);
  DTFX_HIP_CHECK(hipGetLastError());
}

void gps_fetch_add_launch(unsigned long long* ctr, long long delta, unsigned long long* out,
                          const float* extra, int nextra, hipStream_t s) {
  if (nextra < 0 || nextra > 14) throw std::runtime_error("gpu_ps: at most 14 extra words");
  hipLaunchKernelGGL(gps::gps_fetch_add_kernel, dim3(1), dim3(64), 0, s, ctr, delta, out, extra,
                     nextra);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
