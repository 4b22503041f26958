// Shared device helpers for the gfx950 (CDNA4) kernels of this framework.
//
// Everything here is written for a 64-lane wavefront and the f32-input MFMA
// (`v_mfma_f32_16x16x4_f32`): exact f32 products, f32 accumulate.  The
// reference (TF 1.x) computes its MNIST MLP in f32 (worker.py:47-66), so the
// flagship path keeps f32 numerics end to end.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dtfx {

constexpr int kWave = 64;

typedef float f32x4 __attribute__((ext_vector_type(4)));

// 16x16x4 f32 MFMA.  Lane l supplies A[i = l&15][k = l>>4] and
// B[k = l>>4][j = l&15]; the 4-register accumulator holds
// C[row = (l>>4)*4 + r][col = l&15] for r = 0..3.
__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sigmoidf_(float z) {
  // Saturating form: exp of a non-positive argument never overflows.
  if (z >= 0.f) {
    float e = __expf(-z);
    return 1.f / (1.f + e);
  }
  float e = __expf(z);
  return e / (1.f + e);
}

// DPP wave reductions (VALU lane moves, no LDS round trip as __shfl_xor's
// ds_bpermute needs): quad_perm xor1/xor2, row_ror 4/8 -> every lane holds its
// 16-lane row sum; row_bcast15/31 fold rows into lane 63; readlane -> SGPR.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);        // quad_perm(1,0,3,2)
  v += dpp_f<0x4E>(v);        // quad_perm(2,3,0,1)
  v += dpp_f<0x124>(v);       // row_ror:4
  v += dpp_f<0x128>(v);       // row_ror:8
  v += dpp_f<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
  return v;
}

__device__ __forceinline__ int lane_id() { return threadIdx.x & (kWave - 1); }

// Diagnostic stamps (trace builds only): 100 MHz constant-rate wall clock,
// comparable across CUs/XCDs.  STAMP waits for this wave's outstanding memory
// ops first, so each stamp marks "everything issued before has landed".
__device__ __forceinline__ void trace_stamp(unsigned long long* tr, int slot) {
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  const unsigned long long t = __builtin_amdgcn_s_memrealtime();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) tr[slot] = t;
}

// Bijective XCD-aware remap of a 1-D block id (cdna_hip_programming.md §5,
// "XCD swizzle must be bijective"): blocks that the dispatcher deals to the
// same XCD (id % 8 equal) get a contiguous range of logical tile ids, so
// neighbouring tiles share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  constexpr int kXcd = 8;
  if (nwg <= kXcd) return orig;
  const int q = nwg / kXcd, r = nwg % kXcd;
  const int xcd = orig % kXcd, pos = orig / kXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

}  // namespace dtfx

#define DTFX_HIP_CHECK(expr)                                                   \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    if (_e != hipSuccess) {                                                    \
      throw std::runtime_error(std::string("HIP error ") +                    \
                               hipGetErrorString(_e) + " at " + __FILE__ +    \
                               ":" + std::to_string(__LINE__));               \
    }                                                                          \
  } while (0)
