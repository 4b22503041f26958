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
  // Saturating, branch-free: exp of a non-positive argument never overflows;
  // v_rcp_f32 (1 ulp) instead of an IEEE division sequence.
  const float e = __expf(-fabsf(z));
  const float r = __builtin_amdgcn_rcpf(1.f + e);
  return z >= 0.f ? r : e * r;
}

// DPP wave reductions (VALU lane moves, no LDS round trip as __shfl_xor's
// ds_bpermute needs): quad_perm xor1/xor2, row_ror 4/8 -> every lane holds its
// 16-lane row sum; row_bcast15/31 fold rows into lane 63; readlane -> SGPR.
template <int CTRL, int ROW_MASK = 0xF>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}

// N independent wave sums, interleaved step by step so each DPP op's source
// was written N instructions earlier (the VALU->DPP wait states are filled by
// the other reductions, not s_nop).  Within a 16-lane row: quad_perm/row_ror
// adds with old=0 (the identity of +), which the DPP combiner folds into
// v_add_f32_dpp.  Across rows: gfx950 v_permlane16_swap / v_permlane32_swap,
// so every lane ends with the total in a VGPR (no row_bcast masks, no readlane).
template <int N>
__device__ __forceinline__ void wave_sum_n(float (&v)[N]) {
#define DTFX_STEP(CTRL)                                                                    \
  _Pragma("unroll") for (int i = 0; i < N; ++i) v[i] += __int_as_float(                     \
      __builtin_amdgcn_update_dpp(0, __float_as_int(v[i]), CTRL, 0xF, 0xF, false));
  DTFX_STEP(0xB1)
  DTFX_STEP(0x4E)
  DTFX_STEP(0x124)
  DTFX_STEP(0x128)
#undef DTFX_STEP
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int x = __float_as_int(v[i]);
    auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    v[i] = __int_as_float(r[0]) + __int_as_float(r[1]);
  }
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int x = __float_as_int(v[i]);
    auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    v[i] = __int_as_float(r[0]) + __int_as_float(r[1]);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
  float a[1] = {v};
  wave_sum_n(a);
  return a[0];
}

__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }

// tanh(u) = 1 - 2 / (1 + e^{2u}): one v_exp_f32 + one v_rcp_f32 (libm tanhf is a long
// branchy sequence, and GEMM epilogues evaluate it per output element).  Saturates
// correctly (e^{2u} -> inf gives 1, -> 0 gives -1); absolute error ~1e-7.
__device__ __forceinline__ float fast_tanh(float u) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * u));
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
