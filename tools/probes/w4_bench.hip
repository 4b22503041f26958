// Main-loop probe of the 4-wave 256x256 bf16 GEMM tile (gemm_w4_kernel, cfg 7): the same
// staging / fragment primitives (csrc/kernels/gemm_bf16_common.h) in schedule variants, timed
// at two depths K so the per-K-tile cost separates from the fixed per-tile cost.
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc/kernels tools/probes/w4_bench.hip -o /tmp/w4_bench
//   /tmp/w4_bench            (prints one line per variant and K)
//
// Variants: 0 = cfg 7 as built (two 64-deep stages, stage at iteration start, one barrier);
// 1 = no staging inside the loop (compute + barrier only: the LDS-read + MFMA ceiling);
// 2 = four 32-deep stages, three tiles in flight (counted vmcnt).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gemm_bf16_common.h"

using namespace dtfx;
using namespace dtfx::gb;

template <int V>
__global__ __launch_bounds__(256, 1) void w4_probe(int M, int N, int K, const unsigned short* __restrict__ A,
                                                   int lda, const unsigned short* __restrict__ B, int ldb,
                                                   float* __restrict__ out) {
  constexpr int HB = 16384;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles_n = (N + 255) / 256, tiles_m = (M + 255) / 256;
  const int bid0 = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int GM = 4, group = GM * tiles_n, fm = (bid0 / group) * GM;
  const int gm = min(tiles_m - fm, GM), r = bid0 % group;
  const int tm = fm + r % gm, tn = r / gm;
  const int m0 = tm * 256, n0 = tn * 256;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const __amdgpu_buffer_rsrc_t rA = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, 0x7fffffff, 0x00020000);
  const __amdgpu_buffer_rsrc_t rB = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, 0x7fffffff, 0x00020000);
  if constexpr (V == 0 || V == 1) {
    int va[2][4], vb[2][4];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int blk = i * 4 + wave, row = blk * 8 + (lane >> 3), c = (lane & 7) ^ swz_kc(row);
        va[h][i] = (min(m0 + h * 128 + row, M - 1) * lda + c * 8) * 2;
        vb[h][i] = (min(n0 + h * 128 + row, N - 1) * ldb + c * 8) * 2;
      }
    auto stage = [&](int buf, int kt) {
      const int so = kt * BK * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rA, (lds_void*)(smem + (buf * 4 + h) * HB + (i * 4 + wave) * 1024), 16, va[h][i], so, 0, 0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rB, (lds_void*)(smem + (buf * 4 + 2 + h) * HB + (i * 4 + wave) * 1024), 16, vb[h][i], so, 0, 0);
        }
    };
    const int nk = K / BK;
    stage(0, 0);
    if (V == 1) stage(1, 0);
    vm_barrier<0>();
    for (int kt = 0; kt < nk; ++kt) {
      const int b = kt & 1;
      if (V == 0 && kt + 1 < nk) stage(b ^ 1, kt + 1);
      const char* At = smem + (b * 4 + wm) * HB;
      const char* Bt = smem + (b * 4 + 2 + wn) * HB;
      bf16x8 af[2][8], bfr[2][8];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int j = 0; j < 8; ++j) bfr[kk][j] = frag<true, 128>(Bt, j * 16, kk, lane);
#pragma unroll
        for (int i = 0; i < 8; ++i) af[kk][i] = frag<true, 128>(At, i * 16, kk, lane);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[0][i], bfr[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[1][i], bfr[1][j], acc[i][j], 0, 0, 0);
        }
      vm_barrier<0>();
    }
  } else if constexpr (V == 3) {
    // V == 3: V2's four 32-deep stages, but tile kt+1 is retired one iteration earlier (two
    // tiles in flight, vmcnt(8)) so its fragments are read from LDS during tile kt's MFMAs
    // (register double buffer): no MFMA ever waits on an LDS read after the barrier
    constexpr int ST = 32768, HALF = 8192;
    int va[2][2], vb[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int blk = i * 4 + wave, row = blk * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
        va[h][i] = (min(m0 + h * 128 + row, M - 1) * lda + c * 8) * 2;
        vb[h][i] = (min(n0 + h * 128 + row, N - 1) * ldb + c * 8) * 2;
      }
    auto stage = [&](int buf, int kt) {
      const int so = kt * 32 * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rA, (lds_void*)(smem + buf * ST + h * HALF + (i * 4 + wave) * 1024), 16, va[h][i], so, 0, 0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rB, (lds_void*)(smem + buf * ST + 2 * HALF + h * HALF + (i * 4 + wave) * 1024), 16, vb[h][i],
              so, 0, 0);
        }
    };
    auto frag32 = [&](const char* img, int o0) -> bf16x8 {
      const int row = o0 + (lane & 15), c = lane >> 4;
      return *(const bf16x8*)(img + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
    };
    const int nk = K / 32;
    stage(0, 0);
    if (nk > 1) stage(1, 1);
    if (nk > 2) stage(2, 2);
    // tiles 0 and 1 visible (tile 2 may stay in flight)
    if (nk > 2) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    bf16x8 af[2][8], bfr[2][8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bfr[0][j] = frag32(smem + 2 * HALF + wn * HALF, j * 16);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[0][i] = frag32(smem + wm * HALF, i * 16);
    for (int kt = 0; kt < nk; kt += 2) {
      // two tiles per trip so the register buffers stay literal (p = 0 computes, 1 is filled)
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int t = kt + p;  // (nk = K / 32 is even: K % 64 == 0)
        if (t + 3 < nk) stage((t + 3) & 3, t + 3);
        if (t + 1 < nk) {
          const char* At = smem + ((t + 1) & 3) * ST + wm * HALF;
          const char* Bt = smem + ((t + 1) & 3) * ST + 2 * HALF + wn * HALF;
#pragma unroll
          for (int j = 0; j < 8; ++j) bfr[p ^ 1][j] = frag32(Bt, j * 16);
#pragma unroll
          for (int i = 0; i < 8; ++i) af[p ^ 1][i] = frag32(At, i * 16);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[p][i], bfr[p][j], acc[i][j], 0, 0, 0);
        // retire tile t+2 (t+3 may stay in flight); the barrier also orders every wave's
        // reads of tile t+1 before tile t+4 overwrites buffer (t+4)&3 = t&3... (t's buffer
        // is restaged at t+1 as tile t+4: its fragments were read in iteration t-1)
        if (t + 3 < nk) asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
    }
  } else {
    // V == 2: BK = 32 tiles (A and B 256 x 32 each, 64-B rows, chunk c of row r at
    // c ^ ((r >> 2) & 3): the 16 rows of a ds_read_b128 group cover all 16 bank slots), four
    // stages of 32 KB, tiles kt+1..kt+3 in flight while kt computes
    constexpr int ST = 32768, HALF = 8192;  // stage bytes, 128-row half image bytes
    int va[2][2], vb[2][2];
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int blk = i * 4 + wave, row = blk * 16 + (lane >> 2), c = (lane & 3) ^ ((row >> 2) & 3);
        va[h][i] = (min(m0 + h * 128 + row, M - 1) * lda + c * 8) * 2;
        vb[h][i] = (min(n0 + h * 128 + row, N - 1) * ldb + c * 8) * 2;
      }
    auto stage = [&](int buf, int kt) {
      const int so = kt * 32 * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rA, (lds_void*)(smem + buf * ST + h * HALF + (i * 4 + wave) * 1024), 16, va[h][i], so, 0, 0);
          __builtin_amdgcn_raw_ptr_buffer_load_lds(
              rB, (lds_void*)(smem + buf * ST + 2 * HALF + h * HALF + (i * 4 + wave) * 1024), 16, vb[h][i],
              so, 0, 0);
        }
    };
    auto frag32 = [&](const char* img, int o0) -> bf16x8 {
      const int row = o0 + (lane & 15), c = lane >> 4;
      return *(const bf16x8*)(img + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
    };
    const int nk = K / 32;
    stage(0, 0);
    if (nk > 1) stage(1, 1);
    if (nk > 2) stage(2, 2);
    if (nk > 2) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    for (int kt = 0; kt < nk; ++kt) {
      const int b = kt & 3;
      if (kt + 3 < nk) stage((kt + 3) & 3, kt + 3);
      const char* At = smem + b * ST + wm * HALF;
      const char* Bt = smem + b * ST + 2 * HALF + wn * HALF;
      bf16x8 af[8], bfr[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bfr[j] = frag32(Bt, j * 16);
#pragma unroll
      for (int i = 0; i < 8; ++i) af[i] = frag32(At, i * 16);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      // retire tile kt+1: younger tiles (up to 2, 8 loads each) may stay in flight
      if (kt + 3 < nk) asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
      else if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  // keep every accumulator live (no DCE of the MFMAs) without an epilogue
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" ::"a"(acc[i][j]));
  out[blockIdx.x * 256 + threadIdx.x] = acc[0][0][0];
}

template <int V>
static float run(int M, int N, int K, const unsigned short* A, const unsigned short* B, float* out) {
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  hipFuncSetAttribute((const void*)w4_probe<V>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    hipEventRecord(e0);
    for (int it = 0; it < 10; ++it)
      hipLaunchKernelGGL(w4_probe<V>, dim3(tiles), dim3(256), 131072, 0, M, N, K, A, K, B, K, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;
  }
  return best / 10 * 1000.f;  // us
}

int main() {
  const int M = 16384, N = 3072;
  const int Ks[3] = {768, 3072, 6144};
  const size_t na = (size_t)M * 6144, nb = (size_t)N * 6144;
  std::vector<unsigned short> h(na > nb ? na : nb);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned short)(0x3c00 + (rand() & 0xff));  // ~[1, 2)
  unsigned short *A, *B;
  float* out;
  hipMalloc(&A, na * 2);
  hipMalloc(&B, nb * 2);
  hipMalloc(&out, (size_t)4096 * 256 * 4);
  hipMemcpy(A, h.data(), na * 2, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), nb * 2, hipMemcpyHostToDevice);
  for (int k = 0; k < 3; ++k) {
    const int K = Ks[k];
    const double fl = 2.0 * M * N * K;
    float t0 = run<0>(M, N, K, A, B, out), t1 = run<1>(M, N, K, A, B, out), t2 = run<2>(M, N, K, A, B, out);
    float t3 = run<3>(M, N, K, A, B, out);
    printf("{\"M\": %d, \"N\": %d, \"K\": %d, \"us_v0\": %.1f, \"us_v1_noload\": %.1f, \"us_v2_bk32x4\": %.1f, "
           "\"us_v3_bk32_plr\": %.1f, \"tf_v0\": %.0f, \"tf_v1\": %.0f, \"tf_v2\": %.0f, \"tf_v3\": %.0f}\n",
           M, N, K, t0, t1, t2, t3, fl / t0 * 1e-6, fl / t1 * 1e-6, fl / t2 * 1e-6, fl / t3 * 1e-6);
  }
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) printf("error %s\n", hipGetErrorString(err));
  return 0;
}
