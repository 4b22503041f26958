// Generic f32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_16x16x4_f32,
// exact f32, the same numerics class as TF's f32 MatMul used by the
// reference's tf.layers.dense, worker.py:50-53).
//
//   C[M,N] = epilogue( alpha * op(A)[M,K] . op(B)[K,N] )
//   op(A) = A [M][lda]  or  A^T with A stored [K][lda]
//   op(B) = B [K][ldb]  or  B^T with B stored [N][ldb]
//
// Epilogues (fused so the elementwise pass never makes its own HBM trip):
//   + bias[N]                        (dense forward)
//   activation: none / sigmoid / relu / gelu(tanh)
//   * act'(aux[M][N])                (backward through the activation, aux =
//                                     the saved forward OUTPUT for sigmoid/relu,
//                                     the saved PRE-activation for gelu)
//   + beta * C                       (gradient accumulation)
//
// Tiling: 64x64 output tile per 256-thread workgroup (4 waves as 2x2, each a
// 32x32 sub-tile = 2x2 MFMA tiles), BK = 16, LDS tiles stored k-major so the
// MFMA operand reads (16 consecutive m or n per lane group) are conflict-free.
// The next K tile is prefetched into registers while the current one is
// consumed.  Block ids are XCD-remapped so neighbouring tiles share an L2.
#include "common.h"

#include <stdexcept>
#include <string>

namespace dtfx {

enum Act : int { ACT_NONE = 0, ACT_SIGMOID = 1, ACT_RELU = 2, ACT_GELU = 3 };

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  const float th = tanhf(u);
  return 0.5f * (1.f + th) + 0.5f * x * (1.f - th * th) * k0 * (1.f + 3.f * k1 * x * x);
}

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_kernel(
    int M, int N, int K, float alpha, const float* __restrict__ A, int lda,
    const float* __restrict__ Bm, int ldb, float beta, float* __restrict__ Cm, int ldc,
    const float* __restrict__ bias, int act, const float* __restrict__ aux, int ldaux,
    int act_grad) {
  constexpr int BM = 64, BN = 64, BK = 16, PAD = 4;
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int bid = xcd_remap(blockIdx.x, tiles_n * tiles_m);
  const int m0 = (bid / tiles_n) * BM, n0 = (bid % tiles_n) * BN;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int r = lane & 15, q = lane >> 4;
  const int wm = wave >> 1, wn = wave & 1;

  // per-thread staging coordinates
  // A: no-trans -> (m = t/4, k = 4*(t%4)+j) ; trans -> (k = t/16, m = 4*(t%16)+j)
  // B: no-trans -> (k = t/16, n = 4*(t%16)+j) ; trans -> (n = t/4, k = 4*(t%4)+j)
  float ra[4], rb[4];
  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int m, k;
      if (!TA) { m = t >> 2; k = ((t & 3) << 2) + j; }
      else { k = t >> 4; m = ((t & 15) << 2) + j; }
      const int gm = m0 + m, gk = k0 + k;
      ra[j] = (gm < M && gk < K) ? (TA ? A[(size_t)gk * lda + gm] : A[(size_t)gm * lda + gk]) : 0.f;
      int n;
      if (!TB) { k = t >> 4; n = ((t & 15) << 2) + j; }
      else { n = t >> 2; k = ((t & 3) << 2) + j; }
      const int gn = n0 + n, gk2 = k0 + k;
      rb[j] = (gn < N && gk2 < K) ? (TB ? Bm[(size_t)gn * ldb + gk2] : Bm[(size_t)gk2 * ldb + gn]) : 0.f;
    }
  };
  auto store_tiles = [&]() {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!TA) As[((t & 3) << 2) + j][t >> 2] = ra[j];
      else As[t >> 4][((t & 15) << 2) + j] = ra[j];
      if (!TB) Bs[t >> 4][((t & 15) << 2) + j] = rb[j];
      else Bs[((t & 3) << 2) + j][t >> 2] = rb[j];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0, 0, 0, 0};

  load_tiles(0);
  for (int k0 = 0; k0 < K; k0 += BK) {
    __syncthreads();
    store_tiles();
    __syncthreads();
    if (k0 + BK < K) load_tiles(k0 + BK);
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[s * 4 + q][wm * 32 + i * 16 + r];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[s * 4 + q][wn * 32 + j * 16 + r];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16x16x4(a[i], b[j], acc[i][j]);
    }
  }

#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int gm = m0 + wm * 32 + i * 16 + q * 4 + e;
        const int gn = n0 + wn * 32 + j * 16 + r;
        if (gm < M && gn < N) {
          float v = alpha * acc[i][j][e];
          if (bias) v += bias[gn];
          if (act_grad) {
            const float y = aux[(size_t)gm * ldaux + gn];
            if (act == ACT_SIGMOID) v *= y * (1.f - y);
            else if (act == ACT_RELU) v = (y > 0.f) ? v : 0.f;
            else if (act == ACT_GELU) v *= gelu_tanh_grad(y);
          } else {
            if (act == ACT_SIGMOID) v = sigmoidf_(v);
            else if (act == ACT_RELU) v = fmaxf(v, 0.f);
            else if (act == ACT_GELU) v = gelu_tanh(v);
          }
          float* cp = Cm + (size_t)gm * ldc + gn;
          if (beta != 0.f) v += beta * *cp;
          *cp = v;
        }
      }
}

void gemm_f32_launch(bool ta, bool tb, int M, int N, int K, float alpha, const float* A,
                     int lda, const float* B, int ldb, float beta, float* C, int ldc,
                     const float* bias, int act, const float* aux, int ldaux, bool act_grad,
                     hipStream_t stream) {
  if (M <= 0 || N <= 0) return;
  if (K <= 0) throw std::runtime_error("gemm_f32: K must be positive");
  if (act_grad && aux == nullptr) throw std::runtime_error("gemm_f32: act_grad needs aux");
  const int tiles = ((M + 63) / 64) * ((N + 63) / 64);
  dim3 grid(tiles), block(256);
#define DTFX_GEMM_CASE(TA_, TB_)                                                         \
  hipLaunchKernelGGL((gemm_f32_kernel<TA_, TB_>), grid, block, 0, stream, M, N, K, alpha, A, \
                     lda, B, ldb, beta, C, ldc, bias, act, aux, ldaux, act_grad ? 1 : 0)
  if (!ta && !tb) DTFX_GEMM_CASE(false, false);
  else if (!ta && tb) DTFX_GEMM_CASE(false, true);
  else if (ta && !tb) DTFX_GEMM_CASE(true, false);
  else DTFX_GEMM_CASE(true, true);
#undef DTFX_GEMM_CASE
  DTFX_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// column sums: out[n] = beta * out[n] + sum_m G[m][n]   (bias gradients)
// 256 threads = 64 columns x 4 row groups; partial sums combined in LDS.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void colsum_kernel(int M, int N, const float* __restrict__ G,
                                                     int ldg, float beta, float* __restrict__ out) {
  __shared__ float part[4][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int n = blockIdx.x * 64 + c;
  float s = 0.f;
  if (n < N)
    for (int m = g; m < M; m += 4) s += G[(size_t)m * ldg + n];
  part[g][c] = s;
  __syncthreads();
  if (g == 0 && n < N) {
    const float v = part[0][c] + part[1][c] + part[2][c] + part[3][c];
    out[n] = (beta != 0.f ? beta * out[n] : 0.f) + v;
  }
}

void colsum_launch(int M, int N, const float* G, int ldg, float beta, float* out,
                   hipStream_t stream) {
  if (N <= 0) return;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64), dim3(256), 0, stream, M, N, G, ldg,
                     beta, out);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
