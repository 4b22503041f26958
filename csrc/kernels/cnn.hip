// CNN (ResNet-50) kernels for gfx950, NHWC bf16 activations viewed as
// [M = N*H*W][C]: BatchNorm (statistics fused into the convolution GEMM
// epilogue, see gemm_bf16.hip; here finalize / apply(+residual +ReLU) /
// backward), 3x3/s2 max-pool fwd/bwd (argmax byte, gather backward: no
// atomics), global average pool fwd/bwd, and mixed-precision momentum SGD.
// North-star config 4 of BASELINE.json (ResNet-50 synthetic ImageNet); the
// reference itself has no convolutional model (worker.py:47-54).
#include "common.h"
#include "bn_common.h"

#include <algorithm>

#include <stdexcept>

namespace dtfx {

typedef short bf16x8 __attribute__((ext_vector_type(8)));

namespace cn {
__device__ __forceinline__ float bf(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ void unpack8(const bf16x8& v, float* f) {
#pragma unroll
  for (int u = 0; u < 8; ++u) f[u] = bf((unsigned short)v[u]);
}
__device__ __forceinline__ bf16x8 pack8(const float* f) {
  bf16x8 v;
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = (short)tobf(f[u]);
  return v;
}
}  // namespace cn
using namespace cn;

// Column reduction of partial rows: out_s[c] += sum_r part_s[r][c] (and the same for q).
// grid (ceil(C / 64), S): 64 channels x 4 row groups per block, one atomic per channel per block.
__global__ __launch_bounds__(256) void colpart_reduce_kernel(int R, int C, const float* __restrict__ ps,
                                                             const float* __restrict__ pq,
                                                             float* __restrict__ os,
                                                             float* __restrict__ oq) {
  __shared__ float red[2][4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  float a = 0.f, b = 0.f;
  if (c < C) {
    // four rows in flight per thread (independent loads, then the adds): the plain loop
    // made one dependent memory round trip per row
    const int step = 4 * gridDim.y;
    int r = blockIdx.y * 4 + rg;
    for (; r + 3 * step < R; r += 4 * step) {
      float va[4], vb[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        va[u] = ps[(size_t)(r + u * step) * C + c];
        if (pq) vb[u] = pq[(size_t)(r + u * step) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a += va[u];
        b += vb[u];
      }
    }
    for (; r < R; r += step) {
      a += ps[(size_t)r * C + c];
      if (pq) b += pq[(size_t)r * C + c];
    }
  }
  red[0][rg][threadIdx.x & 63] = a;
  red[1][rg][threadIdx.x & 63] = b;
  __syncthreads();
  if (rg == 0 && c < C) {
    const int l = threadIdx.x;
    unsafeAtomicAdd(os + c, red[0][0][l] + red[0][1][l] + red[0][2][l] + red[0][3][l]);
    if (pq) unsafeAtomicAdd(oq + c, red[1][0][l] + red[1][1][l] + red[1][2][l] + red[1][3][l]);
  }
}

// mean = s / M, var = q / M - mean^2 (biased, as used for normalisation),
// running stats updated with the unbiased variance (momentum form of tf/keras).
__global__ void bn_finalize_kernel(int C, float inv_m, float unbias, const float* __restrict__ s,
                                   const float* __restrict__ q, float eps, float* __restrict__ mean,
                                   float* __restrict__ rstd, float* __restrict__ run_mean,
                                   float* __restrict__ run_var, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float mu = s[c] * inv_m;
  const float var = fmaxf(q[c] * inv_m - mu * mu, 0.f);
  mean[c] = mu;
  rstd[c] = rsqrtf(var + eps);
  if (run_mean) {
    run_mean[c] = momentum * run_mean[c] + (1.f - momentum) * mu;
    run_var[c] = momentum * run_var[c] + (1.f - momentum) * var * unbias;
  }
}

// y = act((x - mean) * rstd * gamma + beta + residual); 8 channels per thread, computed as
// y = x * sc + sh (+ res) (ReLU), sc = rstd * gamma, sh = beta - mean * sc.
// When the grid stride is a multiple of the channel-group count (every power-of-two C
// up to 2048: 256 % (C / 8) == 0) each thread keeps ONE channel group for its whole
// grid-stride walk, so its 8 coefficients pairs are loaded once (not 32 scalar loads and
// a 64-bit modulo per 16-B chunk), and the walk keeps 4 chunks in flight.
//
// Fused finalize (st.ssum != null, the forward's training-mode path): the batch statistics
// come in as the column sums ssum / ssq of the conv epilogue, every thread forms mean / rstd
// of its own channels exactly as bn_finalize_kernel does, and block 0 stores mean / rstd (for
// the backward) and updates the running statistics -- one launch per BatchNorm instead of
// finalize + apply (ResNet-50: 53 launches of ~5 us per step).
// A second set (st2.ssum != null) normalises the residual with ITS own batch statistics and
// affine (gamma2 / beta2) before the add: a bottleneck's output relu(bn3(c3) + bn_ds(cds)) in
// one pass over c3 and the raw downsample conv output cds -- the normalised shortcut is never
// written and read back (the downsample backward only needs cds and its mean / rstd).
// (BnStats, bn_store_stats, bn_coef: bn_common.h)
// (STATS / RBN are template parameters: as run-time flags the per-element residual branch and
// the coefficient loads ended up inside the streaming loop -- 4x slower)
template <int U, bool STATS, bool RBN>
__global__ __launch_bounds__(256) void bn_apply_kernel(long long M, int C,
                                                       const unsigned short* __restrict__ x,
                                                       const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta,
                                                       const unsigned short* __restrict__ res,
                                                       int relu, unsigned short* __restrict__ y,
                                                       BnStats st, BnStats st2) {
  const int cg = C >> 3;
  const long long n8 = M * cg;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  constexpr bool rbn = RBN;  // residual normalised by its own BN (res: raw conv output)
  if (STATS && blockIdx.x == 0) {
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      float mu, rs;
      bn_coef<STATS>(st, mean, rstd, c, mu, rs);
      bn_store_stats(st, c, mu, rs);
      if (rbn) {
        bn_coef<true>(st2, nullptr, nullptr, c, mu, rs);
        bn_store_stats(st2, c, mu, rs);
      }
    }
  }
  if (stride % cg == 0) {
    const int c0 = (int)(i0 % cg) * 8;
    float sc[8], sh[8], sc2[8], sh2[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u;
      float mu, rs;
      bn_coef<STATS>(st, mean, rstd, c, mu, rs);
      sc[u] = rs * gamma[c];
      sh[u] = beta[c] - mu * sc[u];
      sc2[u] = 1.f;
      sh2[u] = 0.f;
      if (rbn) {
        bn_coef<true>(st2, nullptr, nullptr, c, mu, rs);
        sc2[u] = rs * st2.gamma2[c];
        sh2[u] = st2.beta2[c] - mu * sc2[u];
      }
    }
    for (long long ib = i0; ib < n8; ib += U * stride) {
      bf16x8 xv[U], rv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const long long i = ib + k * stride;
        const long long ic = i < n8 ? i : i0;  // in-bounds dummy for the tail
        xv[k] = __builtin_nontemporal_load((const bf16x8*)x + ic);
        if (res) rv[k] = __builtin_nontemporal_load((const bf16x8*)res + ic);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const long long i = ib + k * stride;
        if (i >= n8) break;
        float v[8], r[8];
        unpack8(xv[k], v);
        if (res) unpack8(rv[k], r);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float o = v[u] * sc[u] + sh[u];
          if (res) o += rbn ? r[u] * sc2[u] + sh2[u] : r[u];
          if (relu) o = fmaxf(o, 0.f);
          v[u] = o;
        }
        __builtin_nontemporal_store(pack8(v), (bf16x8*)y + (i));
      }
    }
    return;
  }
  for (long long i = i0; i < n8; i += stride) {  // general C
    const int c0 = (int)(i % cg) * 8;
    float v[8], r[8];
    unpack8(__builtin_nontemporal_load((const bf16x8*)x + i), v);
    if (res) unpack8(__builtin_nontemporal_load((const bf16x8*)res + i), r);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u;
      float mu, rs;
      bn_coef<STATS>(st, mean, rstd, c, mu, rs);
      float o = (v[u] - mu) * rs * gamma[c] + beta[c];
      if (res && rbn) {
        bn_coef<true>(st2, nullptr, nullptr, c, mu, rs);
        o += (r[u] - mu) * rs * st2.gamma2[c] + st2.beta2[c];
      } else if (res) {
        o += r[u];
      }
      if (relu) o = fmaxf(o, 0.f);
      v[u] = o;
    }
    __builtin_nontemporal_store(pack8(v), (bf16x8*)y + (i));
  }
}

// Per-channel coefficients of the 1x1 kernels' BatchNorm prologue (conv1x1.hip, PRO):
// op = (s0 a + c) + (s1 b + d), coef = [a | b | c | d] f32 [4][C].
// Forward: exactly bn_apply_kernel<STATS>'s terms (a = rstd gamma, c = beta - mean a; residual
// b = 1, d = 0, or its own BN b = rstd2 gamma2, d = beta2 - mean2 b), and the kernel's block-0
// duty (mean / rstd for the backward, running statistics).
__global__ __launch_bounds__(256) void bn_fwd_coef_kernel(int C, BnStats st, BnStats st2,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, int rbn,
                                                          float* __restrict__ coef) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  float mu, rs;
  bn_coef<true>(st, nullptr, nullptr, c, mu, rs);
  bn_store_stats(st, c, mu, rs);
  const float a = rs * gamma[c];
  float b = 1.f, d = 0.f;
  if (rbn) {
    float mu2, rs2;
    bn_coef<true>(st2, nullptr, nullptr, c, mu2, rs2);
    bn_store_stats(st2, c, mu2, rs2);
    b = rs2 * st2.gamma2[c];
    d = st2.beta2[c] - mu2 * b;
  }
  coef[c] = a;
  coef[C + c] = b;
  coef[2 * C + c] = beta[c] - mu * a;
  coef[3 * C + c] = d;
}
// Backward: bn_bwd_apply_kernel's affine form dx = A de + K1 x + K0 (s0 = de, s1 = x).
__global__ __launch_bounds__(256) void bn_bwd_coef_kernel(int C, const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ sum_dy,
                                                          const float* __restrict__ sum_dyxh,
                                                          float inv_m, float* __restrict__ coef) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const float A = gamma[c] * rstd[c], s1 = sum_dy[c] * inv_m, s2 = sum_dyxh[c] * inv_m;
  coef[c] = A;
  coef[C + c] = -A * rstd[c] * s2;
  coef[2 * C + c] = 0.f;
  coef[3 * C + c] = -A * s1 + A * rstd[c] * s2 * mean[c];
}

// Backward reductions: dy_eff = dy * (y > 0 if relu); per block, sums over its rows of
// dy_eff and dy_eff * xhat per channel, reduced in LDS and written as ONE partial row per
// block ([blocks][C], no atomics); colpart_reduce finishes the column sums.
// Each thread owns 8 channels of one channel group and strides over the block's rows.
__global__ __launch_bounds__(256) void bn_bwd_reduce_kernel(
    long long M, int C, int rows_per_block, const unsigned short* __restrict__ dy,
    const unsigned short* __restrict__ yout, const unsigned short* __restrict__ x,
    const float* __restrict__ mean, const float* __restrict__ rstd, int relu,
    float* __restrict__ part_dy, float* __restrict__ part_dyxh) {
  __shared__ float red[2][2048];  // [sum][rr * tpr * 8 + channel-in-pass]
  const int cg = C >> 3;
  const int tpr = min(cg, 256);  // threads per row (channel groups per pass)
  const int rpp = 256 / tpr;     // rows per pass
  const int t = threadIdx.x;
  const int g = t % tpr, rr = t / tpr;
  const long long r0 = (long long)blockIdx.x * rows_per_block;
  const long long r1 = min(M, r0 + rows_per_block);
  for (int base = 0; base < cg; base += tpr) {  // channel groups [base, base + tpr)
    const int gg = base + g;
    float a[8], b[8], mu[8], rs[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) a[u] = b[u] = 0.f;
    if (rr < rpp && gg < cg) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        mu[u] = mean[gg * 8 + u];
        rs[u] = rstd[gg * 8 + u];
      }
      constexpr int U = 4;  // rows in flight per thread
      for (long long rb = r0 + rr; rb < r1; rb += U * rpp) {
        bf16x8 dv[U], xq[U], yq[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
          const long long r = rb + (long long)k * rpp;
          const long long i = (r < r1 ? r : r0 + rr) * cg + gg;  // in-bounds dummy row
          dv[k] = __builtin_nontemporal_load((const bf16x8*)dy + i);
          xq[k] = __builtin_nontemporal_load((const bf16x8*)x + i);
          if (relu) yq[k] = __builtin_nontemporal_load((const bf16x8*)yout + i);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
          if (rb + (long long)k * rpp >= r1) break;
          float d[8], xv[8], yv[8];
          unpack8(dv[k], d);
          unpack8(xq[k], xv);
          if (relu) unpack8(yq[k], yv);
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float de = (relu && yv[u] <= 0.f) ? 0.f : d[u];
            a[u] += de;
            b[u] += de * (xv[u] - mu[u]) * rs[u];
          }
        }
      }
    }
    __syncthreads();
    if (rr < rpp)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        red[0][rr * tpr * 8 + g * 8 + u] = a[u];
        red[1][rr * tpr * 8 + g * 8 + u] = b[u];
      }
    __syncthreads();
    for (int ch = t; ch < tpr * 8; ch += 256) {
      float sa = 0.f, sb = 0.f;
      for (int q = 0; q < rpp; ++q) {
        sa += red[0][q * tpr * 8 + ch];
        sb += red[1][q * tpr * 8 + ch];
      }
      const int c = base * 8 + ch;
      if (c < C) {
        part_dy[(size_t)blockIdx.x * C + c] = sa;
        part_dyxh[(size_t)blockIdx.x * C + c] = sb;
      }
    }
  }
}

// dx = gamma * rstd * (dy_eff - sum_dy / M - xhat * sum_dyxh / M); dres = dy_eff (optional)
// dx = gamma * rstd * (dy_eff - mean(dy_eff) - xhat * mean(dy_eff * xhat))
//    = A * dy_eff + K1 * x + K0 per channel (A = gamma rstd, K1 = -A rstd S2,
//      K0 = -A S1 + A rstd S2 mean; S1, S2 = the two column sums / M); dres = dy_eff.
// Same per-thread channel group / one-pass U-in-flight walk as bn_apply_kernel.
template <int U>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(
    long long M, int C, const unsigned short* __restrict__ dy, const unsigned short* __restrict__ yout,
    const unsigned short* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ gamma,
    const float* __restrict__ sum_dy, const float* __restrict__ sum_dyxh, int relu, float inv_m,
    unsigned short* __restrict__ dx, unsigned short* __restrict__ dres) {
  const int cg = C >> 3;
  const long long n8 = M * cg;
  const long long stride = (long long)gridDim.x * blockDim.x;
  const long long i0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (stride % cg == 0) {
    const int c0 = (int)(i0 % cg) * 8;
    float ka[8], k1[8], k0[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u;
      const float A = gamma[c] * rstd[c], s1 = sum_dy[c] * inv_m, s2 = sum_dyxh[c] * inv_m;
      ka[u] = A;
      k1[u] = -A * rstd[c] * s2;
      k0[u] = -A * s1 + A * rstd[c] * s2 * mean[c];
    }
    for (long long ib = i0; ib < n8; ib += U * stride) {
      bf16x8 dv[U], xv[U], yv[U];
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const long long i = ib + k * stride;
        const long long ic = i < n8 ? i : i0;
        dv[k] = __builtin_nontemporal_load((const bf16x8*)dy + ic);
        xv[k] = __builtin_nontemporal_load((const bf16x8*)x + ic);
        if (relu) yv[k] = __builtin_nontemporal_load((const bf16x8*)yout + ic);
      }
#pragma unroll
      for (int k = 0; k < U; ++k) {
        const long long i = ib + k * stride;
        if (i >= n8) break;
        float d[8], xf[8], yf[8], o[8];
        unpack8(dv[k], d);
        unpack8(xv[k], xf);
        if (relu) unpack8(yv[k], yf);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float de = (relu && yf[u] <= 0.f) ? 0.f : d[u];
          d[u] = de;
          o[u] = ka[u] * de + k1[u] * xf[u] + k0[u];
        }
        __builtin_nontemporal_store(pack8(o), (bf16x8*)dx + (i));
        if (dres) __builtin_nontemporal_store(pack8(d), (bf16x8*)dres + (i));
      }
    }
    return;
  }
  for (long long i = i0; i < n8; i += stride) {  // general C
    const int c0 = (int)(i % cg) * 8;
    float d[8], xv[8], yv[8], o[8];
    unpack8(__builtin_nontemporal_load((const bf16x8*)dy + i), d);
    unpack8(__builtin_nontemporal_load((const bf16x8*)x + i), xv);
    if (relu) unpack8(__builtin_nontemporal_load((const bf16x8*)yout + i), yv);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = c0 + u;
      const float de = (relu && yv[u] <= 0.f) ? 0.f : d[u];
      d[u] = de;
      const float xh = (xv[u] - mean[c]) * rstd[c];
      o[u] = gamma[c] * rstd[c] * (de - sum_dy[c] * inv_m - xh * sum_dyxh[c] * inv_m);
    }
    __builtin_nontemporal_store(pack8(o), (bf16x8*)dx + (i));
    if (dres) __builtin_nontemporal_store(pack8(d), (bf16x8*)dres + (i));
  }
}

// 3x3 / stride 2 / pad 1 max pool, NHWC, 8 channels (16 B) per thread;
// idx = argmax tap (first max) per output element.  One grid row per output image row
// (blockIdx.y loops over n * OH), threads over (ow, channel group) of that row: 32-bit index
// math, one small division per thread.  (The first version decoded a flat 64-bit index with
// six 64-bit divisions per element: 145 / 243 us forward / backward at ResNet-50's
// 256x112x112x64, against ~95 us of HBM traffic.)
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(int N, int H, int W, int C, int OH, int OW,
                                                          const unsigned short* __restrict__ x,
                                                          unsigned short* __restrict__ y,
                                                          unsigned char* __restrict__ idx) {
  const int cg = C >> 3;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= OW * cg) return;
  const int ow = j / cg, g = j - ow * cg;
  for (int row = blockIdx.y; row < N * OH; row += gridDim.y) {
    const int n = row / OH, oh = row - n * OH;
    float best[8];
    unsigned char bi[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { best[u] = -INFINITY; bi[u] = 0; }
    bf16x8 v[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {  // all 9 taps in flight before the compares
      const int ih = oh * 2 - 1 + t / 3, iw = ow * 2 - 1 + t % 3;
      ok[t] = ih >= 0 && ih < H && iw >= 0 && iw < W;
      if (ok[t]) v[t] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * C + g * 8);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!ok[t]) continue;
      float f[8];
      unpack8(v[t], f);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (f[u] > best[u]) { best[u] = f[u]; bi[u] = (unsigned char)t; }
    }
    const size_t o = ((size_t)row * OW + ow) * cg + g;
    ((bf16x8*)y)[o] = pack8(best);
    uint2 pk;
    pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
    pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((unsigned)bi[7] << 24);
    ((uint2*)idx)[o] = pk;
  }
}

// backward: one grid row per input image row, threads over (iw, channel group); each input
// pixel sums dy of the (at most 2 x 2) outputs whose window chose it.  Input row ih is in
// the windows of output rows (ih + 1 - kh) / 2 for the kh of matching parity: kh = 1 for even
// ih, kh = 0 and 2 for odd ih (likewise columns); all candidate loads are issued first.
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(int N, int H, int W, int C, int OH, int OW,
                                                          const unsigned short* __restrict__ dy,
                                                          const unsigned char* __restrict__ idx,
                                                          unsigned short* __restrict__ dx) {
  const int cg = C >> 3;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= W * cg) return;
  const int iw = j / cg, g = j - iw * cg;
  // column candidates (kw, ow)
  int kwc[2], owc[2];
  bool okw[2];
  if (iw & 1) {
    kwc[0] = 0; owc[0] = (iw + 1) >> 1; okw[0] = owc[0] < OW;
    kwc[1] = 2; owc[1] = (iw - 1) >> 1; okw[1] = true;
  } else {
    kwc[0] = 1; owc[0] = iw >> 1; okw[0] = owc[0] < OW;
    kwc[1] = 1; owc[1] = 0; okw[1] = false;
  }
  for (int row = blockIdx.y; row < N * H; row += gridDim.y) {
    const int n = row / H, ih = row - n * H;
    int khc[2], ohc[2];
    bool okh[2];
    if (ih & 1) {
      khc[0] = 0; ohc[0] = (ih + 1) >> 1; okh[0] = ohc[0] < OH;
      khc[1] = 2; ohc[1] = (ih - 1) >> 1; okh[1] = true;
    } else {
      khc[0] = 1; ohc[0] = ih >> 1; okh[0] = ohc[0] < OH;
      khc[1] = 1; ohc[1] = 0; okh[1] = false;
    }
    uint2 pk[2][2];
    bf16x8 dv[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (okh[a] && okw[c]) {
          const size_t o = (((size_t)n * OH + ohc[a]) * OW + owc[c]) * cg + g;
          pk[a][c] = ((const uint2*)idx)[o];
          dv[a][c] = ((const bf16x8*)dy)[o];
        }
    float acc[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        if (!(okh[a] && okw[c])) continue;
        float d[8];
        unpack8(dv[a][c], d);
        const unsigned tap = khc[a] * 3 + kwc[c];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const unsigned w = q < 4 ? pk[a][c].x : pk[a][c].y;
          if (((w >> (8 * (q & 3))) & 0xFF) == tap) acc[q] += d[q];
        }
      }
    ((bf16x8*)dx)[((size_t)row * W + iw) * cg + g] = pack8(acc);
  }
}

// ---- the ResNet stem's BatchNorm fused into its max pool ----------------------------------
// The stem output a = relu(bn(c)) (N x 112 x 112 x 64, 205 M elements at batch 256) is only
// read by the pool, so it is never written: the forward pools relu(c * A + B) formed per tap
// (bf16-rounded exactly as bn_apply_kernel stores it: the same maxima and argmax taps).  The
// backward gathers the pool gradient per input pixel, masks it with the ReLU recomputed from c
// (the forward's own arithmetic), reduces BatchNorm backward's two sums and writes de in ONE
// pass; the apply is the streaming bn_bwd_apply over de and c.  (Before: maxpool_bwd writing
// da, then bn_bwd reading da, a and c twice.  A version that re-gathered the pool gradient in
// the apply pass instead of writing de ran 610 us against ~500 for the separate passes: the
// gather runs well below streaming rate.)  fcoef: bn_fwd_coef rows [4][C].
__device__ __forceinline__ float bn_relu_bf(float v, float a, float b) {
  return bf(tobf(fmaxf(v * a + b, 0.f)));
}
__global__ __launch_bounds__(256) void maxpool_bn_fwd_kernel(int N, int H, int W, int C, int OH, int OW,
                                                             const unsigned short* __restrict__ x,
                                                             const float* __restrict__ fcoef,
                                                             unsigned short* __restrict__ y,
                                                             unsigned char* __restrict__ idx) {
  const int cg = C >> 3;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= OW * cg) return;
  const int ow = j / cg, g = j - ow * cg;
  float sa[8], sb[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    sa[u] = fcoef[g * 8 + u];
    sb[u] = fcoef[2 * C + g * 8 + u];
  }
  for (int row = blockIdx.y; row < N * OH; row += gridDim.y) {
    const int n = row / OH, oh = row - n * OH;
    float best[8];
    unsigned char bi[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) { best[u] = -INFINITY; bi[u] = 0; }
    bf16x8 v[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ih = oh * 2 - 1 + t / 3, iw = ow * 2 - 1 + t % 3;
      ok[t] = ih >= 0 && ih < H && iw >= 0 && iw < W;
      if (ok[t]) v[t] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * C + g * 8);
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (!ok[t]) continue;
      float f[8];
      unpack8(v[t], f);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float a = bn_relu_bf(f[u], sa[u], sb[u]);
        if (a > best[u]) { best[u] = a; bi[u] = (unsigned char)t; }
      }
    }
    const size_t o = ((size_t)row * OW + ow) * cg + g;
    ((bf16x8*)y)[o] = pack8(best);
    uint2 pk;
    pk.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((unsigned)bi[3] << 24);
    pk.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((unsigned)bi[7] << 24);
    ((uint2*)idx)[o] = pk;
  }
}

// The pool gradient of input pixel (n, ih, iw), channels 8 g .. + 7 (maxpool_bwd_kernel's
// gather), rounded to bf16 as maxpool_bwd stores it.  Branch-free: the (at most 2 x 2)
// candidate windows are loaded from clamped in-range addresses and masked afterwards, so a
// caller's two rows' loads can all be in flight together.
struct PoolCand {
  uint2 pk[2][2];
  bf16x8 dv[2][2];
  unsigned tap[2][2];  // the window tap this pixel is, or 0xFF for no window
};
__device__ __forceinline__ void maxpool_grad8_load(int n, int ih, int iw, int g, int cg, int OH,
                                                   int OW, const unsigned short* __restrict__ dy,
                                                   const unsigned char* __restrict__ idx,
                                                   PoolCand& pc) {
  int khc[2], ohc[2], kwc[2], owc[2];
  bool okh[2], okw[2];
  if (ih & 1) {
    khc[0] = 0; ohc[0] = (ih + 1) >> 1; okh[0] = ohc[0] < OH;
    khc[1] = 2; ohc[1] = (ih - 1) >> 1; okh[1] = true;
  } else {
    khc[0] = 1; ohc[0] = ih >> 1; okh[0] = ohc[0] < OH;
    khc[1] = 1; ohc[1] = 0; okh[1] = false;
  }
  if (iw & 1) {
    kwc[0] = 0; owc[0] = (iw + 1) >> 1; okw[0] = owc[0] < OW;
    kwc[1] = 2; owc[1] = (iw - 1) >> 1; okw[1] = true;
  } else {
    kwc[0] = 1; owc[0] = iw >> 1; okw[0] = owc[0] < OW;
    kwc[1] = 1; owc[1] = 0; okw[1] = false;
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const bool ok = okh[a] && okw[c];
      const size_t o = (((size_t)n * OH + min(ohc[a], OH - 1)) * OW + min(owc[c], OW - 1)) * cg + g;
      pc.pk[a][c] = ((const uint2*)idx)[o];
      pc.dv[a][c] = ((const bf16x8*)dy)[o];
      pc.tap[a][c] = ok ? (unsigned)(khc[a] * 3 + kwc[c]) : 0xFFu;
    }
}
__device__ __forceinline__ void maxpool_grad8_sum(const PoolCand& pc, float* out) {
#pragma unroll
  for (int u = 0; u < 8; ++u) out[u] = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      float d[8];
      unpack8(pc.dv[a][c], d);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const unsigned w = q < 4 ? pc.pk[a][c].x : pc.pk[a][c].y;
        if (((w >> (8 * (q & 3))) & 0xFF) == pc.tap[a][c]) out[q] += d[q];
      }
    }
#pragma unroll
  for (int u = 0; u < 8; ++u) out[u] = bf(tobf(out[u]));
}

// de = da * (bn(c) > 0) written, and per block the sums of de and de * xhat over its rows: one
// partial row per block (blockIdx.y * gridDim.x + blockIdx.x), the threads of a channel group
// meet in LDS.
__global__ __launch_bounds__(256) void maxpool_bn_bwd_reduce_kernel(
    int N, int H, int W, int C, int OH, int OW, const unsigned short* __restrict__ dy,
    const unsigned char* __restrict__ idx, const unsigned short* __restrict__ x,
    const float* __restrict__ fcoef, const float* __restrict__ mean, const float* __restrict__ rstd,
    float* __restrict__ part_dy, float* __restrict__ part_dyxh, unsigned short* __restrict__ de_out) {
  __shared__ float red[256][17];
  const int cg = C >> 3;
  const int j = blockIdx.x * 256 + threadIdx.x;
  const bool live = j < W * cg;
  const int iw = live ? j / cg : 0, g = live ? j - iw * cg : 0;
  float sa[8], sb[8], mu[8], rs[8], s1[8], s2[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    sa[u] = fcoef[g * 8 + u];
    sb[u] = fcoef[2 * C + g * 8 + u];
    mu[u] = mean[g * 8 + u];
    rs[u] = rstd[g * 8 + u];
    s1[u] = s2[u] = 0.f;
  }
  if (live) {
    // two rows per iteration, every load of both issued before the first use
    const int NH = N * H, gy = gridDim.y;
    for (int row = blockIdx.y; row < NH; row += 2 * gy) {
      int rr[2];
      rr[0] = row;
      rr[1] = row + gy < NH ? row + gy : row;  // (a duplicate row: loaded, not stored / summed)
      PoolCand pc[2];
      bf16x8 xv[2];
      size_t o[2];
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int n = rr[k] / H, ih = rr[k] - n * H;
        o[k] = ((size_t)rr[k] * W + iw) * cg + g;
        xv[k] = ((const bf16x8*)x)[o[k]];
        maxpool_grad8_load(n, ih, iw, g, cg, OH, OW, dy, idx, pc[k]);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        if (k == 1 && row + gy >= NH) break;
        float da[8], xf[8];
        maxpool_grad8_sum(pc[k], da);
        unpack8(xv[k], xf);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float de = xf[u] * sa[u] + sb[u] > 0.f ? da[u] : 0.f;
          da[u] = de;
          s1[u] += de;
          s2[u] += de * (xf[u] - mu[u]) * rs[u];
        }
        ((bf16x8*)de_out)[o[k]] = pack8(da);
      }
    }
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    red[threadIdx.x][u] = live ? s1[u] : 0.f;
    red[threadIdx.x][8 + u] = live ? s2[u] : 0.f;
  }
  __syncthreads();
  // channel c = 8 g + u: threads t with (blockIdx.x * 256 + t) % cg == g (256 % cg == 0)
  const size_t prow = (size_t)(blockIdx.y * gridDim.x + blockIdx.x) * C;
  for (int c = threadIdx.x; c < C; c += 256) {
    const int gg = c >> 3, u = c & 7;
    const int t0 = ((gg - (blockIdx.x * 256) % cg) % cg + cg) % cg;
    float a = 0.f, b = 0.f;
    for (int t = t0; t < 256; t += cg) {
      a += red[t][u];
      b += red[t][8 + u];
    }
    part_dy[prow + c] = a;
    part_dyxh[prow + c] = b;
  }
}

// global average pool: x [N][HW][C] -> y [N][C] (bf16); thread per (n, c)
__global__ __launch_bounds__(256) void avgpool_fwd_kernel(int N, int HW, int C,
                                                          const unsigned short* __restrict__ x,
                                                          unsigned short* __restrict__ y) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N * C) return;
  const int n = i / C, c = i % C;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += bf(x[((size_t)n * HW + p) * C + c]);
  y[i] = tobf(s / HW);
}

__global__ __launch_bounds__(256) void avgpool_bwd_kernel(int N, int HW, int C,
                                                          const unsigned short* __restrict__ dy,
                                                          unsigned short* __restrict__ dx) {
  const long long total = (long long)N * HW * C;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c = (int)(i % C);
    const int n = (int)(i / ((long long)HW * C));
    dx[i] = tobf(bf(dy[(size_t)n * C + c]) / HW);
  }
}

// momentum SGD on f32 master weights (+ L2 weight decay), refreshes the bf16 copy
__global__ __launch_bounds__(256) void sgd_momentum_mixed_kernel(
    long long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ v,
    unsigned short* __restrict__ pb, float lr, float mu, float wd, float gscale) {
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pv = ((f32x4*)p)[i], gv = ((const f32x4*)g)[i], vv = ((f32x4*)v)[i];
    ushort4 o;
    unsigned short* op = (unsigned short*)&o;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vv[u] = mu * vv[u] + gv[u] * gscale + wd * pv[u];
      pv[u] -= lr * vv[u];
      op[u] = tobf(pv[u]);
    }
    __builtin_nontemporal_store(pv, (f32x4*)p + (i));
    __builtin_nontemporal_store(vv, (f32x4*)v + (i));
    if (pb) ((ushort4*)pb)[i] = o;
  }
}

// The same momentum SGD with the weight gradients of some flat ranges ("segments") left as
// split-K partial planes by their convolutions (conv_bf16 defer_reduce, one GPU): the planes are
// summed here, in split order (the order splitk_reduce sums them), instead of by a reduce pass
// per weight gradient that writes the gradient only for this kernel to read back (ResNet-50: 49
// reduce launches per step).  Segment k (int64 x 5, sorted, disjoint): {lo4, hi4 (float4
// indices into the flat buffer), planes (f32 pointer), plane stride in float4s, S}; a lane finds
// its segment by binary search in LDS.  (As BERT's adam_mixed_segs_kernel.)
constexpr int kSgdMaxSegs = 128;
__global__ __launch_bounds__(256) void sgd_momentum_mixed_segs_kernel(
    long long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ v,
    unsigned short* __restrict__ pb, float lr, float mu, float wd, float gscale,
    const long long* __restrict__ segs, int nseg) {
  __shared__ long long s_lo[kSgdMaxSegs], s_hi[kSgdMaxSegs], s_pl[kSgdMaxSegs];
  __shared__ const f32x4* s_w[kSgdMaxSegs];
  __shared__ int s_S[kSgdMaxSegs];
  for (int k = threadIdx.x; k < nseg; k += blockDim.x) {
    s_lo[k] = segs[5 * k];
    s_hi[k] = segs[5 * k + 1];
    s_w[k] = (const f32x4*)segs[5 * k + 2];
    s_pl[k] = segs[5 * k + 3];
    s_S[k] = (int)segs[5 * k + 4];
  }
  __syncthreads();
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    int lo = 0, hi = nseg - 1, k = -1;  // last segment with lo <= i
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      if (s_lo[mid] <= i) {
        k = mid;
        lo = mid + 1;
      } else {
        hi = mid - 1;
      }
    }
    f32x4 gv;
    if (k >= 0 && i < s_hi[k]) {
      const f32x4* w = s_w[k] + (i - s_lo[k]);
      const long long pl = s_pl[k];
      const int S = s_S[k];
      // four planes' loads in flight at a time, added in split order
      gv = __builtin_nontemporal_load(w);
      int q = 1;
      for (; q + 3 < S; q += 4) {
        const f32x4 a0 = __builtin_nontemporal_load(w + q * pl),
                    a1 = __builtin_nontemporal_load(w + (q + 1) * pl),
                    a2 = __builtin_nontemporal_load(w + (q + 2) * pl),
                    a3 = __builtin_nontemporal_load(w + (q + 3) * pl);
        gv += a0;
        gv += a1;
        gv += a2;
        gv += a3;
      }
      for (; q < S; ++q) gv += __builtin_nontemporal_load(w + q * pl);
    } else {
      gv = ((const f32x4*)g)[i];
    }
    f32x4 pv = ((f32x4*)p)[i], vv = ((f32x4*)v)[i];
    ushort4 o;
    unsigned short* op = (unsigned short*)&o;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      vv[u] = mu * vv[u] + gv[u] * gscale + wd * pv[u];
      pv[u] -= lr * vv[u];
      op[u] = tobf(pv[u]);
    }
    __builtin_nontemporal_store(pv, (f32x4*)p + (i));
    __builtin_nontemporal_store(vv, (f32x4*)v + (i));
    if (pb) ((ushort4*)pb)[i] = o;
  }
}

// Streaming BatchNorm kernels: each thread makes ONE pass with kEwU 16-B chunks in flight
// (grid = chunks / (256 * kEwU)).  Measured at ResNet-50's largest activation (205M bf16):
// bn_apply 165 -> 144 us (4.97 -> 5.71 TB/s), with residual 253 -> 211 us; the old fixed
// 8192-block grid with 4 chunks per pass reached 4.9 (tools/probes/bn_bw.py sweep).
constexpr int kEwU = 2;
static unsigned grid_once(long long chunks, int u) {
  long long b = (chunks + 256LL * u - 1) / (256LL * u);
  if (b > (1LL << 30)) b = 1LL << 30;
  return (unsigned)(b < 1 ? 1 : b);
}

static unsigned grid_for(long long n, int per = 256) {
  long long b = (n + per - 1) / per;
  if (b > 8192) b = 8192;
  if (b < 1) b = 1;
  return (unsigned)b;
}

void colpart_reduce_launch(int R, int C, const float* ps, const float* pq, float* os, float* oq,
                           hipStream_t st) {
  // >= 16 rows per block (4 per thread), at most 256 row blocks: every block ends in one
  // same-address atomic per channel, so more blocks trade load latency for atomic serialisation
  int S = (R + 15) / 16;
  if (S > 256) S = 256;
  if (S < 1) S = 1;
  hipLaunchKernelGGL(colpart_reduce_kernel, dim3((C + 63) / 64, S), dim3(256), 0, st, R, C, ps, pq,
                     os, oq);
  DTFX_HIP_CHECK(hipGetLastError());
}

void bn_finalize_launch(int C, long long M, const float* s, const float* q, float eps, float* mean,
                        float* rstd, float* run_mean, float* run_var, float momentum,
                        hipStream_t st) {
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, st, C, 1.f / (float)M,
                     M > 1 ? (float)M / (float)(M - 1) : 1.f, s, q, eps, mean, rstd, run_mean,
                     run_var, momentum);
  DTFX_HIP_CHECK(hipGetLastError());
}

void bn_apply_launch(long long M, int C, const void* x, const float* mean, const float* rstd,
                     const float* gamma, const float* beta, const void* res, int relu, void* y,
                     hipStream_t st) {
  if (C % 8) throw std::runtime_error("bn_apply: C % 8 != 0");
  hipLaunchKernelGGL((bn_apply_kernel<kEwU, false, false>), dim3(grid_once(M * C / 8, kEwU)), dim3(256),
                     0, st, M, C, (const unsigned short*)x, mean, rstd, gamma, beta,
                     (const unsigned short*)res, relu, (unsigned short*)y, BnStats{}, BnStats{});
  DTFX_HIP_CHECK(hipGetLastError());
}

// Training-mode forward BatchNorm in one launch: statistics from the column sums s / q
// (sum, sum of squares over M rows), mean / rstd written for the backward, running
// statistics updated (momentum, unbiased variance), y = act(bn(x) [+ res]).  With s2 set the
// residual is a raw conv output normalised by its own statistics s2 / q2 and affine g2 / b2
// (mean2 / rstd2 / running2 written likewise): y = act(bn(x) + bn2(res)).
void bn_apply_stats_launch(long long M, int C, const void* x, const float* s, const float* q,
                           float eps, float* mean, float* rstd, float* run_mean, float* run_var,
                           float momentum, const float* gamma, const float* beta, const void* res,
                           int relu, void* y, const float* s2, const float* q2, const float* g2,
                           const float* b2, float* mean2, float* rstd2, float* run_mean2,
                           float* run_var2, hipStream_t stream) {
  if (C % 8) throw std::runtime_error("bn_apply: C % 8 != 0");
  if (s2 && (!res || !q2 || !g2 || !b2 || !mean2 || !rstd2))
    throw std::runtime_error("bn_apply_stats: residual BN needs res, q2, gamma2, beta2, mean2, rstd2");
  const float inv_m = 1.f / (float)M, unbias = M > 1 ? (float)M / (float)(M - 1) : 1.f;
  BnStats bs{s, q, inv_m, eps, unbias, momentum, mean, rstd, run_mean, run_var, nullptr, nullptr};
  BnStats bs2{s2, q2, inv_m, eps, unbias, momentum, mean2, rstd2, run_mean2, run_var2, g2, b2};
  auto k = s2 ? bn_apply_kernel<kEwU, true, true> : bn_apply_kernel<kEwU, true, false>;
  hipLaunchKernelGGL(k, dim3(grid_once(M * C / 8, kEwU)), dim3(256), 0, stream, M, C,
                     (const unsigned short*)x, (const float*)nullptr, (const float*)nullptr, gamma,
                     beta, (const unsigned short*)res, relu, (unsigned short*)y, bs, bs2);
  DTFX_HIP_CHECK(hipGetLastError());
}

// Coefficients for conv1x1_pro_launch (mode 1): the training-mode BatchNorm of x (column sums
// s / q over M rows, affine gamma / beta) plus the residual term (s2 set: a raw conv output
// with its own BN), mean / rstd (and mean2 / rstd2) stored, running statistics updated --
// bn_apply_stats_launch's bookkeeping, with the elementwise pass left to the consumer conv.
void bn_fwd_coef_launch(long long M, int C, const float* s, const float* q, float eps, float* mean,
                        float* rstd, float* run_mean, float* run_var, float momentum,
                        const float* gamma, const float* beta, const float* s2, const float* q2,
                        const float* g2, const float* b2, float* mean2, float* rstd2,
                        float* run_mean2, float* run_var2, float* coef, hipStream_t stream) {
  if (s2 && (!q2 || !g2 || !b2 || !mean2 || !rstd2))
    throw std::runtime_error("bn_fwd_coef: residual BN needs q2, gamma2, beta2, mean2, rstd2");
  const float inv_m = 1.f / (float)M, unbias = M > 1 ? (float)M / (float)(M - 1) : 1.f;
  BnStats bs{s, q, inv_m, eps, unbias, momentum, mean, rstd, run_mean, run_var, nullptr, nullptr};
  BnStats bs2{s2, q2, inv_m, eps, unbias, momentum, mean2, rstd2, run_mean2, run_var2, g2, b2};
  hipLaunchKernelGGL(bn_fwd_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, C, bs, bs2,
                     gamma, beta, s2 ? 1 : 0, coef);
  DTFX_HIP_CHECK(hipGetLastError());
}
// Coefficients for conv1x1_pro_launch (mode 2): BatchNorm backward's apply half from the final
// reductions (as bn_bwd_apply_launch).
void bn_bwd_coef_launch(long long M, int C, const float* mean, const float* rstd, const float* gamma,
                        const float* sum_dy, const float* sum_dyxh, float* coef, hipStream_t stream) {
  hipLaunchKernelGGL(bn_bwd_coef_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, C, mean, rstd,
                     gamma, sum_dy, sum_dyxh, 1.f / (float)M, coef);
  DTFX_HIP_CHECK(hipGetLastError());
}

// sum_dy / sum_dyxh (f32 [C]) are ACCUMULATED (+=): pass zeroed buffers, or the
// (zeroed) dbeta / dgamma gradient slots themselves -- they are exactly these sums.
// scratch: f32 [2 * bn_bwd_scratch_rows(M, C)][C].
long long bn_bwd_scratch_rows(long long M, int C) {
  const int cg = C / 8, tpr = cg < 256 ? cg : 256, rpp = 256 / tpr;
  long long rpb = (M + 1023) / 1024;
  if (rpb < rpp * 4) rpb = rpp * 4;
  return (M + rpb - 1) / rpb;
}

void bn_bwd_launch(long long M, int C, const void* dy, const void* yout, const void* x,
                   const float* mean, const float* rstd, const float* gamma, int relu,
                   float* sum_dy, float* sum_dyxh, float* scratch, void* dx, void* dres,
                   hipStream_t st) {
  if (C % 8 || C > 2048 * 64) throw std::runtime_error("bn_bwd: C % 8 != 0");
  const int cg = C / 8, tpr = cg < 256 ? cg : 256, rpp = 256 / tpr;
  long long rpb = (M + 1023) / 1024;
  if (rpb < rpp * 4) rpb = rpp * 4;
  const long long blocks = (M + rpb - 1) / rpb;
  float* part_dy = scratch;
  float* part_dyxh = scratch + blocks * C;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3((unsigned)blocks), dim3(256), 0, st, M, C, (int)rpb,
                     (const unsigned short*)dy, (const unsigned short*)yout,
                     (const unsigned short*)x, mean, rstd, relu, part_dy, part_dyxh);
  DTFX_HIP_CHECK(hipGetLastError());
  colpart_reduce_launch((int)blocks, C, part_dy, part_dyxh, sum_dy, sum_dyxh, st);
  if (!dx && !dres) return;  // reductions only (the apply runs in a consumer's prologue)
  hipLaunchKernelGGL(bn_bwd_apply_kernel<kEwU>, dim3(grid_once(M * C / 8, kEwU)), dim3(256), 0, st, M, C,
                     (const unsigned short*)dy, (const unsigned short*)yout,
                     (const unsigned short*)x, mean, rstd, gamma, sum_dy, sum_dyxh, relu,
                     1.f / (float)M, (unsigned short*)dx, (unsigned short*)dres);
  DTFX_HIP_CHECK(hipGetLastError());
}

// Apply half of BatchNorm backward when the reductions were fused into the producing conv
// dgrad (conv_bf16 mode 2 with relu_y / bn_x): de is already dL/d(BN output) (masked),
// sum_dy / sum_dyxh are final.
void bn_bwd_apply_launch(long long M, int C, const void* de, const void* x, const float* mean,
                         const float* rstd, const float* gamma, const float* sum_dy,
                         const float* sum_dyxh, void* dx, hipStream_t st) {
  if (C % 8) throw std::runtime_error("bn_bwd_apply: C % 8 != 0");
  hipLaunchKernelGGL(bn_bwd_apply_kernel<kEwU>, dim3(grid_once(M * C / 8, kEwU)), dim3(256), 0, st, M, C,
                     (const unsigned short*)de, (const unsigned short*)nullptr,
                     (const unsigned short*)x, mean, rstd, gamma, sum_dy, sum_dyxh, 0,
                     1.f / (float)M, (unsigned short*)dx, (unsigned short*)nullptr);
  DTFX_HIP_CHECK(hipGetLastError());
}

void maxpool_fwd_launch(int N, int H, int W, int C, const void* x, void* y, void* idx, hipStream_t st) {
  if (C % 8) throw std::runtime_error("maxpool: C % 8 != 0");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int rows = std::min(N * OH, 65535);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3((OW * (C / 8) + 255) / 256, rows), dim3(256), 0, st, N,
                     H, W, C, OH, OW, (const unsigned short*)x, (unsigned short*)y,
                     (unsigned char*)idx);
  DTFX_HIP_CHECK(hipGetLastError());
}

void maxpool_bwd_launch(int N, int H, int W, int C, const void* dy, const void* idx, void* dx,
                        hipStream_t st) {
  if (C % 8) throw std::runtime_error("maxpool: C % 8 != 0");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int rows = std::min(N * H, 65535);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((W * (C / 8) + 255) / 256, rows), dim3(256), 0, st, N,
                     H, W, C, OH, OW, (const unsigned short*)dy, (const unsigned char*)idx,
                     (unsigned short*)dx);
  DTFX_HIP_CHECK(hipGetLastError());
}

// The stem's BatchNorm + ReLU + 3x3/2 max pool (see maxpool_bn_fwd_kernel).
void maxpool_bn_fwd_launch(int N, int H, int W, int C, const void* x, const float* fcoef, void* y,
                           void* idx, hipStream_t st) {
  if (C % 8 || 256 % (C / 8)) throw std::runtime_error("maxpool_bn: C % 8 != 0, 256 % (C / 8) == 0");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int rows = std::min(N * OH, 65535);
  hipLaunchKernelGGL(maxpool_bn_fwd_kernel, dim3((OW * (C / 8) + 255) / 256, rows), dim3(256), 0, st,
                     N, H, W, C, OH, OW, (const unsigned short*)x, fcoef, (unsigned short*)y,
                     (unsigned char*)idx);
  DTFX_HIP_CHECK(hipGetLastError());
}
// Partial-row count of maxpool_bn_bwd's reduce pass ([rows][C] each of part_dy / part_dyxh):
// ~7 input rows per thread at ResNet-50's 256 x 112 rows -- one row per block would write
// 115 k partial rows, 112 rows per thread left the pass latency-bound (242 us).
static int maxpool_bn_bwd_gy(int N, int H) { return std::min(N * H, 4096); }
int maxpool_bn_bwd_rows(int N, int H, int W, int C) {
  return ((W * (C / 8) + 255) / 256) * maxpool_bn_bwd_gy(N, H);
}
// Backward: de (the masked pool gradient, written to `de`) with BatchNorm backward's sums
// ACCUMULATED into sum_dy / sum_dyxh (the zeroed dbeta / dgamma slots), then the apply
// dx = dL/dc over de and c (bn_bwd_apply_kernel) -- or, with dx null, only its coefficients.
void maxpool_bn_bwd_launch(int N, int H, int W, int C, const void* dy, const void* idx,
                           const void* x, const float* fcoef, const float* mean, const float* rstd,
                           const float* gamma, float* sum_dy, float* sum_dyxh, float* scratch,
                           void* de, void* dx, float* bcoef, hipStream_t st) {
  if (C % 8 || 256 % (C / 8)) throw std::runtime_error("maxpool_bn: C % 8 != 0, 256 % (C / 8) == 0");
  const int OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  const int gx = (W * (C / 8) + 255) / 256, gy = maxpool_bn_bwd_gy(N, H);
  const int R = gx * gy;
  hipLaunchKernelGGL(maxpool_bn_bwd_reduce_kernel, dim3(gx, gy), dim3(256), 0, st, N, H, W, C, OH, OW,
                     (const unsigned short*)dy, (const unsigned char*)idx,
                     (const unsigned short*)x, fcoef, mean, rstd, scratch, scratch + (size_t)R * C,
                     (unsigned short*)de);
  DTFX_HIP_CHECK(hipGetLastError());
  colpart_reduce_launch(R, C, scratch, scratch + (size_t)R * C, sum_dy, sum_dyxh, st);
  // dx == null: the consumer forms dL/dc itself (the stem weight gradient's prologue) from the
  // apply coefficients, written to bcoef
  if (dx) bn_bwd_apply_launch((long long)N * H * W, C, de, x, mean, rstd, gamma, sum_dy, sum_dyxh, dx, st);
  else bn_bwd_coef_launch((long long)N * H * W, C, mean, rstd, gamma, sum_dy, sum_dyxh, bcoef, st);
}

void avgpool_fwd_launch(int N, int HW, int C, const void* x, void* y, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_fwd_kernel, dim3((N * C + 255) / 256), dim3(256), 0, st, N, HW, C,
                     (const unsigned short*)x, (unsigned short*)y);
  DTFX_HIP_CHECK(hipGetLastError());
}

void avgpool_bwd_launch(int N, int HW, int C, const void* dy, void* dx, hipStream_t st) {
  hipLaunchKernelGGL(avgpool_bwd_kernel, dim3(grid_for((long long)N * HW * C)), dim3(256), 0, st, N,
                     HW, C, (const unsigned short*)dy, (unsigned short*)dx);
  DTFX_HIP_CHECK(hipGetLastError());
}

void sgd_momentum_mixed_launch(long long n, float* p, const float* g, float* v, void* pb, float lr,
                               float mu, float wd, float gscale, hipStream_t st,
                               const long long* segs, int nseg) {
  if (n % 4) throw std::runtime_error("sgd_momentum_mixed: n % 4 != 0");
  if (nseg < 0 || nseg > kSgdMaxSegs || (nseg && !segs))
    throw std::runtime_error("sgd_momentum_mixed: 0..128 segments with a table");
  if (nseg) {
    hipLaunchKernelGGL(sgd_momentum_mixed_segs_kernel, dim3(grid_for(n / 4)), dim3(256), 0, st, n,
                       p, g, v, (unsigned short*)pb, lr, mu, wd, gscale, segs, nseg);
    DTFX_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(sgd_momentum_mixed_kernel, dim3(grid_for(n / 4)), dim3(256), 0, st, n, p, g, v,
                     (unsigned short*)pb, lr, mu, wd, gscale);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
