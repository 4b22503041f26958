// 3x3 / stride 1 / pad 1 convolution forward with 64 input and 64 output channels (ResNet-50
// layer1's conv2 at 56 x 56), NHWC bf16, BatchNorm statistics of the output fused (partial
// rows, reduced by colpart_reduce).
//
// The stem's scheme (stem_conv.hip) applied to layer1: all 64 x 576 weights stay in LDS for a
// persistent block's life, and per 8 x 28-pixel output tile the 10 x 30-pixel input patch is
// staged ONCE (prefetched a tile ahead into registers), so the MFMA A fragments of every tap
// are read from the patch at the tap's offset instead of re-gathering each input pixel nine
// times through L2 (the implicit GEMM's 256x64 tile: 181 us per call at batch 256, against
// ~32 us of HBM traffic).  Patch pixels are 128-B rows of 8 16-B channel chunks, chunk c of
// pixel q stored at c ^ (q & 7): the 16 lanes of a fragment read 16 consecutive pixels.
//
// k-group kg = (tap kg / 2, channel half kg % 2): 18 groups of 32; the wave layout of the
// forward / data gradient is at conv3x3_c64_kernel, the weight gradient's at its kernel (which
// keeps 4 x 28 tiles).
#include "common.h"

#include <algorithm>
#include <stdexcept>

namespace dtfx {
namespace c3 {

typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int C = 64, TH = 4, TW = 28, PH = TH + 2, PW = TW + 2;  // 6 x 30 patch
constexpr int NPX = TH * TW;                                     // 112 = 7 groups of 16
constexpr int WP = 584;                                          // weight row pitch, bf16
constexpr int W_BYTES = C * WP * 2;                              // 74752
constexpr int P_BYTES = PH * PW * 128;                           // 23040 (output staging too)
constexpr int PCH = PH * PW * 8;                                 // 1440 patch chunks
// forward / data gradient: 8 x 28 output tiles (10 x 30 patch), K-half partials in LDS
constexpr int TH2 = 8, NPX2 = TH2 * TW;                          // 224 = 14 groups of 16
constexpr int PCH2 = (TH2 + 2) * PW * 8;                         // 2400 patch chunks
constexpr int PP2 = 144;                                         // patch pixel pitch (bytes)
constexpr int R_BYTES = 2 * 2 * 2 * 7 * 64 * 16;                 // 57344 (> the 43200-B patch)

__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

// Forward (DGRAD false) and data gradient (DGRAD true) on 8 x 28-pixel output tiles (14
// pixel groups of 16, a 10 x 30 input patch).  8 waves: wave w owns output channels
// 32 (w & 1) .. + 31, input-channel half (w >> 1) & 1 (the K split: k-groups 2 tap + half)
// and pixel groups 7 (w >> 2) .. + 6: per k-group 7 A + 2 B fragment reads for 14 MFMAs.  The
// first version (wave = 16 output channels x the whole K x 4 or 3 groups of a 4 x 28 tile:
// 4 A + 1 B reads per 4 MFMAs, and a 4 / 3 group imbalance) was bound by LDS bandwidth at
// ~2.6x its MFMA time.  The K halves are summed through LDS after the last k-group: of each
// pair, the half-0 wave finalises groups 0-3 and the half-1 wave groups 4-6 of its seven.
//
// The data gradient of a stride-1 3x3 conv is the forward conv of dy with the kernel flipped
// and transposed, W'[ci][tap][co] = W[co][8 - tap][ci] (conv3x3_c64_flip_kernel, once per call
// into a workspace: each block building it with 2-byte gathers cost ~15 us); with relu_y the BatchNorm backward is fused as the GEMM path's epilogue:
// de = dx * (relu_y > 0) and sum(de), sum(de * xhat) (xhat from bn_x, mean, rstd) as partial
// rows, one per wave and tile ([8 * tiles][64]); relu_y / bn_x may be null (plain dgrad).
// Forward: the output's BatchNorm statistics (f32 values) as partial rows [4 * tiles][64].
// W' [ci][tap * 64 + co] = W [co][(8 - tap) * 64 + ci]
__global__ __launch_bounds__(256) void conv3x3_c64_flip_kernel(const unsigned short* __restrict__ w,
                                                               int ldw, unsigned short* __restrict__ wf) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // output element
  if (i >= C * 9 * C) return;
  const int ci = i / (9 * C), rem = i - ci * 9 * C, tap = rem / C, co = rem - tap * C;
  wf[i] = w[(size_t)co * ldw + (8 - tap) * C + ci];
}

// PRO (forward): x is the raw output c of the previous conv and the patch is formed as
// relu(c a + b) per channel (coef rows 0 / 2 of bn_fwd_coef) while it is staged; in-image
// pixels only (the zero padding stays zero), and each tile writes its own (interior) pixels of
// the result to xo once -- the backward reads it.  The bn_apply pass that wrote it and this
// kernel's read of it become one read of c.
template <bool DGRAD, bool PRO = false>
__global__ __launch_bounds__(512, 1) void conv3x3_c64_kernel(
    int N, int H, int W, const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
    int ldw, unsigned short* __restrict__ y, const unsigned short* __restrict__ relu_y,
    const unsigned short* __restrict__ bn_x, const float* __restrict__ bn_mean,
    const float* __restrict__ bn_rstd, float* __restrict__ psum, float* __restrict__ psq,
    const float* __restrict__ coef = nullptr, unsigned short* __restrict__ xo = nullptr) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Ws = sm;
  char* Ps = sm + W_BYTES;  // patch, then the K-half partials, then the output staging
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < C * 72; i += 512) {  // weights [64 co][576 k] (dgrad: W'), once
    const int co = i / 72, c = i - co * 72;
    *(bf16x8*)(Ws + co * WP * 2 + c * 16) = *(const bf16x8*)(w + (size_t)co * ldw + c * 8);
  }
  const int tiles_w = W / TW, tiles_img = (H / TH2) * tiles_w, tiles = N * tiles_img;
  const int cl = lane & 15, g = lane >> 4;
  const int cb = wave & 1, kh = (wave >> 1) & 1, ph = wave >> 2;
  const bool fused = DGRAD && relu_y != nullptr;
  const int ec = tid & 7;  // the 8-channel chunk this thread handles in the epilogue
  float mu[8], rs[8];
  if (fused) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      mu[u] = bn_mean[ec * 8 + u];
      rs[u] = bn_rstd[ec * 8 + u];
    }
  }
  float pa[8], pc_[8];  // PRO: this thread's channels (chunk tid & 7) scale / shift
  if constexpr (PRO) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      pa[u] = coef[ec * 8 + u];
      pc_[u] = coef[2 * C + ec * 8 + u];
    }
  }
  bf16x8 v[5];  // patch chunks of the next tile: 2400 / 512 -> 5 per thread
  int lpr[5], lpc[5];  // their patch rows / columns (tile-invariant)
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const int q = (tid + 512 * k) >> 3;
    lpr[k] = q / PW;
    lpc[k] = q - lpr[k] * PW;
  }
  auto load_patch = [&](int tt) {
    const int n = tt / tiles_img, r = tt - n * tiles_img;
    const int ih0 = (r / tiles_w) * TH2 - 1, iw0 = (r % tiles_w) * TW - 1;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int e = tid + 512 * k, c = e & 7;
      const int ih = ih0 + lpr[k], iw = iw0 + lpc[k];
      v[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (e < PCH2 && ih >= 0 && ih < H && iw >= 0 && iw < W)
        v[k] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * C + c * 8);
    }
  };
  // A fragment addresses of tap (0, 0): this lane's pixel in each of its groups, its chunk.
  // Patch pixels are 144-B rows (16 consecutive pixels: 16 distinct 16-B bank slots), so a
  // tap's offset is a compile-time immediate of the LDS read.
  int abase[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int p = 16 * (7 * ph + i) + cl;
    abase[i] = ((p / TW) * PW + (p % TW)) * PP2 + (kh * 4 + g) * 16;
  }
  const int bbase = (32 * cb + cl) * WP * 2 + (32 * kh + 8 * g) * 2;
  if (blockIdx.x < tiles) load_patch(blockIdx.x);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int n = t / tiles_img, r = t - n * tiles_img;
    const int oh0 = (r / tiles_w) * TH2, ow0 = (r % tiles_w) * TW;
    __syncthreads();  // the previous tile's output staging is consumed
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const int e = tid + 512 * k, q = e >> 3, c = e & 7;
      if (e < PCH2) {
        bf16x8 o = v[k];
        if constexpr (PRO) {
          const int ih = oh0 - 1 + lpr[k], iw = ow0 - 1 + lpc[k];
          if (ih >= 0 && ih < H && iw >= 0 && iw < W) {
#pragma unroll
            for (int u = 0; u < 8; ++u)
              o[u] = (short)tobf(fmaxf(__uint_as_float((unsigned)(unsigned short)v[k][u] << 16) * pa[u] + pc_[u], 0.f));
            if (lpr[k] >= 1 && lpr[k] <= TH2 && lpc[k] >= 1 && lpc[k] <= TW)  // this tile's own pixel
              __builtin_nontemporal_store(o, (bf16x8*)(xo + (((size_t)n * H + ih) * W + iw) * C + c * 8));
          }
        }
        *(bf16x8*)(Ps + q * PP2 + c * 16) = o;
      }
    }
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_patch(t + gridDim.x);
    // data gradient: the epilogue's side inputs requested now, in flight during the MFMAs
    bf16x8 ysv[4], xsv[4];
    if (fused) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = tid + 512 * k, p = e >> 3;
        if (e < NPX2 * 8) {
          const size_t go = (((size_t)n * H + oh0 + p / TW) * W + ow0 + p % TW) * C + ec * 8;
          ysv[k] = *(const bf16x8*)(relu_y + go);
          xsv[k] = *(const bf16x8*)(bn_x + go);
        }
      }
    }
    f32x4 acc[7][2];
#pragma unroll
    for (int i = 0; i < 7; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int th = tap / 3, tw = tap - th * 3;
      const bf16x8 b0 = *(const bf16x8*)(Ws + bbase + tap * 128);
      const bf16x8 b1 = *(const bf16x8*)(Ws + bbase + 16 * WP * 2 + tap * 128);
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const bf16x8 a = *(const bf16x8*)(Ps + abase[i] + (th * PW + tw) * PP2);
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc[i][1], 0, 0, 0);
      }
    }
    __syncthreads();  // every wave is done with the patch
    // K halves: write the partner's pixel groups, then add the partner's partials of ours
    f32x4* red = (f32x4*)Ps;  // [ph][cb][j][group][lane]
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if ((i < 4) != (kh == 0))
#pragma unroll
        for (int j = 0; j < 2; ++j) red[(((ph * 2 + cb) * 2 + j) * 7 + i) * 64 + lane] = acc[i][j];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if ((i < 4) == (kh == 0))
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4 o = red[(((ph * 2 + cb) * 2 + j) * 7 + i) * 64 + lane];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) acc[i][j][rr] += o[rr];
        }
    __syncthreads();  // partials consumed: the region takes the output staging
    if (!DGRAD) {  // partial row 4 t + 2 ph + kh: this wave's finalised groups
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        float s = 0.f, sq = 0.f;
#pragma unroll
        for (int i = 0; i < 7; ++i)
          if ((i < 4) == (kh == 0))
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
              s += acc[i][j][rr];
              sq += acc[i][j][rr] * acc[i][j][rr];
            }
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        sq += __shfl_xor(sq, 16);
        sq += __shfl_xor(sq, 32);
        if (g == 0) {
          const size_t o = (size_t)(4 * t + 2 * ph + kh) * C + 32 * cb + 16 * j + cl;
          psum[o] = s;
          psq[o] = sq;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if ((i < 4) == (kh == 0))
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            *(unsigned short*)(Ps + (16 * (7 * ph + i) + 4 * g + rr) * 128 + (32 * cb + 16 * j + cl) * 2) =
                tobf(acc[i][j][rr]);
    __syncthreads();
    if (!DGRAD) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // 224 px x 8 chunks, 16-B coalesced stores
        const int e = tid + 512 * k, p = e >> 3, c = e & 7;
        if (e < NPX2 * 8)
          *(bf16x8*)(y + (((size_t)n * H + oh0 + p / TW) * W + ow0 + p % TW) * C + c * 8) =
              *(const bf16x8*)(Ps + p * 128 + c * 16);
      }
    } else {
      float cs[8], cq[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) cs[u] = cq[u] = 0.f;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = tid + 512 * k, p = e >> 3;
        if (e >= NPX2 * 8) continue;
        bf16x8 o = *(const bf16x8*)(Ps + p * 128 + ec * 16);
        if (fused) {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const float yy = __uint_as_float((unsigned)(unsigned short)ysv[k][u] << 16);
            const float d = yy > 0.f ? __uint_as_float((unsigned)(unsigned short)o[u] << 16) : 0.f;
            o[u] = yy > 0.f ? o[u] : (short)0;
            const float xx = __uint_as_float((unsigned)(unsigned short)xsv[k][u] << 16);
            cs[u] += d;
            cq[u] += d * (xx - mu[u]) * rs[u];
          }
        }
        __builtin_nontemporal_store(o, (bf16x8*)(y + (((size_t)n * H + oh0 + p / TW) * W + ow0 + p % TW) * C + ec * 8));
      }
      if (fused) {  // lanes of one chunk: lane & 7 equal -> partial row of this wave
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          cs[u] += __shfl_xor(cs[u], 8);
          cs[u] += __shfl_xor(cs[u], 16);
          cs[u] += __shfl_xor(cs[u], 32);
          cq[u] += __shfl_xor(cq[u], 8);
          cq[u] += __shfl_xor(cq[u], 16);
          cq[u] += __shfl_xor(cq[u], 32);
        }
        if (lane < 8) {
          const size_t o = (size_t)(8 * t + wave) * C + ec * 8;
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            psum[o + u] = cs[u];
            psq[o + u] = cq[u];
          }
        }
      }
    }
  }
}

// Weight gradient dW[co][k] (+)= sum_p dy[p][co] * x[p + tap][ci], k = tap * 64 + ci: per
// 4 x 28 tile the dy tile (112 px x 64 co, 144-B rows) and the input patch are staged once
// (prefetched a tile ahead); M = 64 co x N = 576 (36 blocks of 16 = tap x channel quarter)
// x K = 112 pixels (+16 zero pixels: 4 k-groups of 32).  Both operands are k-strided, read
// with ds_read_b64_tr_b16 from per-lane pixel rows; wave w owns n-blocks w, w + 8, ... (4-5
// blocks) x all 4 co blocks; a persistent block sums its tiles in registers and adds its
// 64 x 576 partial with one f32 atomic per element at the end.
constexpr int DP = 144;  // dy tile row pitch (bytes)

__device__ __forceinline__ bf16x8 tr_pair(const char* a0, const char* a1) {
  typedef short bf16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) bf16x4 lds4;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)a0);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds4*)a1);
  bf16x8 v;
  v.lo = lo;
  v.hi = hi;
  return v;
}

__global__ __launch_bounds__(512, 1) void conv3x3_c64_wgrad_kernel(
    int N, int H, int W, const unsigned short* __restrict__ x, const unsigned short* __restrict__ dy,
    float* __restrict__ dw, int ldw) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Ds = sm;             // [128 px][64 co] (rows >= 112 zero)
  char* Ps = sm + 128 * DP;  // patch, swizzled 16-B chunks as in the forward
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_w = W / TW, tiles_img = (H / TH) * tiles_w, tiles = N * tiles_img;
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int nnb = wave < 4 ? 5 : 4;  // n-blocks w + 8 j, j < nnb (36 blocks over 8 waves)
  for (int i = tid; i < 16 * 8; i += 512)  // the 16 pad pixel rows of the dy tile stay zero
    *(bf16x8*)(Ds + (NPX + (i >> 3)) * DP + (i & 7) * 16) = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  f32x4 acc[4][5];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 5; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 dv[2], pv[3];
  auto load_tile = [&](int tt) {
    const int n = tt / tiles_img, r = tt - n * tiles_img;
    const int oh0 = (r / tiles_w) * TH, ow0 = (r % tiles_w) * TW;
#pragma unroll
    for (int k = 0; k < 2; ++k) {  // dy: 112 px x 8 chunks = 896 over 512 threads
      const int e = tid + 512 * k, p = e >> 3, c = e & 7;
      dv[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (e < NPX * 8)
        dv[k] = *(const bf16x8*)(dy + (((size_t)n * H + oh0 + p / TW) * W + ow0 + p % TW) * C + c * 8);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int e = tid + 512 * k, qq = e >> 3, c = e & 7, pr = qq / PW, pc = qq - pr * PW;
      const int ih = oh0 - 1 + pr, iw = ow0 - 1 + pc;
      pv[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (e < PCH && ih >= 0 && ih < H && iw >= 0 && iw < W)
        pv[k] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * C + c * 8);
    }
  };
  if (blockIdx.x < tiles) load_tile(blockIdx.x);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + 512 * k;
      if (e < NPX * 8) *(bf16x8*)(Ds + (e >> 3) * DP + (e & 7) * 16) = dv[k];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int e = tid + 512 * k, qq = e >> 3, c = e & 7;
      if (e < PCH) *(bf16x8*)(Ps + qq * 128 + ((c ^ (qq & 7)) << 4)) = pv[k];
    }
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_tile(t + gridDim.x);
#pragma unroll
    for (int kg = 0; kg < 4; ++kg) {
      const int k0 = 32 * kg + 8 * g + q, k1 = k0 + 4;  // this lane's two pixel rows
      bf16x8 a[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = tr_pair(Ds + k0 * DP + (16 * i + 4 * p4) * 2, Ds + k1 * DP + (16 * i + 4 * p4) * 2);
      // patch pixel of tap (0, 0) for the two pixel rows (pad pixels >= 112: any valid pixel,
      // their dy rows are zero)
      const int pk0 = min(k0, NPX - 1), pk1 = min(k1, NPX - 1);
      const int pb0 = (pk0 / TW) * PW + pk0 % TW, pb1 = (pk1 / TW) * PW + pk1 % TW;
#pragma unroll
      for (int j = 0; j < 5; ++j) {
        if (j < nnb) {
          const int nb = wave + 8 * j, tap = nb >> 2, kh = tap / 3, kw = tap - kh * 3;
          const int ch = (nb & 3) * 16 + 4 * p4;  // this lane's 4 channels
          const int q0 = pb0 + kh * PW + kw, q1 = pb1 + kh * PW + kw;
          const int off = (ch & 7) * 2;  // byte offset inside the 16-B chunk
          const bf16x8 b = tr_pair(Ps + q0 * 128 + (((ch >> 3) ^ (q0 & 7)) << 4) + off,
                                   Ps + q1 * 128 + (((ch >> 3) ^ (q1 & 7)) << 4) + off);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b, acc[i][j], 0, 0, 0);
        }
      }
    }
  }
  // lane (cl, g): column n = cl of block nb (k = tap * 64 + 16 (nb & 3) + cl), co 16 i + 4 g + rr
  const int cl = lane & 15;
#pragma unroll
  for (int j = 0; j < 5; ++j) {
    if (j >= nnb) continue;
    const int nb = wave + 8 * j, k = (nb >> 2) * C + (nb & 3) * 16 + cl;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        unsafeAtomicAdd(dw + (size_t)(16 * i + 4 * g + rr) * ldw + k, acc[i][j][rr]);
  }
}


}  // namespace c3

bool conv3x3_c64_applies(int H, int W, int C, int Cout, int KH, int KW, int stride, int pad) {
  return C == c3::C && Cout == c3::C && KH == 3 && KW == 3 && stride == 1 && pad == 1 &&
         H % c3::TH2 == 0 && W % c3::TW == 0;
}

// dx (+ fused BN backward when relu_y is given: psum / psq partial rows [8 * tiles][64],
// tiles = N*H*W / 224)
void conv3x3_c64_dgrad_launch(int N, int H, int W, const void* dy, const void* w, int ldw, void* dx,
                              const void* relu_y, const void* bn_x, const float* bn_mean,
                              const float* bn_rstd, float* psum, float* psq, void* wf, hipStream_t s) {
  using namespace c3;
  if (!conv3x3_c64_applies(H, W, C, C, 3, 3, 1, 1))
    throw std::runtime_error("conv3x3_c64: unsupported geometry");
  if (ldw < 9 * C || !wf ||
      (((uintptr_t)dy | (uintptr_t)dx | (uintptr_t)relu_y | (uintptr_t)bn_x | (uintptr_t)wf) & 15))
    throw std::runtime_error("conv3x3_c64_dgrad: ld >= 576, a [64][576] bf16 workspace wf, 16-B aligned tensors");
  if (relu_y && (!bn_x || !bn_mean || !bn_rstd || !psum || !psq))
    throw std::runtime_error("conv3x3_c64_dgrad: fused BN backward needs bn_x, mean, rstd, partials");
  const int tiles = N * (H / TH2) * (W / TW);
  const size_t lds = W_BYTES + R_BYTES;
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_c64_kernel<true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int blocks = std::min(tiles, 256);
  hipLaunchKernelGGL(conv3x3_c64_flip_kernel, dim3((C * 9 * C + 255) / 256), dim3(256), 0, s,
                     (const unsigned short*)w, ldw, (unsigned short*)wf);
  hipLaunchKernelGGL(conv3x3_c64_kernel<true>, dim3(blocks), dim3(512), lds, s, N, H, W,
                     (const unsigned short*)dy, (const unsigned short*)wf, 9 * C, (unsigned short*)dx,
                     (const unsigned short*)relu_y, (const unsigned short*)bn_x, bn_mean, bn_rstd,
                     psum, psq);
  DTFX_HIP_CHECK(hipGetLastError());
}

// dw (f32 [64][ldw], the first 576 columns) (+)= the weight gradient: beta 1 accumulates,
// beta 0 overwrites.
void conv3x3_c64_wgrad_launch(int N, int H, int W, const void* x, const void* dy, float* dw,
                              int ldw, float beta, hipStream_t s) {
  using namespace c3;
  if (!conv3x3_c64_applies(H, W, C, C, 3, 3, 1, 1))
    throw std::runtime_error("conv3x3_c64: unsupported geometry");
  if (ldw < 9 * C || (((uintptr_t)x | (uintptr_t)dy) & 15))
    throw std::runtime_error("conv3x3_c64_wgrad: ld >= 576 and 16-B aligned inputs");
  if (beta != 0.f && beta != 1.f) throw std::runtime_error("conv3x3_c64_wgrad: beta must be 0 or 1");
  if (beta == 0.f)
    DTFX_HIP_CHECK(hipMemset2DAsync(dw, sizeof(float) * ldw, 0, sizeof(float) * 9 * C, C, s));
  const int tiles = N * (H / TH) * (W / TW);
  const size_t lds = 128 * DP + P_BYTES;
  const int blocks = std::min(tiles, 256);
  hipLaunchKernelGGL(conv3x3_c64_wgrad_kernel, dim3(blocks), dim3(512), lds, s, N, H, W,
                     (const unsigned short*)x, (const unsigned short*)dy, dw, ldw);
  DTFX_HIP_CHECK(hipGetLastError());
}

// y = conv3x3(x, w), psum / psq: partial statistic rows [4 * tiles][64] (tiles = N*H*W / 224)
// coef / xo (both or neither): x is the previous conv's raw output and relu(bn(x)) (coef: the
// [4][64] bn_fwd_coef rows) is formed as the patch is staged and written to xo.
void conv3x3_c64_fwd_launch(int N, int H, int W, const void* x, const void* w, int ldw, void* y,
                            float* psum, float* psq, hipStream_t s, const float* coef, void* xo) {
  using namespace c3;
  if (!conv3x3_c64_applies(H, W, C, C, 3, 3, 1, 1))
    throw std::runtime_error("conv3x3_c64: unsupported geometry");
  if (ldw < 9 * C || ldw % 8 || (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)xo) & 15))
    throw std::runtime_error("conv3x3_c64: weights need ld >= 576 (% 8), 16-B aligned tensors");
  if ((coef != nullptr) != (xo != nullptr))
    throw std::runtime_error("conv3x3_c64: the BN prologue needs both coef and xo");
  const int tiles = N * (H / TH2) * (W / TW);
  const size_t lds = W_BYTES + R_BYTES;
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_c64_kernel<false>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_c64_kernel<false, true>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int blocks = std::min(tiles, 256);
  auto k = coef ? conv3x3_c64_kernel<false, true> : conv3x3_c64_kernel<false, false>;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(512), lds, s, N, H, W, (const unsigned short*)x,
                     (const unsigned short*)w, ldw, (unsigned short*)y, nullptr, nullptr, nullptr,
                     nullptr, psum, psq, coef, (unsigned short*)xo);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
