// 3x3 / stride 1 / pad 1 convolution with 128 input and 128 output channels at 28 x 28 (ResNet-50
// layer2's conv2): forward with the fused BatchNorm statistics, and the data gradient with the
// fused BatchNorm backward, NHWC bf16.
//
// conv3x3_c64.hip's staged patch with the weights STREAMED: the 128 x 1152 weights (295 KB) do
// not fit in LDS, so a persistent block keeps one 6 x 30-pixel input patch (4 x 28 output
// tile, 48 KB, prefetched a tile ahead into registers) and double-buffers the 128 x 128 weight
// slice of one tap at a time (34 KB each, the next tap's slice loaded into registers during the
// current tap's MFMAs).  Every input
// pixel is read from HBM / L2 once per tile instead of once per tap.  Patch pixels are 272-B
// rows (256 B of channels + 16 B pad).
//
// The data gradient of a stride-1 3x3 conv is the forward conv of dy with the kernel flipped
// and transposed, W'[ci][tap][co] = W[co][8 - tap][ci]: conv3x3_c128_flip builds W' once per
// call into a workspace, then the same kernel runs with the BN-backward epilogue.
//
// 8 waves: wave w owns output channels 32 (w & 3) .. + 31 and input-channel half w >> 2 (the K
// split) for all 7 pixel groups (of 16): 14 MFMA tiles, per k-group 7 A + 2 B fragment reads for
// 14 MFMAs.  The first version (wave = 16 output channels x the whole K: 7 A + 1 B reads per 7
// MFMAs) was LDS-bandwidth-bound at ~2.3x its MFMA time (every A fragment read fed one MFMA).
// The two K halves are summed through LDS after the last tap: wave (cb, 0) finalises pixel
// groups 0-3, wave (cb, 1) groups 4-6, each writing the other's groups first.
#include "common.h"

#include <algorithm>
#include <stdexcept>

namespace dtfx {
namespace c3b {

typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int C = 128, TH = 4, TW = 28, PH = TH + 2, PW = TW + 2;  // 6 x 30 patch
constexpr int NPX = TH * TW;                                      // 112 = 7 groups of 16
constexpr int NCH = C / 8;                                        // 16 chunks per pixel
constexpr int PP = C * 2 + 16;                                    // patch pixel pitch 272 B
constexpr int P_BYTES = PH * PW * PP;                             // 48960
constexpr int PCH = PH * PW * NCH;                                // 2880 patch chunks
constexpr int WT_PITCH = C * 2 + 16;                              // 272 B per weight row
constexpr int WT_BYTES = C * WT_PITCH;                            // 34816 per tap slice
constexpr int R_BYTES = 4 * 2 * 7 * 64 * 16;                       // K-half partials 57344
constexpr int S_BYTES = R_BYTES > P_BYTES ? R_BYTES : P_BYTES;     // patch / partials / staging
constexpr int LDS = S_BYTES + 2 * WT_BYTES;                       // 126976

__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float bf(short h) { return __uint_as_float((unsigned)(unsigned short)h << 16); }

// W' [ci][tap * 128 + co] = W [co][(8 - tap) * 128 + ci]
__global__ __launch_bounds__(256) void conv3x3_c128_flip_kernel(const unsigned short* __restrict__ w,
                                                                int ldw, unsigned short* __restrict__ wf) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // output element
  if (i >= C * 9 * C) return;
  const int ci = i / (9 * C), rem = i - ci * 9 * C, tap = rem / C, co = rem - tap * C;
  wf[i] = w[(size_t)co * ldw + (8 - tap) * C + ci];
}

template <bool DGRAD>
__global__ __launch_bounds__(512, 1) void conv3x3_c128_kernel(
    int N, int H, int W, const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
    int ldw, unsigned short* __restrict__ y, const unsigned short* __restrict__ relu_y,
    const unsigned short* __restrict__ bn_x, const float* __restrict__ bn_mean,
    const float* __restrict__ bn_rstd, float* __restrict__ psum, float* __restrict__ psq) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Ps = sm;
  char* Wt = sm + S_BYTES;  // [2][128 co][272 B]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_w = W / TW, tiles_img = (H / TH) * tiles_w, tiles = N * tiles_img;
  const int cl = lane & 15, g = lane >> 4;
  const int cb = wave & 3, kh = wave >> 2;  // 32 output channels, input-channel half
  bf16x8 pv[6], wv[4];
  int lpr[6], lpc[6];  // patch rows / columns of this thread's chunks (tile-invariant)
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int q = (tid + 512 * k) >> 4;
    lpr[k] = q / PW;
    lpc[k] = q - lpr[k] * PW;
  }
  auto load_patch = [&](int tt) {
    const int n = tt / tiles_img, r = tt - n * tiles_img;
    const int ih0 = (r / tiles_w) * TH - 1, iw0 = (r % tiles_w) * TW - 1;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int e = tid + 512 * k, c = e & 15;
      const int ih = ih0 + lpr[k], iw = iw0 + lpc[k];
      pv[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (e < PCH && ih >= 0 && ih < H && iw >= 0 && iw < W)
        pv[k] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * C + c * 8);
    }
  };
  auto load_w = [&](int tap) {  // the 128 x 128 slice of one tap: 2048 chunks, 4 per thread
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = tid + 512 * k, co = e >> 4, c = e & 15;
      wv[k] = *(const bf16x8*)(w + (size_t)co * ldw + tap * C + c * 8);
    }
  };
  auto store_w = [&](int buf) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = tid + 512 * k, co = e >> 4, c = e & 15;
      *(bf16x8*)(Wt + buf * WT_BYTES + co * WT_PITCH + c * 16) = wv[k];
    }
  };
  // A fragment addresses of tap (0, 0): this lane's pixel in each group, its chunk of input
  // half kh.  Patch pixels are 272-B rows (16 consecutive pixels: 16 distinct 16-B bank
  // slots), so a tap is one uniform offset and a k-group an immediate.
  int abase[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    const int p = 16 * i + cl;
    abase[i] = ((p / TW) * PW + (p % TW)) * PP + (8 * kh + g) * 16;
  }
  int buf = 0;
  if (blockIdx.x < tiles) {
    load_w(0);
    store_w(0);
    load_patch(blockIdx.x);
  }
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int n = t / tiles_img, r = t - n * tiles_img;
    const int oh0 = (r / tiles_w) * TH, ow0 = (r % tiles_w) * TW;
    __syncthreads();  // the previous tile's output staging is consumed
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int e = tid + 512 * k, q = e >> 4, c = e & 15;
      if (e < PCH) *(bf16x8*)(Ps + q * PP + c * 16) = pv[k];
    }
    __syncthreads();
    const bool more = t + (int)gridDim.x < tiles;
    if (more) load_patch(t + gridDim.x);
    f32x4 acc[7][2];
#pragma unroll
    for (int i = 0; i < 7; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // data gradient: the epilogue's side inputs, requested with the last tap (in flight during
    // its MFMAs and the K-half reduction)
    const int ec = tid & 15;
    const bool fused = DGRAD && relu_y != nullptr;
    bf16x8 ysv[4], xsv[4];
#pragma unroll 1
    for (int tap = 0; tap < 9; ++tap) {
      const bool next_w = tap < 8 || more;
      if (next_w) load_w(tap < 8 ? tap + 1 : 0);
      if (fused && tap == 8) {  // after the weight loads: their wait leaves these in flight
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int e = tid + 512 * k, p = e >> 4;
          if (e < NPX * NCH) {
            const size_t go = (((size_t)n * H + oh0 + p / TW) * W + ow0 + p % TW) * C + ec * 8;
            ysv[k] = *(const bf16x8*)(relu_y + go);
            xsv[k] = *(const bf16x8*)(bn_x + go);
          }
        }
      }
      const int th = tap / 3, tw = tap - th * 3, toff = (th * PW + tw) * PP;
      const char* wb = Wt + buf * WT_BYTES + (32 * cb + cl) * WT_PITCH + (64 * kh + 8 * g) * 2;
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const bf16x8 b0 = *(const bf16x8*)(wb + k2 * 64);
        const bf16x8 b1 = *(const bf16x8*)(wb + 16 * WT_PITCH + k2 * 64);
#pragma unroll
        for (int i = 0; i < 7; ++i) {
          const bf16x8 a = *(const bf16x8*)(Ps + abase[i] + toff + k2 * 64);
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc[i][1], 0, 0, 0);
        }
      }
      if (next_w) store_w(buf ^ 1);
      __syncthreads();  // the next slice is in; every wave is done with this one
      buf ^= 1;
    }
    // K halves: write the partner's pixel groups, then add the partner's partials of ours
    f32x4* red = (f32x4*)sm;  // [cb][j][group][lane]
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if ((i < 4) != (kh == 0))
#pragma unroll
        for (int j = 0; j < 2; ++j) red[((cb * 2 + j) * 7 + i) * 64 + lane] = acc[i][j];
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if ((i < 4) == (kh == 0))
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const f32x4 o = red[((cb * 2 + j) * 7 + i) * 64 + lane];
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) acc[i][j][rr] += o[rr];
        }
    __syncthreads();  // partials consumed: the region takes the output staging
    if (!DGRAD) {  // BN statistics of the f32 values: partial row 2 t + kh (this wave's groups)
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
          const size_t o = (size_t)(2 * t + kh) * C + 32 * cb + 16 * j + cl;
          psum[o] = s;
          psq[o] = sq;
        }
      }
    }
    // output staging in the patch region
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if ((i < 4) == (kh == 0))
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            *(unsigned short*)(Ps + (16 * i + 4 * g + rr) * 256 + (32 * cb + 16 * j + cl) * 2) =
                tobf(acc[i][j][rr]);
    __syncthreads();
    if (!DGRAD) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // 112 px x 16 chunks
        const int e = tid + 512 * k, p = e >> 4, c = e & 15;
        if (e < NPX * NCH)
          *(bf16x8*)(y + (((size_t)n * H + oh0 + p / TW) * W + ow0 + p % TW) * C + c * 8) =
            *(const bf16x8*)(Ps + p * 256 + c * 16);
      }
    } else {
      // BN backward: de = dx * (relu_y > 0); sum(de), sum(de * xhat) for this thread's chunk
      // (ec = tid & 15 for every k), reduced over the wave, one partial row per wave and tile
      float cs[8], cq[8], mu[8], rs[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        cs[u] = cq[u] = 0.f;
        mu[u] = fused ? bn_mean[ec * 8 + u] : 0.f;
        rs[u] = fused ? bn_rstd[ec * 8 + u] : 0.f;
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = tid + 512 * k, p = e >> 4;
        if (e >= NPX * NCH) continue;
        const size_t go = (((size_t)n * H + oh0 + p / TW) * W + ow0 + p % TW) * C + ec * 8;
        bf16x8 o = *(const bf16x8*)(Ps + p * 256 + ec * 16);
        if (fused) {
          const bf16x8 yv = ysv[k], xv = xsv[k];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            const bool pos = bf(yv[u]) > 0.f;
            if (!pos) o[u] = 0;
            const float d = bf(o[u]);
            cs[u] += d;
            cq[u] += d * (bf(xv[u]) - mu[u]) * rs[u];
          }
        }
        __builtin_nontemporal_store(o, (bf16x8*)(y + go));
      }
      if (fused) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          cs[u] += __shfl_xor(cs[u], 16);
          cs[u] += __shfl_xor(cs[u], 32);
          cq[u] += __shfl_xor(cq[u], 16);
          cq[u] += __shfl_xor(cq[u], 32);
        }
        if (lane < 16) {
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

}  // namespace c3b

bool conv3x3_c128_applies(int H, int W, int C, int Cout, int KH, int KW, int stride, int pad) {
  return C == c3b::C && Cout == c3b::C && KH == 3 && KW == 3 && stride == 1 && pad == 1 &&
         H % c3b::TH == 0 && W % c3b::TW == 0;
}

// mode 1: y = conv(x, w), psum / psq partial statistic rows [2 * tiles][128];
// mode 2: y = dx of dy = x (w flipped into wf, [128][1152] bf16 workspace), with relu_y given
//         the fused BN backward, psum / psq partial rows [8 * tiles][128]
// (tiles = N * H * W / 112)
void conv3x3_c128_launch(int mode, int N, int H, int W, const void* x, const void* w, int ldw,
                         void* y, void* wf, const void* relu_y, const void* bn_x,
                         const float* bn_mean, const float* bn_rstd, float* psum, float* psq,
                         hipStream_t s) {
  using namespace c3b;
  if (!conv3x3_c128_applies(H, W, C, C, 3, 3, 1, 1))
    throw std::runtime_error("conv3x3_c128: unsupported geometry");
  if (ldw < 9 * C || ldw % 8 ||
      (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)wf | (uintptr_t)relu_y |
        (uintptr_t)bn_x) & 15))
    throw std::runtime_error("conv3x3_c128: ld >= 1152 (% 8) and 16-B aligned tensors");
  const int tiles = N * (H / TH) * (W / TW);
  const int blocks = std::min(tiles, 256);
  if (mode == 1) {
    static bool attr = false;
    if (!attr) {
      DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_c128_kernel<false>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
      attr = true;
    }
    hipLaunchKernelGGL(conv3x3_c128_kernel<false>, dim3(blocks), dim3(512), LDS, s, N, H, W,
                       (const unsigned short*)x, (const unsigned short*)w, ldw, (unsigned short*)y,
                       nullptr, nullptr, nullptr, nullptr, psum, psq);
  } else {
    if (!wf) throw std::runtime_error("conv3x3_c128: dgrad needs the flipped-weight workspace");
    hipLaunchKernelGGL(conv3x3_c128_flip_kernel, dim3((C * 9 * C + 255) / 256), dim3(256), 0, s,
                       (const unsigned short*)w, ldw, (unsigned short*)wf);
    static bool attr = false;
    if (!attr) {
      DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_c128_kernel<true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, LDS));
      attr = true;
    }
    hipLaunchKernelGGL(conv3x3_c128_kernel<true>, dim3(blocks), dim3(512), LDS, s, N, H, W,
                       (const unsigned short*)x, (const unsigned short*)wf, 9 * C,
                       (unsigned short*)y, (const unsigned short*)relu_y,
                       (const unsigned short*)bn_x, bn_mean, bn_rstd, psum, psq);
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
