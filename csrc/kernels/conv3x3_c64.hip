// 3x3 / stride 1 / pad 1 convolution forward with 64 input and 64 output channels (ResNet-50
// layer1's conv2 at 56 x 56), NHWC bf16, BatchNorm statistics of the output fused (partial
// rows, reduced by colpart_reduce).
//
// The stem's scheme (stem_conv.hip) applied to layer1: all 64 x 576 weights stay in LDS for a
// persistent block's life, and per 4 x 28-pixel output tile the 6 x 30-pixel input patch is
// staged ONCE (prefetched a tile ahead into registers), so the MFMA A fragments of every tap
// are read from the patch at the tap's offset instead of re-gathering each input pixel nine
// times through L2 (the implicit GEMM's 256x64 tile: 181 us per call at batch 256, against
// ~32 us of HBM traffic).  Patch pixels are 128-B rows of 8 16-B channel chunks, chunk c of
// pixel q stored at c ^ (q & 7): the 16 lanes of a fragment read 16 consecutive pixels.
//
// k-group kg = (tap kg / 2, channel half kg % 2): 18 groups of 32.  8 waves: wave w owns
// output channels 16 (w & 3) .. + 15 and pixel groups (of 16) 0-3 (w < 4) or 4-6.
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

__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

__global__ __launch_bounds__(512, 1) void conv3x3_c64_fwd_kernel(
    int N, int H, int W, const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
    int ldw, unsigned short* __restrict__ y, float* __restrict__ psum, float* __restrict__ psq) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Ws = sm;
  char* Ps = sm + W_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < C * 72; i += 512) {  // weights [64 co][576 k], once
    const int co = i / 72, c = i - co * 72;
    *(bf16x8*)(Ws + co * WP * 2 + c * 16) = *(const bf16x8*)(w + (size_t)co * ldw + c * 8);
  }
  const int tiles_w = W / TW, tiles_img = (H / TH) * tiles_w, tiles = N * tiles_img;
  const int cl = lane & 15, g = lane >> 4;
  const int cb = wave & 3;                         // output channel block
  const int g0 = wave < 4 ? 0 : 4, ng = wave < 4 ? 4 : 3;  // pixel groups of this wave
  bf16x8 v[3];  // patch chunks of the next tile: 1440 / 512 -> 3 per thread
  auto load_patch = [&](int tt) {
    const int n = tt / tiles_img, r = tt - n * tiles_img;
    const int ih0 = (r / tiles_w) * TH - 1, iw0 = (r % tiles_w) * TW - 1;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int e = tid + 512 * k, q = e >> 3, c = e & 7, pr = q / PW, pc = q - pr * PW;
      const int ih = ih0 + pr, iw = iw0 + pc;
      v[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (e < PCH && ih >= 0 && ih < H && iw >= 0 && iw < W)
        v[k] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * C + c * 8);
    }
  };
  if (blockIdx.x < tiles) load_patch(blockIdx.x);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int n = t / tiles_img, r = t - n * tiles_img;
    const int oh0 = (r / tiles_w) * TH, ow0 = (r % tiles_w) * TW;
    __syncthreads();  // the previous tile's output staging is done
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int e = tid + 512 * k, q = e >> 3, c = e & 7;
      if (e < PCH) *(bf16x8*)(Ps + q * 128 + ((c ^ (q & 7)) << 4)) = v[k];
    }
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_patch(t + gridDim.x);
    // this lane's pixel in each of its groups: patch pixel of tap (0, 0)
    int pq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = 16 * (g0 + i) + cl;
      pq[i] = (p / TW) * PW + (p % TW);
    }
    f32x4 acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int kg = 0; kg < 18; ++kg) {
      const int tap = kg >> 1, kh = tap / 3, kw = tap - kh * 3, chunk = (kg & 1) * 4 + g;
      const bf16x8 b = *(const bf16x8*)(Ws + (16 * cb + cl) * WP * 2 + (32 * kg + 8 * g) * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < ng) {
          const int q = pq[i] + kh * PW + kw;
          const bf16x8 a = *(const bf16x8*)(Ps + q * 128 + ((chunk ^ (q & 7)) << 4));
          acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[i], 0, 0, 0);
        }
      }
    }
    // BN statistics (f32 values): lane (cl, g) holds channel 16 cb + cl of pixels 4 g + rr
    {
      float s = 0.f, sq = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (i < ng)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            s += acc[i][rr];
            sq += acc[i][rr] * acc[i][rr];
          }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      sq += __shfl_xor(sq, 16);
      sq += __shfl_xor(sq, 32);
      if (g == 0) {  // partial row 2 t + (pixel half), channels of this wave's block
        const size_t o = (size_t)(2 * t + (wave >> 2)) * C + 16 * cb + cl;
        psum[o] = s;
        psq[o] = sq;
      }
    }
    __syncthreads();  // every wave is done with the patch: stage the output there
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < ng)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
          *(unsigned short*)(Ps + (16 * (g0 + i) + 4 * g + rr) * 128 + (16 * cb + cl) * 2) =
              tobf(acc[i][rr]);
    __syncthreads();
    for (int e = tid; e < NPX * 8; e += 512) {  // 112 px x 8 chunks, 16-B coalesced stores
      const int p = e >> 3, c = e & 7;
      const int oh = oh0 + p / TW, ow = ow0 + p % TW;
      *(bf16x8*)(y + (((size_t)n * H + oh) * W + ow) * C + c * 8) = *(const bf16x8*)(Ps + p * 128 + c * 16);
    }
  }
}

}  // namespace c3

bool conv3x3_c64_applies(int H, int W, int C, int Cout, int KH, int KW, int stride, int pad) {
  return C == c3::C && Cout == c3::C && KH == 3 && KW == 3 && stride == 1 && pad == 1 &&
         H % c3::TH == 0 && W % c3::TW == 0;
}

// y = conv3x3(x, w), psum / psq: partial statistic rows [2 * tiles][64] (tiles = N*H*W / 112)
void conv3x3_c64_fwd_launch(int N, int H, int W, const void* x, const void* w, int ldw, void* y,
                            float* psum, float* psq, hipStream_t s) {
  using namespace c3;
  if (!conv3x3_c64_applies(H, W, C, C, 3, 3, 1, 1))
    throw std::runtime_error("conv3x3_c64: unsupported geometry");
  if (ldw < 9 * C || ldw % 8 || (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) & 15))
    throw std::runtime_error("conv3x3_c64: weights need ld >= 576 (% 8), 16-B aligned tensors");
  const int tiles = N * (H / TH) * (W / TW);
  const size_t lds = W_BYTES + P_BYTES;
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv3x3_c64_fwd_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int blocks = std::min(tiles, 256);
  hipLaunchKernelGGL(conv3x3_c64_fwd_kernel, dim3(blocks), dim3(512), lds, s, N, H, W,
                     (const unsigned short*)x, (const unsigned short*)w, ldw, (unsigned short*)y,
                     psum, psq);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
