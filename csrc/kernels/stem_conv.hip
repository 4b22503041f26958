// ResNet-50 stem convolution forward (7x7, stride 2, pad 3, 8 input channels -- the image's
// 3 + 5 zero channels -- 64 output channels), NHWC bf16, with the BatchNorm statistics of the
// output fused (partial rows, one per 32 output pixels, reduced by colpart_reduce).
//
// Why a kernel of its own: as an implicit GEMM (gemm_bf16.hip MODE 1, 256x64 tile) the stem
// gathers every input pixel once per tap it feeds -- 49 taps x 16 B per output pixel through
// L2 -- and ran 606 us at ResNet-50's 256x224x224 input (MI355X), against ~95 us of HBM
// traffic (205 MB in, 411 MB out).  Here a persistent block keeps all 64 x 392 weights in LDS
// for its whole life and, per 8 x 16-pixel output tile, stages the 21 x 37-pixel input patch
// the tile reads ONCE (12 KB); the MFMA A fragments (16 output pixels x 4 taps x 8 channels)
// are read from the patch at the tap's offset, so nothing is re-fetched per tap.
//
// MFMA v_mfma_f32_16x16x32_bf16: k-group kg = taps 4kg..4kg+3 x 8 channels (13 groups, taps
// 49-51 zero weights); wave w owns output rows 2w, 2w+1 of the tile (2 x 16 pixels) x 64
// channels = 2 x 4 accumulator tiles.
#include "common.h"

#include <algorithm>
#include <stdexcept>

namespace dtfx {
namespace stem {

typedef short bf16x8 __attribute__((ext_vector_type(8)));

constexpr int KS = 7, STR = 2, PAD = 3, CIN = 8, COUT = 64;
constexpr int TH = 8, TW = 16;                                  // output tile
constexpr int PR = (TH - 1) * STR + KS, PC = (TW - 1) * STR + KS;  // 21 x 37 input patch
constexpr int NKG = 13;                                        // k-groups of 4 taps
constexpr int WP = 456;                                        // weight row pitch (bf16): 912 B
constexpr int W_BYTES = COUT * WP * 2;                         // 58368
constexpr int P_BYTES = 16384;  // patch (777 x 16 B) / output staging (4 waves x 32 px x 128 B)

__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}

// Forward tiles: 16 x 16 output pixels, wave w owns output rows 4w..4w+3 (4 A fragments of
// 16 pixels) x 64 channels (4 B fragments): 8 LDS fragment reads per 16 MFMAs (the first
// version's 8 x 16 tiles with 2 rows per wave read 6 per 8 and were LDS-bound).  The 37 x 37
// input patch is stored column-parity-major ([row][even columns | odd columns]) so the 16
// lanes of a fragment, which read every second patch column, hit 16 consecutive 16-B slots.
// A last tile row of an OH % 16 != 0 image is partial: rows >= OH are masked.
constexpr int FTH = 16;                                        // forward output tile rows
constexpr int FPR = (FTH - 1) * STR + KS;                      // 37 patch rows
constexpr int FPH = (PC + 1) / 2;                              // 19 even-column slots per row
constexpr int FPP = 2 * FPH;                                   // 38 slots per patch row
constexpr int FP_BYTES = FPR * FPP * 16;                       // 22496 (output staging: 16 KB)

__global__ __launch_bounds__(256, 2) void stem_conv_fwd_kernel(
    int N, int H, int W, int OH, int OW, const unsigned short* __restrict__ x,
    const unsigned short* __restrict__ w, int ldw, unsigned short* __restrict__ y,
    float* __restrict__ psum, float* __restrict__ psq) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Ws = sm;
  char* Ps = sm + W_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // weights, once: [64 co][448 k] -> 912-B rows (k >= 392 are the zero pad of the layout)
  for (int i = tid; i < COUT * 56; i += 256) {
    const int co = i / 56, c = i - co * 56;
    *(bf16x8*)(Ws + co * WP * 2 + c * 16) = *(const bf16x8*)(w + (size_t)co * ldw + c * 8);
  }
  const int tiles_w = OW / TW, tiles_h = (OH + FTH - 1) / FTH, tiles_img = tiles_h * tiles_w;
  const int tiles = N * tiles_img;
  const int cl = lane & 15, g = lane >> 4;
  // input patch of tile tt into registers (zero outside the image): 1369 16-B pixels, 6 per
  // thread -- issued one tile ahead, so the loads are in flight during the MFMAs
  bf16x8 v[6];
  int pslot[6];  // LDS slot of each (tile-invariant)
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const int p = tid + 256 * k, pr = p / PC, pc = p - pr * PC;
    pslot[k] = p < FPR * PC ? pr * FPP + (pc & 1) * FPH + (pc >> 1) : -1;
  }
  auto load_patch = [&](int tt) {
    const int n = tt / tiles_img, r = tt - n * tiles_img;
    const int ih0 = (r / tiles_w) * FTH * STR - PAD, iw0 = (r % tiles_w) * TW * STR - PAD;
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      const int p = tid + 256 * k, pr = p / PC, pc = p - pr * PC;
      const int ih = ih0 + pr, iw = iw0 + pc;
      v[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (p < FPR * PC && ih >= 0 && ih < H && iw >= 0 && iw < W)
        v[k] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * CIN);
    }
  };
  if (blockIdx.x < tiles) load_patch(blockIdx.x);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    const int n = t / tiles_img, r = t - n * tiles_img;
    const int oh0 = (r / tiles_w) * FTH, ow0 = (r % tiles_w) * TW;
    __syncthreads();  // the previous tile's output staging (same LDS) is done
#pragma unroll
    for (int k = 0; k < 6; ++k)
      if (pslot[k] >= 0) *(bf16x8*)(Ps + pslot[k] * 16) = v[k];
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_patch(t + gridDim.x);
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kg = 0; kg < NKG; ++kg) {
      const int tap = 4 * kg + g, kh = tap / KS, kw = tap - kh * KS;
      // this lane's pixel: output row 4 wave + i, column cl -> patch row 2 (4 wave + i) + kh,
      // column 2 cl + kw (parity kw & 1, slot cl + kw / 2)
      const int abase = ((8 * wave + kh) * FPP + (kw & 1) * FPH + cl + (kw >> 1)) * 16;
      bf16x8 a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        a[i] = tap < KS * KS ? *(const bf16x8*)(Ps + abase + i * 2 * FPP * 16)
                             : bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = *(const bf16x8*)(Ws + (16 * j + cl) * WP * 2 + (32 * kg + 8 * g) * 2);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    // BN statistics of the f32 values: lane (cl, g) holds channel 16 j + cl of pixels 4 g + rr
    // of output row 4 wave + i; rows past OH (a partial last tile row) are masked
    const int prow = t * 4 + wave;  // one partial row per wave (64 pixels)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float s = 0.f, q = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (oh0 + 4 * wave + i < OH)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr) {
            s += acc[i][j][rr];
            q += acc[i][j][rr] * acc[i][j][rr];
          }
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      q += __shfl_xor(q, 16);
      q += __shfl_xor(q, 32);
      if (g == 0) {
        psum[(size_t)prow * COUT + 16 * j + cl] = s;
        psq[(size_t)prow * COUT + 16 * j + cl] = q;
      }
    }
    __syncthreads();  // every wave is done reading the patch: reuse it for the output
    char* st = Ps + wave * 4096;  // [32 px][64 co] bf16, 128-B rows: two rows per pass
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h) __builtin_amdgcn_wave_barrier();  // (the first pass's reads are done)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int rr = 0; rr < 4; ++rr)
            *(unsigned short*)(st + (16 * i + 4 * g + rr) * 128 + (16 * j + cl) * 2) =
                tobf(acc[2 * h + i][j][rr]);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // 32 px x 8 chunks: 4 per lane, 16 B each, coalesced rows
        const int e = lane + 64 * k, px = e >> 3, c = e & 7;
        const int oh = oh0 + 4 * wave + 2 * h + (px >> 4), ow = ow0 + (px & 15);
        if (oh < OH)
          *(bf16x8*)(y + (((size_t)n * OH + oh) * OW + ow) * COUT + c * 8) =
              *(const bf16x8*)(st + px * 128 + c * 16);
      }
    }
  }
}


// Weight gradient dW[co][k] (+)= sum_p dy[p][co] * x_patch[p][k], k = (kh, kw, c): per
// 8 x 16-pixel tile the dy tile (128 px x 64 co) and the input patch are staged once; the
// GEMM is M = 64 co x N = 7 kh x 4 blocks of 16 (kw pairs x 8 channels: 16 bf16 contiguous in
// a patch row, the 8th kw of the last block discarded) x K = 128 pixels.  Both operands are
// k-strided (k = pixel), read with ds_read_b64_tr_b16 from per-lane row addresses (the
// pixel -> patch offset is not a uniform stride).  Wave w owns n-blocks 7w..7w+6 x all 4
// co blocks (28 accumulator tiles); a persistent block sums all its tiles in registers and
// adds its 64 x 392 partial with one f32 atomic per element at the end.
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

// PRO: dy is the gradient at the stem BatchNorm's output (the masked pool gradient de) and the
// conv output gradient is formed as it is staged, dc = A de + K1 c + K0 (bn_bwd_apply_kernel's
// affine form; coef rows 0, 1, 3 of bn_bwd_coef, c = bnx, the BN input): the apply pass that
// wrote dc and this kernel's read of it become one read of de and c.  A thread's four dy chunks
// share one channel chunk (tid & 7), so its coefficients stay in registers.
template <bool PRO>
__global__ __launch_bounds__(256, 1) void stem_conv_wgrad_kernel(
    int N, int H, int W, int OH, int OW, const unsigned short* __restrict__ x,
    const unsigned short* __restrict__ dy, float* __restrict__ dw, int ldw,
    const unsigned short* __restrict__ bnx, const float* __restrict__ coef) {
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Ds = sm;             // [128 px][64 co] bf16, 144-B rows
  char* Ps = sm + 128 * DP;  // [21][37] pixels x 8 channels
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_w = OW / TW, tiles_img = (OH / TH) * tiles_w;
  const int tiles = N * tiles_img;
  const int g = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  f32x4 acc[4][7];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 7; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // dy tile and input patch of tile tt into registers, issued one tile ahead (in flight
  // during the previous tile's MFMAs)
  bf16x8 dv[4], pv[4], cv[4];
  float ka[8], k1[8], k0[8];
  if constexpr (PRO) {
    const int cc = (tid & 7) * 8;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      ka[u] = coef[cc + u];
      k1[u] = coef[COUT + cc + u];
      k0[u] = coef[3 * COUT + cc + u];
    }
  }
  auto load_tile = [&](int tt) {
    const int n = tt / tiles_img, r = tt - n * tiles_img;
    const int oh0 = (r / tiles_w) * TH, ow0 = (r % tiles_w) * TW;
    const int ih0 = oh0 * STR - PAD, iw0 = ow0 * STR - PAD;
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // dy tile: 128 px x 8 chunks; patch: 777 pixels
      const int e = tid + 256 * k, px = e >> 3, c = e & 7;
      const size_t o = (((size_t)n * OH + oh0 + (px >> 4)) * OW + ow0 + (px & 15)) * COUT + c * 8;
      dv[k] = *(const bf16x8*)(dy + o);
      if constexpr (PRO) cv[k] = *(const bf16x8*)(bnx + o);
      const int pr = e / PC, pc = e - pr * PC, ih = ih0 + pr, iw = iw0 + pc;
      pv[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (e < PR * PC && ih >= 0 && ih < H && iw >= 0 && iw < W)
        pv[k] = *(const bf16x8*)(x + (((size_t)n * H + ih) * W + iw) * CIN);
    }
  };
  if (blockIdx.x < tiles) load_tile(blockIdx.x);
  for (int t = blockIdx.x; t < tiles; t += gridDim.x) {
    __syncthreads();  // the previous tile's fragment reads are done
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = tid + 256 * k, px = e >> 3, c = e & 7;
      bf16x8 d8 = dv[k];
      if constexpr (PRO) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float de = __uint_as_float((unsigned)(unsigned short)dv[k][u] << 16);
          const float xf = __uint_as_float((unsigned)(unsigned short)cv[k][u] << 16);
          const __bf16 o = (__bf16)(ka[u] * de + k1[u] * xf + k0[u]);
          d8[u] = (short)__builtin_bit_cast(unsigned short, o);
        }
      }
      *(bf16x8*)(Ds + px * DP + c * 16) = d8;
      if (e < PR * PC) *(bf16x8*)(Ps + e * 16) = pv[k];
    }
    __syncthreads();
    if (t + (int)gridDim.x < tiles) load_tile(t + gridDim.x);
#pragma unroll
    for (int kg = 0; kg < 4; ++kg) {  // 32 pixels = tile rows 2 kg, 2 kg + 1
      const int k0 = 32 * kg + 8 * g + q, k1 = k0 + 4;  // this lane's two pixel rows
      bf16x8 a[4], b[7];
#pragma unroll
      for (int i = 0; i < 4; ++i)  // A: (co 16 i + ..., pixel) from the dy tile
        a[i] = tr_pair(Ds + k0 * DP + (16 * i + 4 * p4) * 2, Ds + k1 * DP + (16 * i + 4 * p4) * 2);
      const int pb0 = ((k0 >> 4) * STR) * PC + (k0 & 15) * STR;  // patch pixel of (kh 0, kw 0)
      const int pb1 = ((k1 >> 4) * STR) * PC + (k1 & 15) * STR;
#pragma unroll
      for (int j = 0; j < 7; ++j) {  // B: (k = kh, kw0 + n / 8, c = n % 8) from the patch
        const int nb = 7 * wave + j, kh = nb >> 2, kw0 = 2 * (nb & 3);
        const int off = (kh * PC + kw0) * 16 + 4 * p4 * 2;
        b[j] = tr_pair(Ps + pb0 * 16 + off, Ps + pb1 * 16 + off);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc[i][j], 0, 0, 0);
    }
  }
  // lane (cl, g): column n = cl of block nb, co rows 16 i + 4 g + r
  const int cl = lane & 15;
#pragma unroll
  for (int j = 0; j < 7; ++j) {
    const int nb = 7 * wave + j, kh = nb >> 2, kw = 2 * (nb & 3) + (cl >> 3), c = cl & 7;
    if (kw >= KS) continue;
    const int k = (kh * KS + kw) * CIN + c;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        unsafeAtomicAdd(dw + (size_t)(16 * i + 4 * g + rr) * ldw + k, acc[i][j][rr]);
  }
}

}  // namespace stem

// True when the stem kernel takes this convolution (the caller then sizes the partial
// statistic rows as N * OH * OW / 32).
bool stem_conv_applies(int H, int W, int C, int Cout, int KH, int KW, int stride, int pad) {
  const int OH = (H + 2 * pad - KH) / stride + 1, OW = (W + 2 * pad - KW) / stride + 1;
  return C == stem::CIN && Cout == stem::COUT && KH == stem::KS && KW == stem::KS &&
         stride == stem::STR && pad == stem::PAD && OH % stem::TH == 0 && OW % stem::TW == 0;
}

// dw (f32 [64][ldw], the first 392 columns) (+)= the stem's weight gradient: beta 1
// accumulates, beta 0 overwrites.
// With bnx / coef (bn_bwd_coef rows [4][64]): dy is the gradient at the stem BatchNorm's
// output and the conv output gradient is formed on the fly (see stem_conv_wgrad_kernel).
void stem_conv_wgrad_launch(int N, int H, int W, const void* x, const void* dy, float* dw, int ldw,
                            float beta, hipStream_t s, const void* bnx, const float* coef) {
  using namespace stem;
  if (!stem_conv_applies(H, W, CIN, COUT, KS, KS, STR, PAD))
    throw std::runtime_error("stem_conv: unsupported geometry");
  if (ldw < KS * KS * CIN || (((uintptr_t)x | (uintptr_t)dy | (uintptr_t)bnx) & 15))
    throw std::runtime_error("stem_conv_wgrad: ld >= 392 and 16-B aligned inputs");
  if ((bnx != nullptr) != (coef != nullptr))
    throw std::runtime_error("stem_conv_wgrad: the BN prologue needs both bnx and coef");
  if (beta != 0.f && beta != 1.f) throw std::runtime_error("stem_conv_wgrad: beta must be 0 or 1");
  if (beta == 0.f)
    DTFX_HIP_CHECK(hipMemset2DAsync(dw, sizeof(float) * ldw, 0, sizeof(float) * KS * KS * CIN,
                                    COUT, s));
  const int OH = (H + 2 * PAD - KS) / STR + 1, OW = (W + 2 * PAD - KS) / STR + 1;
  const int tiles = N * (OH / TH) * (OW / TW);
  const size_t lds = 128 * DP + P_BYTES;
  const int blocks = std::min(tiles, 256);  // one persistent block per CU: 28 accumulator tiles
  auto k = bnx ? stem_conv_wgrad_kernel<true> : stem_conv_wgrad_kernel<false>;
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), lds, s, N, H, W, OH, OW, (const unsigned short*)x,
                     (const unsigned short*)dy, dw, ldw, (const unsigned short*)bnx, coef);
  DTFX_HIP_CHECK(hipGetLastError());
}

// psum / psq: stem_conv_fwd_rows() partial rows of 64 floats each
int stem_conv_fwd_rows(int N, int OH, int OW) {
  return N * ((OH + stem::FTH - 1) / stem::FTH) * (OW / stem::TW) * 4;
}

void stem_conv_fwd_launch(int N, int H, int W, const void* x, const void* w, int ldw, void* y,
                          float* psum, float* psq, hipStream_t s) {
  using namespace stem;
  if (!stem_conv_applies(H, W, CIN, COUT, KS, KS, STR, PAD))
    throw std::runtime_error("stem_conv: unsupported geometry");
  if (ldw < 56 * 8 || ldw % 8 || (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y) & 15))
    throw std::runtime_error("stem_conv: weights need ld >= 448 (% 8), 16-B aligned tensors");
  const int OH = (H + 2 * PAD - KS) / STR + 1, OW = (W + 2 * PAD - KS) / STR + 1;
  const int tiles = N * ((OH + FTH - 1) / FTH) * (OW / TW);
  const size_t lds = W_BYTES + FP_BYTES;
  static_assert(FP_BYTES >= 4 * 4096, "output staging");
  static_assert(2 * (W_BYTES + FP_BYTES) <= 160 * 1024, "two blocks per CU");
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)stem_conv_fwd_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int blocks = std::min(tiles, 2 * 256);  // persistent: two blocks per CU
  hipLaunchKernelGGL(stem_conv_fwd_kernel, dim3(blocks), dim3(256), lds, s, N, H, W, OH, OW,
                     (const unsigned short*)x, (const unsigned short*)w, ldw, (unsigned short*)y,
                     psum, psq);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
