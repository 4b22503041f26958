// Device-side building blocks of the bf16 GEMM family (gemm_bf16.hip): bf16 <-> f32, the
// GELU epilogue math, the implicit-GEMM convolution descriptor, the LDS image swizzles, the
// glds staging / fragment readers and the epilogue descriptor.  A header so that the kernel
// probes under tools/probes/ build variants of the tile schedules on the same primitives.
#pragma once

#include "common.h"

namespace dtfx {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ float bf2f(unsigned short h) {
  return __uint_as_float((unsigned)h << 16);
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: round-to-nearest-even, NaN stays NaN
  return __builtin_bit_cast(unsigned short, b);
}

// GELU (tanh form) and its derivative, as sigmoids: 0.5 (1 + tanh(u)) = sigmoid(2u), so
//   gelu(x)  = x * s,  s = 1 / (1 + 2^(-x (A + B x^2)))   (A, B: 2 sqrt(2/pi) (1, 0.044715),
//                                                           pre-scaled by log2(e))
//   gelu'(x) = s + x s (1 - s) (2u)',  (2u)' = C (1 + 3 * 0.044715 x^2)
// One v_exp_f32 (base 2, no range reduction) + one v_rcp_f32 and 5-6 plain VALU per element
// -- the tanh form took ~13 (epilogue VALU is exposed: BERT's FFN1 forward lost 13 % of its
// GEMM rate to the GELU math, tools/gemm_cfg_ab.py "ffn1_fwd_gelu_noaux" vs "ffn1_fwd_bias").
// Saturates: 2^(+large) = inf -> s = 0 (x -> -inf gives -0), 2^(-large) = 0 -> s = 1.
__device__ __forceinline__ float gelu_sig(float x) {
  constexpr float A = 2.302208198f;   // 2 * sqrt(2 / pi) * log2(e)
  constexpr float B = 0.1029432397f;  // A * 0.044715
  const float t = x * __builtin_fmaf(B, x * x, A);
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-t));
}
__device__ __forceinline__ float gelu_f(float x) { return x * gelu_sig(x); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  constexpr float C = 1.5957691216f;   // 2 * sqrt(2 / pi)
  constexpr float D = 0.2140644640f;   // C * 3 * 0.044715
  const float s = gelu_sig(x);
  return __builtin_fmaf(x * s * (1.f - s), __builtin_fmaf(D, x * x, C), s);
}
// gelu(x), with gelu'(x) from the same sigmoid (act 3: the forward stores the derivative, so the
// backward epilogue is one multiply instead of a second exp + rcp per element)
__device__ __forceinline__ float gelu_fg(float x, float& gp) {
  constexpr float C = 1.5957691216f, D = 0.2140644640f;
  const float s = gelu_sig(x), xs = x * s;
  gp = __builtin_fmaf(xs * (1.f - s), __builtin_fmaf(D, x * x, C), s);
  return xs;
}

// Convolution as implicit GEMM (NHWC bf16 activations, weights [Cout][KH][KW][Cin]).
//   MODE 1 fwd   : C[pix][co]  = sum_k im2col(x)[pix][k] * W[co][k],   k = (kh, kw, ci)
//   MODE 2 dgrad : dX[pix][ci] = sum_k col2im(dy)[pix][k] * W'[k][ci], k = (kh, kw, co)
//   MODE 3 wgrad : dW[co][j]   = sum_p dy[p][co] * im2col(x)[p][j],    j = (kh, kw, ci)
// The gathers run in the glds staging: every lane computes its own 16-B source
// address (8 consecutive channels of one tap; C % 8 == 0), and padding taps /
// K tails point at a 16-B zero page, so no im2col buffer ever exists.
//
// MODE 2 runs as stride x stride phase classes (blockIdx.z): the input pixels
// h = i*s + ph, w = j*s + pw of class (ph, pw) only receive the taps kh = kh0 + s*th,
// kw = kw0 + s*tw (kh0 = (ph + pad) % s), and for those taps dy is read at
// (i + oy - th, j + ox - tw), oy = (ph + pad - kh0) / s -- a dense stride-1 product over
// the class's pixels with a nkh x nkw kernel.  A strided dgrad thus does no MFMA work on
// the (s^2 - 1)/s^2 taps a pixel never receives (it used to gather zeros for them: the
// stride-2 dgrads of ResNet-50 ran at ~100 TFLOP/s against ~330 at stride 1).  The
// epilogue maps class row m back to pixel (n, i*s + ph, j*s + pw).
struct ConvDesc {
  int N, H, W, C;        // input
  int OH, OW, K;         // output spatial, output channels
  int KH, KW, stride, pad;
  int ktot;              // reduction length of the GEMM (MODE 1: KH*KW*C, MODE 2: KH*KW*K)
  int wld;               // weight row stride (elements) for MODE 2
  // MODE 2 phase class (set in the kernel from blockIdx.z; see above)
  int ph, pw, Hc, Wc, oy, ox, kh0, kw0, nkh, nkw;
  int prc;               // partial statistic rows per class (MODE 2, col_partial)
};

// MODE 2: this block's phase class -> the class fields of d, d.ktot; returns the class's
// pixel count (GEMM M)
__device__ __forceinline__ int dgrad_class(ConvDesc& d, int z) {
  const int s = d.stride;
  d.ph = z / s;
  d.pw = z - d.ph * s;
  d.Hc = (d.H - d.ph + s - 1) / s;
  d.Wc = (d.W - d.pw + s - 1) / s;
  d.kh0 = (d.ph + d.pad) % s;
  d.kw0 = (d.pw + d.pad) % s;
  d.nkh = d.KH > d.kh0 ? (d.KH - d.kh0 + s - 1) / s : 0;
  d.nkw = d.KW > d.kw0 ? (d.KW - d.kw0 + s - 1) / s : 0;
  d.oy = (d.ph + d.pad - d.kh0) / s;
  d.ox = (d.pw + d.pad - d.kw0) / s;
  d.ktot = d.nkh * d.nkw * d.K;
  return d.N * d.Hc * d.Wc;
}

__device__ __attribute__((aligned(16))) unsigned short g_zero16[8];

// q = a / d, r = a % d for 0 <= a < 2^24, d > 0 (float reciprocal + one correction)
__device__ __forceinline__ void fdivmod(int a, int d, float inv, int& q, int& r) {
  q = (int)((float)a * inv);
  r = a - q * d;
  if (r >= d) { ++q; r -= d; }
  if (r < 0) { --q; r += d; }
}

namespace gb {
constexpr int BN = 128, BK = 64;  // tile N and K; the tile height BM is a template parameter

// k-contiguous images (128-B rows, 8 chunks of 16 B): chunk c of row r is stored at
// c ^ swz_kc(r).  A ds_read_b128 16-lane group reads 16 consecutive rows at one chunk; even
// and odd rows sit on opposite 128-B halves of the 256-B bank row, so XOR-ing with r >> 1
// (not r) spreads the 16 reads over all 16 slots (r & 7 left rows r and r + 8 on one slot:
// 2-way conflicts).
__device__ __forceinline__ int swz_kc(int r) { return (r >> 1) & 7; }
__device__ __forceinline__ int swz_tr(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }
// 64-wide k-strided images (128-B rows: even rows on banks 0-31, odd rows on 32-63): a
// ds_read_b64_tr_b16 half-wave reads rows {q, q+8} (q = 0..3) x 2 chunks; the XOR puts the 4
// same-parity rows on 4 disjoint chunk pairs (conflict-free; values stay < 8 chunks)
__device__ __forceinline__ int swz64(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }
template <int OUTER>
__device__ __forceinline__ int swz_k(int r) { return OUTER == 64 ? swz64(r) : swz_tr(r); }

// Stage one operand tile of OUTER x 64 (OUTER * 128 bytes) with glds: NW waves, each wave
// instruction fills one 1 KB block.
//  KCONT: tile rows = OUTER outer (m or n) indices x 64 k (128-B rows); src row stride ld.
//  else : tile rows = 64 k x OUTER outer (OUTER*2-B rows); src row stride ld.
template <bool KCONT, int OUTER, int NW>
__device__ __forceinline__ void stage(const unsigned short* __restrict__ src, int ld, int outer0,
                                      int outer_max, int k0, char* lds_tile, int wave, int lane,
                                      int kmax) {
  constexpr int NB = OUTER / 8;            // 1 KB blocks per tile
  constexpr int LPR = OUTER / 8;           // lanes per k-row in the k-strided image
  constexpr int RPB = 64 / LPR;            // k-rows per block
#pragma unroll
  for (int i = 0; i < NB / NW; ++i) {
    const int blk = i * NW + wave;  // 1 KB block of the tile this wave-instruction fills
    const unsigned short* g;
    if (KCONT) {
      const int row = blk * 8 + (lane >> 3), cs = lane & 7;
      const int c = cs ^ swz_kc(row);
      const int o = min(outer0 + row, outer_max);
      g = src + (size_t)o * ld + k0 + c * 8;
    } else {
      const int kr = blk * RPB + lane / LPR, cs = lane % LPR;
      const int c = cs ^ swz_k<OUTER>(kr);
      const int o = min(outer0 + c * 8, outer_max);  // outer_max is 8-aligned-safe (host)
      g = src + (size_t)min(k0 + kr, kmax) * ld + o;  // clamped K tail: partner operand is 0
    }
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(lds_tile + blk * 1024), 16, 0, 0);
  }
}

// Fragment (8 bf16 along k) for MFMA 16x16x32: lane holds [outer = o0 + (l&15)][k = kk*32 + 8(l>>4) + j]
template <bool KCONT, int OUTER>
__device__ __forceinline__ bf16x8 frag(const char* lds_tile, int o0, int kk, int lane) {
  constexpr int RB = OUTER * 2;  // row bytes of the k-strided image
  if (KCONT) {
    const int row = o0 + (lane & 15);
    const int c = kk * 4 + (lane >> 4);
    return *(const bf16x8*)(lds_tile + row * 128 + ((c ^ swz_kc(row)) << 4));
  } else {
    // ds_read_b64_tr_b16: 16-lane group g reads k rows kk*32+8g+{0..3} (+4 for the 2nd
    // read), cols o0..o0+15; lane 4q+p addresses row q, cols 4p..4p+3.
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int col = o0 + 4 * p;
    const int cch = col >> 3, cb = (col & 7) * 2;
    const int r0 = kk * 32 + 8 * g + q, r1 = r0 + 4;
    const char* a0 = lds_tile + r0 * RB + ((cch ^ swz_k<OUTER>(r0)) << 4) + cb;
    const char* a1 = lds_tile + r1 * RB + ((cch ^ swz_k<OUTER>(r1)) << 4) + cb;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)a0);
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) bf16x4*)a1);
    bf16x8 v;
    v.lo = lo;
    v.hi = hi;
    return v;
  }
}
// MODE 1/2 A operand (k-contiguous image [BM pix][64 k]): per-lane row state, computed once.
// NBLK = 1 KB blocks (8 rows each) per wave: BM / 8 / NW (4 for 128x128 / 256x128, 8 for the
// 256x64 tile); entries past NBLK are never referenced (registers only for the used ones).
struct RowState {
  int nb[8], y0[8], x0[8];  // n*H*W (or -1 past M), spatial base of each of the lane's rows
};

template <int NW, int NBLK>
__device__ __forceinline__ void conv_rows(const ConvDesc& d, int mode, int M, int m0, int wave,
                                          int lane, RowState& rs) {
  static_assert(NBLK <= 8, "RowState holds 8 rows per lane");
  const int PW = mode == 1 ? d.OW : d.Wc, PHW = mode == 1 ? d.OH * d.OW : d.Hc * d.Wc;
  const float ipw = 1.f / PW, iphw = 1.f / PHW;
#pragma unroll
  for (int i = 0; i < NBLK; ++i) {
    const int m = m0 + (i * NW + wave) * 8 + (lane >> 3);
    int n, rem, py, px;
    fdivmod(min(m, M - 1), PHW, iphw, n, rem);
    fdivmod(rem, PW, ipw, py, px);
    rs.nb[i] = m < M ? n : -1;
    if (mode == 1) {
      rs.y0[i] = py * d.stride - d.pad;
      rs.x0[i] = px * d.stride - d.pad;
    } else {  // dgrad (class-local pixel): dy row of tap th is y0 - th
      rs.y0[i] = py + d.oy;
      rs.x0[i] = px + d.ox;
    }
  }
}

// A tile gather for conv fwd (mode 1: src = x, channels C) / dgrad (mode 2: src = dy, channels K);
// tile height 8 * NBLK * NW rows: NBLK blocks per wave
template <int NW, int NBLK>
__device__ __forceinline__ void stage_a_conv(const ConvDesc& d, int mode, const RowState& rs,
                                             const unsigned short* __restrict__ src, int k0,
                                             char* lds_tile, int wave, int lane) {
  const int CH = mode == 1 ? d.C : d.K;
  const bool uni = (CH & 63) == 0;  // a 64-wide k step stays inside one tap
  const int tap_u = k0 / CH, c_u = k0 - tap_u * CH;
#pragma unroll
  for (int i = 0; i < NBLK; ++i) {
    const int blk = i * NW + wave;
    const int row = blk * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz_kc(row);
    const int k = k0 + c * 8;
    int tap, ch;
    if (uni) { tap = tap_u; ch = c_u + c * 8; }
    else { tap = k / CH; ch = k - tap * CH; }
    const int TW = mode == 1 ? d.KW : d.nkw;  // (mode 2: class taps)
    const int kh = tap / TW, kw = tap - kh * TW;
    bool ok = rs.nb[i] >= 0 && k < d.ktot;
    int yy, xx;
    if (mode == 1) {
      yy = rs.y0[i] + kh;
      xx = rs.x0[i] + kw;
      ok = ok && yy >= 0 && yy < d.H && xx >= 0 && xx < d.W;
    } else {
      yy = rs.y0[i] - kh;
      xx = rs.x0[i] - kw;
      ok = ok && yy >= 0 && xx >= 0 && yy < d.OH && xx < d.OW;
    }
    const int SH = mode == 1 ? d.H : d.OH, SW = mode == 1 ? d.W : d.OW;
    const unsigned short* g =
        ok ? src + ((size_t)(rs.nb[i] * SH + yy) * SW + xx) * CH + ch : g_zero16;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(lds_tile + blk * 1024), 16, 0, 0);
  }
}

// B tile for dgrad (k-strided image [64 k][OUTER ci], OUTER = 128 or 64):
// W'[k = (kh, kw, co)][ci] = W[co][kh][kw][ci]
template <int NW, int OUTER>
__device__ __forceinline__ void stage_b_wtap(const ConvDesc& d, const unsigned short* __restrict__ w,
                                             int n0, int k0, char* lds_tile, int wave, int lane) {
  constexpr int LPR = OUTER / 8, RPB = 64 / LPR;  // lanes per k-row, k-rows per 1 KB block
  const int ctap = k0 / d.K, co0 = k0 - ctap * d.K;  // host: K % 64 == 0
  const int th = ctap / max(d.nkw, 1), tw = ctap - th * d.nkw;  // class tap -> kernel tap
  const int tap = (d.kh0 + d.stride * th) * d.KW + d.kw0 + d.stride * tw;
#pragma unroll
  for (int i = 0; i < (OUTER / 8) / NW; ++i) {
    const int blk = i * NW + wave;
    const int kr = blk * RPB + lane / LPR;
    const int c = (lane % LPR) ^ swz_k<OUTER>(kr);
    const int o = n0 + c * 8;
    const bool ok = k0 + kr < d.ktot && o < d.C;
    const unsigned short* g =
        ok ? w + (size_t)(co0 + kr) * d.wld + (size_t)tap * d.C + o : g_zero16;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(lds_tile + blk * 1024), 16, 0, 0);
  }
}

// B tile for wgrad (k-strided image [64 pixels][128 j]): im2col(x)[p][j = (kh, kw, ci)].
// The column half of the gather is hoisted out of the K loop: a lane's 16-B
// chunk always covers the same 8 columns j (its k-row kr and swizzled chunk are fixed), so
// (tap, ci) -> (kh - pad, kw - pad, ci) is decoded ONCE per block (im2col_cols) and each K tile
// only decodes its pixels (2 fdivmods per chunk instead of 4).
struct Im2colCols {
  int ci[4], dh[4], dw[4];  // channel offset, kh - pad, kw - pad of the lane's i-th chunk
  int jok;                  // bit i: the chunk's columns are inside KH * KW * C
};
template <int NW>
__device__ __forceinline__ void im2col_cols(const ConvDesc& d, int n0, int wave, int lane, Im2colCols& s) {
  static_assert(16 / NW <= 4, "Im2colCols holds 4 chunks per lane");
  const float ikw = 1.f / d.KW, ic = 1.f / d.C;
  const int jtot = d.KH * d.KW * d.C;
  s.jok = 0;
#pragma unroll
  for (int i = 0; i < 16 / NW; ++i) {
    const int blk = i * NW + wave;
    const int kr = blk * 4 + (lane >> 4);
    const int c = (lane & 15) ^ swz_tr(kr);
    const int j = n0 + c * 8;
    int tap, ci, kh, kw;
    fdivmod(min(j, jtot - 8), d.C, ic, tap, ci);
    fdivmod(tap, d.KW, ikw, kh, kw);
    s.ci[i] = ci;
    s.dh[i] = kh - d.pad;
    s.dw[i] = kw - d.pad;
    s.jok |= (j < jtot ? 1 : 0) << i;
  }
}
template <int NW>
__device__ __forceinline__ void stage_b_im2col_h(const ConvDesc& d, const unsigned short* __restrict__ x,
                                                 int NP, int k0, const Im2colCols& s, char* lds_tile,
                                                 int wave, int lane) {
  const int ohw = d.OH * d.OW;
  const float iohw = 1.f / ohw, iow = 1.f / d.OW;
#pragma unroll
  for (int i = 0; i < 16 / NW; ++i) {
    const int blk = i * NW + wave;
    const int kr = blk * 4 + (lane >> 4);
    const int p = k0 + kr;
    int n, rem, oh, ow;
    fdivmod(min(p, NP - 1), ohw, iohw, n, rem);
    fdivmod(rem, d.OW, iow, oh, ow);
    const int yy = oh * d.stride + s.dh[i], xx = ow * d.stride + s.dw[i];
    const bool ok = p < NP && ((s.jok >> i) & 1) && (unsigned)yy < (unsigned)d.H &&
                    (unsigned)xx < (unsigned)d.W;
    const unsigned short* g = ok ? x + ((size_t)(n * d.H + yy) * d.W + xx) * d.C + s.ci[i] : g_zero16;
    __builtin_amdgcn_global_load_lds((const void*)g, (lds_void*)(lds_tile + blk * 1024), 16, 0, 0);
  }
}
// s_waitcnt vmcnt(N) + lgkmcnt(0) + s_barrier in one asm statement: the LDS-DMA (glds) of
// the newest N loads stays in flight across the barrier ("memory" keeps the compiler's
// LDS reads of the retiring buffer before it).
template <int N>
__device__ __forceinline__ void vm_barrier() {
  asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}
}  // namespace gb

struct GemmEpi {
  float alpha, beta;
  const float* bias;            // [N] or null
  int act;                      // 0 none, 1 gelu, 2 relu
  const unsigned short* aux_in; // [M][ld_aux] pre-activation (bf16) for act_grad, or null
  unsigned short* aux_out;      // [M][ld_aux] store pre-activation, or null
  int ld_aux;
  const unsigned short* residual;  // [M][ld_res] bf16 or null
  int ld_res;
  int act_grad;                 // multiply by act'(aux_in)
  float* colsum;                // [N] += column sums of the final values (bias gradient), or null
  float* colsq;                 // [N] += column sums of squares (BatchNorm statistics), or null
  int col_partial;              // 1: colsum/colsq are [2 * m_tiles][N] partial rows (plain stores,
                                //    no same-address atomics: BatchNorm statistics of tall convs)
  // BatchNorm-backward statistics fused into a conv dgrad: with bn_x set, colsq accumulates
  // v * xhat, xhat = (bn_x[m][n] - bn_mean[n]) * bn_rstd[n] (bn_x: the BN input, ld = ldc),
  // instead of v^2 -- colsum / colsq are then exactly BatchNorm's sum(dy) / sum(dy * xhat).
  const unsigned short* bn_x;
  const float* bn_mean;
  const float* bn_rstd;
  // split-K partials: with ws set, split s writes its tile to ws[s][M][N] with plain stores and
  // splitk_reduce folds them into C afterwards (f32 atomics run at the memory side, ~1.3 TB/s
  // chip-wide: a 512-block split-K wave adds ~34 MB, ~26 us, against ~6 us of plain stores)
  float* ws;
};
}  // namespace dtfx
