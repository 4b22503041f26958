// 1x1 / stride 1 convolutions with 64, 128 or 256 reduction channels and 256 * 2^i output
// channels (ResNet-50's expansions: conv3 and layer1's downsample forward, 64 -> 256,
// 128 -> 512, 256 -> 1024; conv1's data gradient, 64 / 128 / 256 -> 256 ... 1024), NHWC
// bf16, as a streaming product: persistent blocks, the weights held in REGISTERS for the
// block's life, per pixel tile only the pixels' K channels read and the output written, with
// the BatchNorm work fused:
//   forward:  y = x W^T, partial rows of sum(y) / sum(y^2) per output channel;
//   dgrad:    de = (dy W + residual) * (relu_y > 0), partial rows of sum(de) and
//             sum(de * xhat) (xhat = (bn_x - mean) * rstd, formed at the end from
//             sum(de * bn_x) - mean * sum(de)), for bn_bwd_apply.
// These are memory-bound products (K = 64: 2 FLOP per output byte): on the implicit-GEMM
// tile they ran at 2.4-3.5 TB/s (layer1 conv3 forward 216 us against 79 us of HBM traffic);
// here 4.1-6.1 TB/s (profiles/r2/conv1x1_streaming.txt).
//
// The product is computed transposed, D[channel][pixel] = W[channel][:] . x[pixel][:], so
// an MFMA lane's 4 accumulator rows are 4 CONSECUTIVE channels of one pixel: outputs and side
// inputs move as 8-B vectors of NHWC rows, and a lane's statistics stay its own 4 channels
// for the whole block.  Compute wave w owns 32 channels (2 MFMA row tiles) of the block's 256.
#include "common.h"
#include "bn_common.h"

#include <algorithm>
#include <cstdlib>
#include <stdexcept>

namespace dtfx {
namespace pw {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));

constexpr int NTW = 2, NW = 8;
constexpr int NC = NW * NTW * 16;  // 256 channels per block

__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float bf(short v) {
  return __uint_as_float((unsigned)(unsigned short)v << 16);
}

// Forward with a loader wave: wave NW (the ninth) only moves 64-pixel x tiles into a ring of
// 3 LDS buffers (global_load_lds, counted vmcnt), the 8 compute waves only read LDS and store.
// A wave that waits on a load also waits for every store it issued before that load (one
// in-order vmcnt counter), so when the compute waves fetched their own pixels each held at
// most a tile of stores in flight: ~5 us per 32-pixel tile, 2.2 TB/s.  Here nothing behind
// the stores waits on memory.  x rows in LDS: 16-B chunk c of row r at c ^ swz(r) (K = 64:
// 128-B rows, swz = (r >> 1) & 7; K >= 128: swz = r & 15): the 16 rows a fragment read
// touches land on distinct bank groups.
typedef __attribute__((address_space(3))) void lds_void;
constexpr int NBUF = 3;
constexpr int OPITCH = NC * 2 + 16;  // output staging row (bytes): 16-B skew per pixel
template <int K>
constexpr int ftm() {  // forward pixels per tile: LDS for 2 blocks per CU (1 for K = 256)
  return K == 128 ? 32 : 64;
}
template <int K>
constexpr int fbpc() {  // forward blocks per CU: K = 256 needs 64 VGPRs of weights
  return K == 256 ? 1 : 2;
}

template <int K>
__device__ __forceinline__ int xswz(int r) {
  return K == 64 ? (r >> 1) & 7 : r & 15;
}

// PRO 3: the x tile is formed as relu(x a + c) in LDS before the MFMAs (the BatchNorm + ReLU
// of the conv that produced x, coef rows 0 and 2 of bn_fwd_coef) and written to xo by the
// first column block: the BN's output is written once and never read back for this product.
template <int K, int PRO = 0>
__global__ __launch_bounds__(576, fbpc<K>() == 2 ? 5 : 3) void conv1x1_fwd_kernel(
    int M, int N, const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
    int ldw, unsigned short* __restrict__ y, float* __restrict__ ps, float* __restrict__ pq,
    BnCoefSrc coef, unsigned short* __restrict__ xo) {
  constexpr int FTM = ftm<K>(), KK = K / 32, MT = FTM / 16, CPR = K / 8;  // chunks per row
  constexpr int TB = FTM * K * 2, NQ = TB / 1024;  // tile bytes, DMA rounds per tile
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* stg = sm + NBUF * TB;  // output staging [FTM][OPITCH]
  const int nbn = N / NC, PB = gridDim.x / nbn;
  const int b = blockIdx.x, i8 = b >> 3;
  const int cb = i8 % nbn, pb = (i8 / nbn) * 8 + (b & 7);
  const int tid = threadIdx.x, lane = tid & 63, cl = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = M / FTM;
  const int nmy = pb < T ? (T - pb + PB - 1) / PB : 0;  // this block's tiles pb, pb + PB, ...
  if (wave == NW) {
    auto issue = [&](int it) {
      const int tile = pb + it * PB;
      char* d = sm + (it % NBUF) * TB;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int P = q * 64 + lane, r = P / CPR, c = (P % CPR) ^ xswz<K>(r);
        const unsigned short* src = x + ((size_t)tile * FTM + r) * K + c * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(d + q * 1024), 16, 0, 0);
      }
    };
    if (nmy > 0) issue(0);
    if (nmy > 1) {
      issue(1);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQ) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    for (int it = 0; it < nmy; ++it) {
      if constexpr (PRO != 0) asm volatile("s_barrier" ::: "memory");  // (the transform's barrier)
      if (it + 2 < nmy) {
        issue(it + 2);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQ) : "memory");  // tile it + 1 landed
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __syncthreads();  // (the compute waves' staging barrier)
      __syncthreads();
    }
    return;
  }
  const int c0 = cb * NC + wave * (NTW * 16);
  bf16x8 wf[NTW][KK];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      wf[j][kk] = *(const bf16x8*)(w + (size_t)(c0 + 16 * j + cl) * ldw + 32 * kk + 8 * g);
  float s1[NTW][4], s2[NTW][4];
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
  // PRO: thread tid transforms chunk column tcc of rows tr0 + j * RPP; the coefficient rows
  // a / c sit in LDS after the output staging (in registers they pushed the two-blocks-per-CU
  // variants past 96 VGPRs into scratch)
  constexpr int RPP = 512 / CPR, NPASS = FTM / RPP;
  const int tcc = tid % CPR, tr0 = tid / CPR;
  float* ctab = (float*)(stg + FTM * OPITCH);  // [2][K]
  if constexpr (PRO != 0) {
    for (int i = tid; i < K; i += NW * 64) {
      float a, b, c, d;
      bn_coef_at(coef, K, i, a, b, c, d);
      ctab[i] = a;
      ctab[K + i] = c;
    }
    if (blockIdx.x == 0) bn_coef_duty(coef, K, tid, NW * 64);
  }
  __syncthreads();  // tile 0 in LDS
  for (int it = 0; it < nmy; ++it) {
    char* xs = sm + (it % NBUF) * TB;
    const int p0 = (pb + it * PB) * FTM;
    if constexpr (PRO != 0) {
#pragma unroll
      for (int j = 0; j < NPASS; ++j) {
        const int r = tr0 + j * RPP, off = r * (K * 2) + ((tcc ^ xswz<K>(r)) << 4);
        const bf16x8 a8 = *(const bf16x8*)(xs + off);
        const f32x4 a0 = *(const f32x4*)(ctab + tcc * 8), a1 = *(const f32x4*)(ctab + tcc * 8 + 4);
        const f32x4 c0_ = *(const f32x4*)(ctab + K + tcc * 8), c1_ = *(const f32x4*)(ctab + K + tcc * 8 + 4);
        const float ca[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        const float cc[8] = {c0_[0], c0_[1], c0_[2], c0_[3], c1_[0], c1_[1], c1_[2], c1_[3]};
        bf16x8 o8;
#pragma unroll
        for (int u = 0; u < 8; ++u) o8[u] = (short)tobf(fmaxf(bf(a8[u]) * ca[u] + cc[u], 0.f));
        *(bf16x8*)(xs + off) = o8;
        if (xo && cb == 0) __builtin_nontemporal_store(o8, (bf16x8*)(xo + (size_t)(p0 + r) * K + tcc * 8));
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll K == 64 ? MT : 1
    for (int i = 0; i < MT; ++i) {
      bf16x8 xf[KK];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        const int r = 16 * i + cl;
        xf[kk] = *(const bf16x8*)(xs + r * (K * 2) + (((4 * kk + g) ^ xswz<K>(r)) << 4));
      }
#pragma unroll
      for (int j = 0; j < NTW; ++j) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], xf[kk], acc, 0, 0, 0);
        bf16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = (short)tobf(acc[r]);
          s1[j][r] += acc[r];
          s2[j][r] += acc[r] * acc[r];
        }
        *(bf16x4*)(stg + (16 * i + cl) * OPITCH + (wave * (NTW * 16) + 16 * j + 4 * g) * 2) = o;
      }
    }
    __syncthreads();
    // the block's FTM x 256 output rows as 16-B chunks: 32 chunks per pixel, 16 pixels per pass
#pragma unroll
    for (int q = 0; q < FTM / 16; ++q) {
      const int e = q * 512 + tid, p = e >> 5, c = e & 31;
      *(bf16x8*)(y + (size_t)(p0 + p) * N + cb * NC + c * 8) = *(const bf16x8*)(stg + p * OPITCH + c * 16);
    }
    __syncthreads();
  }
  if (!ps) return;
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int m = 1; m < 16; m <<= 1) {
        s1[j][r] += __shfl_xor(s1[j][r], m);
        s2[j][r] += __shfl_xor(s2[j][r], m);
      }
    }
  if (cl == 0) {
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      const int ch = c0 + 16 * j + 4 * g;
      f32x4 a, q;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        a[r] = s1[j][r];
        q[r] = s2[j][r];
      }
      *(f32x4*)(ps + (size_t)pb * N + ch) = a;
      *(f32x4*)(pq + (size_t)pb * N + ch) = q;
    }
  }
}

// Data gradient with the loader wave: per 16-pixel tile the loader moves the dy rows
// (swizzled, for the MFMA fragments) and the block's 256-channel slices of the shortcut
// gradient, relu_y and bn_x (plain rows) into a 4-deep LDS ring; the compute waves stage the
// f32 products through LDS and run the epilogue in row layout, so every side input is read and
// every output written as 16-B chunks of whole 512-B row slices, and nothing that stores waits
// on a load.  Thread t always owns channels 8 (t & 31) .. + 7 of the slice: its statistics
// are summed over the block's pixels in registers and reduced across waves once at the end.
constexpr int DTM = 16;
constexpr int SPITCH = NC * 4 + 16;  // f32 staging row (bytes), 16-B skew per pixel
// the DMA source of a stride-2 residual's zero pixels (one 512-B channel slice)
__device__ __attribute__((aligned(16))) unsigned short g_zero_slice[NC];
template <int K, bool RES, bool BN, int PRO = 0>
constexpr int dgrad_ring() {
  constexpr int nqt = DTM * K * 2 * (PRO ? 2 : 1) / 1024 +
                      ((RES ? 1 : 0) + (BN ? 2 : 0)) * (DTM * NC * 2 / 1024);
  return 2 * nqt <= 63 ? 4 : 3;
}

// w here is the transposed weight copy wt [N][K] (transpose_bf16_kernel).
// PRO 2: dy is formed per tile as s0 a + (s1 b + d) from dy and src1 (BatchNorm backward's
// apply of the BN behind this conv, as in conv1x1_narrow_kernel; bn_bwd_coef's c row is zero)
// and written to xo by the first column block.
template <int K, bool RES, bool BN, int PRO = 0>
__global__ __launch_bounds__(576, 1) void conv1x1_dgrad_kernel(
    int M, int N, const unsigned short* __restrict__ dy, const unsigned short* __restrict__ w,
    int ldw, unsigned short* __restrict__ dx, const unsigned short* __restrict__ res,
    const unsigned short* __restrict__ relu_y, const unsigned short* __restrict__ bn_x,
    const float* __restrict__ bn_mean, const float* __restrict__ bn_rstd, float* __restrict__ ps,
    float* __restrict__ pq, const unsigned short* __restrict__ src1 = nullptr,
    BnCoefSrc coef = BnCoefSrc{}, unsigned short* __restrict__ xo = nullptr,
    int rs_h = 0, int rs_w = 0) {
  constexpr int KK = K / 32, CPR = K / 8;
  constexpr int DYB = DTM * K * 2, SB = DTM * NC * 2, NSIDE = (RES ? 1 : 0) + (BN ? 2 : 0);
  constexpr int DYS = DYB * (PRO ? 2 : 1);  // side tiles after the source tile(s)
  constexpr int STAGE = DYS + NSIDE * SB, NQD = DYB / 1024, NQS = SB / 1024;
  constexpr int NQT = NQD * (PRO ? 2 : 1) + NSIDE * NQS;  // DMA instructions per tile
  // ring depth: vmcnt holds at most 63 in flight, so 2 younger tiles only while 2 NQT <= 63
  constexpr int DB = dgrad_ring<K, RES, BN, PRO>(), D = DB - 1;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* stg = sm + DB * STAGE;
  const int nbn = N / NC, PB = gridDim.x / nbn;
  const int b = blockIdx.x, i8 = b >> 3;
  const int cb = i8 % nbn, pb = (i8 / nbn) * 8 + (b & 7);
  const int tid = threadIdx.x, lane = tid & 63, cl = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = M / DTM;
  const int nmy = pb < T ? (T - pb + PB - 1) / PB : 0;
  if (wave == NW) {
    auto issue = [&](int it) {
      const int tile = pb + it * PB;
      char* d = sm + (it % DB) * STAGE;
#pragma unroll
      for (int q = 0; q < NQD; ++q) {
        const int P = q * 64 + lane, r = P / CPR, c = (P % CPR) ^ xswz<K>(r);
        const unsigned short* src = dy + ((size_t)tile * DTM + r) * K + c * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(d + q * 1024), 16, 0, 0);
        if constexpr (PRO != 0) {
          const unsigned short* src2 = src1 + ((size_t)tile * DTM + r) * K + c * 8;
          __builtin_amdgcn_global_load_lds((const void*)src2, (lds_void*)(d + DYB + q * 1024), 16, 0, 0);
        }
      }
      const unsigned short* sides[3] = {res, relu_y, bn_x};
      // stride-2 residual: the tile's first pixel (n0, h0, w0), once per tile (DTM <= rs_w, so
      // the tile's pixels sit on at most two grid rows: per pixel one compare instead of the
      // four integer divisions -- those made the loader wave the bottleneck, +110 us per call)
      int rw0 = 0, rh0 = 0, rn0 = 0;
      if (RES && rs_w) {
        const int m0 = tile * DTM;
        const int hq0 = (int)((float)m0 * (1.f / (float)rs_w));  // exact: m0 < 2^24
        const int hq = hq0 - (hq0 * rs_w > m0) + ((hq0 + 1) * rs_w <= m0);
        rw0 = m0 - hq * rs_w;
        rn0 = (int)((float)hq * (1.f / (float)rs_h));
        rn0 = rn0 - (rn0 * rs_h > hq) + ((rn0 + 1) * rs_h <= hq);
        rh0 = hq - rn0 * rs_h;
      }
#pragma unroll
      for (int si = 0; si < 3; ++si) {
        if ((si == 0 && !RES) || (si > 0 && !BN)) continue;
        const int slot = (RES ? si : si - 1);
#pragma unroll
        for (int q = 0; q < NQS; ++q) {
          const int r = 2 * q + (lane >> 5), c = lane & 31;
          const unsigned short* src = sides[si] + ((size_t)tile * DTM + r) * N + cb * NC + c * 8;
          if (si == 0 && rs_w) {  // stride-2 residual: stored compact, zero at odd rows / columns
            int ww = rw0 + r, hh = rh0, nn = rn0;
            if (ww >= rs_w) {
              ww -= rs_w;
              if (++hh == rs_h) hh = 0, ++nn;
            }
            src = ((hh | ww) & 1)
                      ? g_zero_slice + c * 8
                      : res + ((((size_t)nn * (rs_h >> 1) + (hh >> 1)) * (rs_w >> 1)) + (ww >> 1)) *
                                    N + cb * NC + c * 8;
          }
          __builtin_amdgcn_global_load_lds((const void*)src,
                                           (lds_void*)(d + DYS + slot * SB + q * 1024), 16, 0, 0);
        }
      }
    };
    // wait until the oldest outstanding tile landed, `younger` newer tiles still in flight
    auto wait_oldest = [&](int younger) {
      if (D >= 3 && younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D >= 3 ? 2 * NQT : 0) : "memory");
      else if (younger >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    for (int it = 0; it < D && it < nmy; ++it) issue(it);
    wait_oldest(min(D, nmy) - 1);
    __syncthreads();
    for (int it = 0; it < nmy; ++it) {
      if constexpr (PRO != 0) asm volatile("s_barrier" ::: "memory");  // (the transform's barrier)
      if (it + D < nmy) issue(it + D);
      wait_oldest(min(D, nmy - 1 - it) - 1);  // tile it + 1 landed
      __syncthreads();  // (the compute waves' staging barrier)
      __syncthreads();
    }
    __syncthreads();  // (the statistics reduction's barrier)
    return;
  }
  // PRO: thread tid < DTM * CPR transforms chunk tid % CPR of row tid / CPR
  const int tcc = tid % CPR, tr = tid / CPR;
  float ca[8], cb_[8], cd[8];  // (coef row 2 is zero for BatchNorm backward: not held)
  if constexpr (PRO != 0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      float c_;
      bn_coef_at(coef, K, tcc * 8 + u, ca[u], cb_[u], c_, cd[u]);
    }
  }
  const int c0 = wave * (NTW * 16);  // the wave's channels inside the slice
  bf16x8 wf[NTW][KK];                // A operand: W^T[n][k], rows of the transposed copy wt
#pragma unroll
  for (int j = 0; j < NTW; ++j)
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      wf[j][kk] = *(const bf16x8*)(w + (size_t)(cb * NC + c0 + 16 * j + cl) * K + 32 * kk + 8 * g);
  float s1[8], s2[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) s1[u] = s2[u] = 0.f;
  const int ep = tid >> 5, ec = tid & 31;  // epilogue: pixel, 16-B chunk of the slice
  __syncthreads();  // tile 0 in LDS
  for (int it = 0; it < nmy; ++it) {
    char* buf = sm + (it % DB) * STAGE;
    const int p0 = (pb + it * PB) * DTM;
    if constexpr (PRO != 0) {
      if (tid < DTM * CPR) {
        const int off = tr * (K * 2) + ((tcc ^ xswz<K>(tr)) << 4);
        const bf16x8 a8 = *(const bf16x8*)(buf + off);
        const bf16x8 b8 = *(const bf16x8*)(buf + DYB + off);
        bf16x8 o8;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float o = bf(a8[u]) * ca[u];
          o += bf(b8[u]) * cb_[u] + cd[u];
          o8[u] = (short)tobf(o);
        }
        *(bf16x8*)(buf + off) = o8;
        if (xo && cb == 0) __builtin_nontemporal_store(o8, (bf16x8*)(xo + (size_t)(p0 + tr) * K + tcc * 8));
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    bf16x8 xf[KK];
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
      xf[kk] = *(const bf16x8*)(buf + cl * (K * 2) + (((4 * kk + g) ^ xswz<K>(cl)) << 4));
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[j][kk], xf[kk], acc, 0, 0, 0);
      *(f32x4*)(stg + cl * SPITCH + (c0 + 16 * j + 4 * g) * 4) = acc;
    }
    __syncthreads();
    {
      const f32x4 a0 = *(const f32x4*)(stg + ep * SPITCH + ec * 32);
      const f32x4 a1 = *(const f32x4*)(stg + ep * SPITCH + ec * 32 + 16);
      float v[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const int so = ep * (NC * 2) + ec * 16;
      if constexpr (RES) {
        const bf16x8 r8 = *(const bf16x8*)(buf + DYS + so);
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] += bf(r8[u]);
      }
      bf16x8 o;
      if constexpr (BN) {
        const bf16x8 y8 = *(const bf16x8*)(buf + DYS + (RES ? 1 : 0) * SB + so);
        const bf16x8 x8 = *(const bf16x8*)(buf + DYS + (RES ? 2 : 1) * SB + so);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          o[u] = (short)tobf(bf(y8[u]) > 0.f ? v[u] : 0.f);
          const float d = bf(o[u]);
          s1[u] += d;
          s2[u] += d * bf(x8[u]);
        }
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = (short)tobf(v[u]);
      }
      __builtin_nontemporal_store(o, (bf16x8*)(dx + (size_t)(p0 + ep) * N + cb * NC + ec * 8));
    }
    __syncthreads();
  }
  if constexpr (BN) {
    // channels 8 ec .. + 7: lanes l and l ^ 32 of a wave, then the 8 waves through LDS
    float* red = (float*)stg;  // [8 waves][32 chunks][16]
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      s1[u] += __shfl_xor(s1[u], 32);
      s2[u] += __shfl_xor(s2[u], 32);
    }
    if (lane < 32) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        red[(wave * 32 + ec) * 16 + u] = s1[u];
        red[(wave * 32 + ec) * 16 + 8 + u] = s2[u];
      }
    }
    __syncthreads();
    if (tid < NC) {
      const int c = tid >> 3, u = tid & 7;
      float a = 0.f, q = 0.f;
#pragma unroll
      for (int wv = 0; wv < NW; ++wv) {
        a += red[(wv * 32 + c) * 16 + u];
        q += red[(wv * 32 + c) * 16 + 8 + u];
      }
      const int ch = cb * NC + tid;
      ps[(size_t)pb * N + ch] = a;
      pq[(size_t)pb * N + ch] = bn_rstd[ch] * (q - bn_mean[ch] * a);
    }
  } else {
    __syncthreads();
  }
}

// Narrow products: 64 or 128 output channels from 256 or 512 reduction channels (ResNet-50's
// reductions: conv1 forward 256 -> 64 / 128 and 512 -> 128, conv3's data gradient into conv2's
// 64 / 128 channels with conv2's BatchNorm backward fused).  Same loader-wave / LDS-ring scheme
// with one block per CU owning ALL N channels: compute wave w takes MFMA row tile w % NT and
// K part w / NT (KS = 8 / NT parts, the parts' f32 products summed in the staged epilogue), so
// the N x K weights (32-128 KB) sit in the 8 waves' registers.
//
// PRO (BatchNorm prologue): the reduction operand is not read from memory as is but formed per
// tile from TWO [M][K] sources and per-channel coefficients, op = (s0 a + c) + (s1 b + d)
// (coef = [a | b | c | d], f32 [4][K]):
//   PRO 1 (forward, + ReLU): s0 = conv3 output c3, s1 = the shortcut (b = 1, d = 0) or the raw
//         downsample output (its own BN as b, d): op = the bottleneck output
//         relu(bn3(c3) + shortcut), which is also written to xo -- the next block's conv1 forms
//         its input itself instead of a separate bn_apply pass writing it and conv1 reading it
//         back (one full read of the 4w-channel block output fewer per block);
//   PRO 2 (data gradient): s0 = dL/d(BN3 output) de3, s1 = c3: op = BN3's dL/dc3 (the affine
//         form of bn_bwd_apply), written to xo for conv3's weight gradient -- the bn_bwd_apply
//         pass (read de3 + c3, write dc3) and this kernel's read of dc3 become one pass.
// The 8 compute waves transform the landed tile in place in LDS (thread t owns one 16-B chunk
// column, so its 8 channels' coefficients stay in registers), one barrier, then the MFMAs read
// it as before.  The loader wave moves both sources (twice the tile bytes: half the pixels per
// tile).
//   PRO 4 (plain data gradient): PRO 2's operand without a BatchNorm behind the conv's input --
//         no ReLU mask, no side tiles, no statistics (the stride-1 downsample conv of ResNet's
//         first block: its own BN's backward apply in the prologue).
template <bool DG, int PRO>
constexpr bool nside() {  // the data gradient's relu_y / bn_x side tiles ride along
  return DG && PRO != 4;
}
template <int K, int N_, bool DG, int PRO = 0>
constexpr int ntm() {  // pixels per tile (LDS: 3-4 ring stages + the f32 staging)
  return PRO ? ((K == 512 || (DG && N_ == 128)) ? 16 : 32) : DG ? (N_ == 64 ? 32 : 16) : (N_ == 64 ? 64 : 32);
}
template <int K, int N_, bool DG, int PRO = 0>
constexpr int nqt_narrow() {  // DMA instructions per tile
  return ntm<K, N_, DG, PRO>() * K * 2 * (PRO ? 2 : 1) / 1024 +
         (nside<DG, PRO>() ? 2 * ntm<K, N_, DG, PRO>() * N_ * 2 / 1024 : 0);
}

template <int K, int N_, bool DG, int PRO>
__global__ __launch_bounds__(576, 1) void conv1x1_narrow_kernel(
    int M, const unsigned short* __restrict__ x, const unsigned short* __restrict__ w,
    unsigned short* __restrict__ y, const unsigned short* __restrict__ relu_y,
    const unsigned short* __restrict__ bn_x, const float* __restrict__ bn_mean,
    const float* __restrict__ bn_rstd, float* __restrict__ ps, float* __restrict__ pq,
    const unsigned short* __restrict__ src1, BnCoefSrc coef,
    unsigned short* __restrict__ xo) {
  constexpr int NT = N_ / 16, KS = 8 / NT, KKW = K / 32 / KS, CPR = K / 8, NCH = N_ / 8;
  constexpr int TM = ntm<K, N_, DG, PRO>(), MT = TM / 16;
  constexpr int XB = TM * K * 2, SB = TM * N_ * 2;
  constexpr int XS = XB * (PRO ? 2 : 1);  // side tiles (relu_y, bn_x) after the source tile(s)
  constexpr bool SIDE = nside<DG, PRO>();
  constexpr int STAGE = XS + (SIDE ? 2 * SB : 0);
  constexpr int NQX = XB / 1024, NQS = SB / 1024, NQT = nqt_narrow<K, N_, DG, PRO>();
  constexpr int DB = 2 * NQT <= 63 ? 4 : 3, D = DB - 1;
  static_assert(!PRO || (512 % CPR == 0 && TM % (512 / CPR) == 0), "PRO: whole chunk columns");
  constexpr int PITCH = N_ * 4 + 16;           // f32 staging row (bytes)
  constexpr int NE = TM * NCH;                 // epilogue chunks per tile
  constexpr int EP = (NE + 511) / 512;         // epilogue passes
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* stg = sm + DB * STAGE;                 // [KS][TM][PITCH]
  const int PB = gridDim.x, pb = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, cl = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int T = M / TM;
  const int nmy = pb < T ? (T - pb + PB - 1) / PB : 0;
  if (wave == NW) {
    auto issue = [&](int it) {
      const int tile = pb + it * PB;
      char* d = sm + (it % DB) * STAGE;
#pragma unroll
      for (int q = 0; q < NQX; ++q) {
        const int P = q * 64 + lane, r = P / CPR, c = (P % CPR) ^ xswz<K>(r);
        const unsigned short* src = x + ((size_t)tile * TM + r) * K + c * 8;
        __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(d + q * 1024), 16, 0, 0);
      }
      if constexpr (PRO != 0) {  // the second source, same swizzled image
#pragma unroll
        for (int q = 0; q < NQX; ++q) {
          const int P = q * 64 + lane, r = P / CPR, c = (P % CPR) ^ xswz<K>(r);
          const unsigned short* src = src1 + ((size_t)tile * TM + r) * K + c * 8;
          __builtin_amdgcn_global_load_lds((const void*)src, (lds_void*)(d + XB + q * 1024), 16, 0, 0);
        }
      }
      if constexpr (SIDE) {
#pragma unroll
        for (int si = 0; si < 2; ++si) {
          const unsigned short* side = si == 0 ? relu_y : bn_x;
#pragma unroll
          for (int q = 0; q < NQS; ++q) {
            const int P = q * 64 + lane;  // row-major [TM][N_] in 16-B chunks
            const unsigned short* src = side + (size_t)tile * TM * N_ + P * 8;
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (lds_void*)(d + XS + si * SB + q * 1024), 16, 0, 0);
          }
        }
      }
    };
    auto wait_oldest = [&](int younger) {
      if (D >= 3 && younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D >= 3 ? 2 * NQT : 0) : "memory");
      else if (younger >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NQT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    for (int it = 0; it < D && it < nmy; ++it) issue(it);
    wait_oldest(min(D, nmy) - 1);
    __syncthreads();
    for (int it = 0; it < nmy; ++it) {
      if constexpr (PRO != 0) asm volatile("s_barrier" ::: "memory");  // (the transform's barrier)
      if (it + D < nmy) issue(it + D);
      wait_oldest(min(D, nmy - 1 - it) - 1);  // tile it + 1 landed
      __syncthreads();
      __syncthreads();
    }
    if constexpr (!DG || SIDE) __syncthreads();  // (the statistics reduction)
    return;
  }
  const int nt = wave % NT, part = wave / NT, kk0 = part * KKW;
  bf16x8 wf[KKW];  // A operand rows: channel 16 nt + cl (forward: w [N][ldw]; dgrad: wt [N][K])
#pragma unroll
  for (int kk = 0; kk < KKW; ++kk)
    wf[kk] = *(const bf16x8*)(w + (size_t)(16 * nt + cl) * K + 32 * (kk0 + kk) + 8 * g);
  float s1[8], s2[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) s1[u] = s2[u] = 0.f;
  // PRO: thread tid transforms chunk column tcc of rows tr0 + j * RPP
  constexpr int RPP = PRO ? 512 / CPR : 1, NPASS = PRO ? TM / RPP : 0;
  const int tcc = tid % CPR, tr0 = tid / CPR;
  float ca[8], cb[8], cc[8], cd[8];
  if constexpr (PRO != 0) {
#pragma unroll
    for (int u = 0; u < 8; ++u) bn_coef_at(coef, K, tcc * 8 + u, ca[u], cb[u], cc[u], cd[u]);
    if (PRO == 1 && blockIdx.x == 0) bn_coef_duty(coef, K, tid, 512);
  }
  __syncthreads();  // tile 0 in LDS
  for (int it = 0; it < nmy; ++it) {
    char* buf = sm + (it % DB) * STAGE;
    const int p0 = (pb + it * PB) * TM;
    if constexpr (PRO != 0) {
#pragma unroll
      for (int j = 0; j < NPASS; ++j) {
        const int r = tr0 + j * RPP, off = r * (K * 2) + ((tcc ^ xswz<K>(r)) << 4);
        const bf16x8 a8 = *(const bf16x8*)(buf + off);
        const bf16x8 b8 = *(const bf16x8*)(buf + XB + off);
        bf16x8 o8;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float o = bf(a8[u]) * ca[u] + cc[u];  // (bn_apply_kernel's order: bn(s0), then + s1 term)
          o += bf(b8[u]) * cb[u] + cd[u];
          if (PRO == 1) o = fmaxf(o, 0.f);
          o8[u] = (short)tobf(o);
        }
        *(bf16x8*)(buf + off) = o8;
        if (xo) __builtin_nontemporal_store(o8, (bf16x8*)(xo + (size_t)(p0 + r) * K + tcc * 8));
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int r = 16 * i + cl;
#pragma unroll
      for (int kk = 0; kk < KKW; ++kk) {
        const bf16x8 xf = *(const bf16x8*)(buf + r * (K * 2) + (((4 * (kk0 + kk) + g) ^ xswz<K>(r)) << 4));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[kk], xf, acc, 0, 0, 0);
      }
      *(f32x4*)(stg + (part * TM + r) * PITCH + (16 * nt + 4 * g) * 4) = acc;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < EP; ++q) {
      const int e = q * 512 + tid;
      if (NE % 512 == 0 || e < NE) {
        const int p = e / NCH, c = e % NCH;
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = 0.f;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const f32x4 a0 = *(const f32x4*)(stg + (ks * TM + p) * PITCH + c * 32);
          const f32x4 a1 = *(const f32x4*)(stg + (ks * TM + p) * PITCH + c * 32 + 16);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            v[u] += a0[u];
            v[4 + u] += a1[u];
          }
        }
        bf16x8 o;
        if constexpr (DG && !SIDE) {
#pragma unroll
          for (int u = 0; u < 8; ++u) o[u] = (short)tobf(v[u]);
        } else if constexpr (DG) {
          const bf16x8 y8 = *(const bf16x8*)(buf + XS + p * (N_ * 2) + c * 16);
          const bf16x8 x8 = *(const bf16x8*)(buf + XS + SB + p * (N_ * 2) + c * 16);
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            o[u] = (short)tobf(bf(y8[u]) > 0.f ? v[u] : 0.f);
            const float d = bf(o[u]);
            s1[u] += d;
            s2[u] += d * bf(x8[u]);
          }
        } else {
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            o[u] = (short)tobf(v[u]);
            s1[u] += v[u];
            s2[u] += v[u] * v[u];
          }
        }
        __builtin_nontemporal_store(o, (bf16x8*)(y + (size_t)(p0 + p) * N_ + c * 8));
      }
    }
    __syncthreads();
  }
  if constexpr (DG && !SIDE) return;
  // statistics: thread tid owns channels 8 (tid % NCH) .. + 7; sum the 512 / NCH owners
  float* red = (float*)sm;  // the ring is idle now: [512][16]
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    red[tid * 16 + u] = s1[u];
    red[tid * 16 + 8 + u] = s2[u];
  }
  __syncthreads();
  if (tid < N_) {
    const int c = tid >> 3, u = tid & 7;
    float a = 0.f, q = 0.f;
    for (int r = c; r < 512; r += NCH) {
      a += red[r * 16 + u];
      q += red[r * 16 + 8 + u];
    }
    ps[(size_t)pb * N_ + tid] = a;
    pq[(size_t)pb * N_ + tid] = DG ? bn_rstd[tid] * (q - bn_mean[tid] * a) : q;
  }
}

// dst[c][r] = src[r][c] for a rows x cols bf16 block (ld_src >= cols): 32 x 32 tiles via LDS.
__global__ __launch_bounds__(256) void transpose_bf16_kernel(int rows, int cols,
                                                            const unsigned short* __restrict__ src,
                                                            int ld_src, unsigned short* __restrict__ dst) {
  __shared__ unsigned short t[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = r < rows && c < cols ? src[(size_t)r * ld_src + c] : 0;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[(size_t)c * rows + r] = t[tx][i];
  }
}

// Many transposes in one launch (ResNet-50: the 1x1 convolutions' data gradients read their
// weights transposed, 20 per step, each a ~5 us launch of its own): entry k of the int64 table
// [n][6] = {src, dst, rows, cols, ld_src, first tile}; block b runs 32 x 32 tile b - first of the
// entry whose tile range holds it (binary search), as transpose_bf16_kernel.
__global__ __launch_bounds__(256) void transpose_bf16_batch_kernel(const long long* __restrict__ tab,
                                                                  int n) {
  __shared__ unsigned short t[32][33];
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1, k = 0;
  while (lo <= hi) {
    const int mid = (lo + hi) >> 1;
    if (tab[6 * mid + 5] <= b) {
      k = mid;
      lo = mid + 1;
    } else {
      hi = mid - 1;
    }
  }
  const unsigned short* src = (const unsigned short*)tab[6 * k];
  unsigned short* dst = (unsigned short*)tab[6 * k + 1];
  const int rows = (int)tab[6 * k + 2], cols = (int)tab[6 * k + 3], ld_src = (int)tab[6 * k + 4];
  const int tl = b - (int)tab[6 * k + 5], tx_n = (cols + 31) / 32;
  const int r0 = (tl / tx_n) * 32, c0 = (tl % tx_n) * 32, tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + tx;
    t[i][tx] = r < rows && c < cols ? src[(size_t)r * ld_src + c] : 0;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows) dst[(size_t)c * rows + r] = t[tx][i];
  }
}

}  // namespace pw

static bool conv1x1_narrow(int K, int N) {
  static const bool on = [] {  // DTFX_CONV1X1_NARROW=0: reductions stay on the implicit GEMM
    const char* e = std::getenv("DTFX_CONV1X1_NARROW");
    return !(e && std::atoi(e) == 0);
  }();
  return on && ((K == 256 && (N == 64 || N == 128)) || (K == 512 && N == 128));
}

bool conv1x1_applies(int M, int K, int N) {
  if (M <= 0 || M % 64) return false;
  if (conv1x1_narrow(K, N)) return true;
  const int nbn = N / pw::NC;  // column blocks: a power of two <= 8 (the XCD pairing)
  return (K == 64 || K == 128 || K == 256) && N % pw::NC == 0 && (nbn & (nbn - 1)) == 0 &&
         nbn <= 8;
}

// Persistent blocks of a launch: 1 or 2 per CU (256 CUs), a multiple of 8 pixel blocks.
static int conv1x1_blocks(int mode, int K) {
  return mode == 2 || K == 256 ? 256 : 512;
}

// Partial statistics rows a launch of this mode writes ([rows][N] each of ps / pq).
int conv1x1_rows(int mode, int M, int K, int N) {
  (void)M;
  if (conv1x1_narrow(K, N)) return 256;
  return conv1x1_blocks(mode, K) / (N / pw::NC);
}

template <int K, int N_, bool DG, int PRO = 0>
static void conv1x1_narrow_go(int M, const void* x, const void* w, void* y, const void* relu_y,
                              const void* bn_x, const float* mean, const float* rstd, float* ps,
                              float* pq, hipStream_t s, const void* s1 = nullptr,
                              const BnCoefSrc& coef = BnCoefSrc{}, void* xo = nullptr) {
  using namespace pw;
  constexpr int TM = ntm<K, N_, DG, PRO>(), NQT = nqt_narrow<K, N_, DG, PRO>();
  constexpr int DB = 2 * NQT <= 63 ? 4 : 3;
  constexpr size_t ring = (size_t)DB * (TM * K * 2 * (PRO ? 2 : 1) + (nside<DG, PRO>() ? 2 * TM * N_ * 2 : 0));
  constexpr size_t lds = ring + (size_t)(8 / (N_ / 16)) * TM * (N_ * 4 + 16);
  static_assert(ring >= 512 * 16 * 4, "the statistics reduction reuses the ring");
  static_assert(lds <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv1x1_narrow_kernel<K, N_, DG, PRO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL((conv1x1_narrow_kernel<K, N_, DG, PRO>), dim3(256), dim3(576), lds, s, M,
                     (const unsigned short*)x, (const unsigned short*)w, (unsigned short*)y,
                     (const unsigned short*)relu_y, (const unsigned short*)bn_x, mean, rstd, ps, pq,
                     (const unsigned short*)s1, coef, (unsigned short*)xo);
}

template <int K, int PRO = 0>
static void conv1x1_fwd_go(dim3 grid, int M, int N, const void* x, const void* w, int ldw, void* y,
                           float* ps, float* pq, hipStream_t s, const BnCoefSrc& coef = BnCoefSrc{},
                           void* xo = nullptr) {
  using namespace pw;
  const size_t lds = (size_t)NBUF * ftm<K>() * K * 2 + (size_t)ftm<K>() * OPITCH +
                     (PRO ? (size_t)2 * K * 4 : 0);
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv1x1_fwd_kernel<K, PRO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL((conv1x1_fwd_kernel<K, PRO>), grid, dim3(576), lds, s, M, N,
                     (const unsigned short*)x, (const unsigned short*)w, ldw, (unsigned short*)y, ps,
                     pq, coef, (unsigned short*)xo);
}

template <int K, bool RES, bool BN, int PRO = 0>
static void conv1x1_dgrad_go(dim3 grid, int M, int N, const void* dy, const void* w, int ldw,
                             void* dx, const void* res, const void* relu_y, const void* bn_x,
                             const float* mean, const float* rstd, float* ps, float* pq,
                             hipStream_t s, const void* src1 = nullptr,
                             const BnCoefSrc& coef = BnCoefSrc{}, void* xo = nullptr, int rs_h = 0,
                             int rs_w = 0) {
  using namespace pw;
  const size_t lds =
      (size_t)dgrad_ring<K, RES, BN, PRO>() *
          (DTM * K * 2 * (PRO ? 2 : 1) + ((RES ? 1 : 0) + (BN ? 2 : 0)) * DTM * NC * 2) +
      (size_t)DTM * SPITCH;
  static_assert(PRO == 0 || (size_t)dgrad_ring<K, RES, BN, PRO>() *
                                    (DTM * K * 2 * 2 + ((RES ? 1 : 0) + (BN ? 2 : 0)) * DTM * NC * 2) +
                                (size_t)DTM * SPITCH <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)conv1x1_dgrad_kernel<K, RES, BN, PRO>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL((conv1x1_dgrad_kernel<K, RES, BN, PRO>), grid, dim3(576), lds, s, M, N,
                     (const unsigned short*)dy, (const unsigned short*)w, ldw, (unsigned short*)dx,
                     (const unsigned short*)res, (const unsigned short*)relu_y,
                     (const unsigned short*)bn_x, mean, rstd, ps, pq, (const unsigned short*)src1,
                     coef, (unsigned short*)xo, rs_h, rs_w);
}

template <int K, int PRO = 0>
static void conv1x1_dgrad_pick(dim3 grid, int M, int N, const void* dy, const void* w, int ldw,
                               void* dx, const void* res, const void* relu_y, const void* bn_x,
                               const float* mean, const float* rstd, float* ps, float* pq,
                               hipStream_t s, const void* src1 = nullptr,
                               const BnCoefSrc& coef = BnCoefSrc{}, void* xo = nullptr, int rs_h = 0,
                               int rs_w = 0) {
  if (res && ps)
    conv1x1_dgrad_go<K, true, true, PRO>(grid, M, N, dy, w, ldw, dx, res, relu_y, bn_x, mean, rstd, ps, pq, s, src1, coef, xo, rs_h, rs_w);
  else if (res)
    conv1x1_dgrad_go<K, true, false, PRO>(grid, M, N, dy, w, ldw, dx, res, relu_y, bn_x, mean, rstd, ps, pq, s, src1, coef, xo, rs_h, rs_w);
  else if (ps)
    conv1x1_dgrad_go<K, false, true, PRO>(grid, M, N, dy, w, ldw, dx, res, relu_y, bn_x, mean, rstd, ps, pq, s, src1, coef, xo, rs_h, rs_w);
  else
    conv1x1_dgrad_go<K, false, false, PRO>(grid, M, N, dy, w, ldw, dx, res, relu_y, bn_x, mean, rstd, ps, pq, s, src1, coef, xo, rs_h, rs_w);
}

// mode 1: forward (x [M][K], w [N][ldw]); mode 2: data gradient (x = dy [M][K], w [K][ldw],
// optional residual; with ps / pq the ReLU mask relu_y and the BN statistics of bn_x / mean /
// rstd).  ps / pq (optional): conv1x1_rows() partial rows of N floats each.  wt (dgrad): an
// N x K bf16 workspace for the transposed weights.
void conv1x1_launch(int mode, int M, int K, int N, const void* x, const void* w, int ldw, void* y,
                    const void* res, const void* relu_y, const void* bn_x, const float* mean,
                    const float* rstd, float* ps, float* pq, void* wt, hipStream_t s) {
  using namespace pw;
  if (!conv1x1_applies(M, K, N)) throw std::runtime_error("conv1x1: unsupported shape");
  if (ldw % 8 || (mode == 1 ? ldw < K : ldw < N) ||
      (((uintptr_t)x | (uintptr_t)w | (uintptr_t)y | (uintptr_t)res | (uintptr_t)relu_y |
        (uintptr_t)bn_x) & 15))
    throw std::runtime_error("conv1x1: ldw % 8, ldw >= reduction row, 16-B aligned tensors");
  if ((ps != nullptr) != (pq != nullptr) ||
      (mode == 2 && ps && (!relu_y || !bn_x || !mean || !rstd)))
    throw std::runtime_error("conv1x1: statistics need ps, pq (and for dgrad relu_y, bn_x, mean, rstd)");
  if (mode == 2 && relu_y && !ps)
    throw std::runtime_error("conv1x1: the ReLU mask comes with the BN statistics");
  if (conv1x1_narrow(K, N)) {
    // one partial statistics row per block, always written (the model's reductions all feed
    // a BatchNorm); dgrad: the mask / statistics are required, no shortcut gradient
    if (!ps || (mode == 1 && ldw != K) || (mode == 2 && (res || !relu_y)) || (mode != 1 && mode != 2))
      throw std::runtime_error("conv1x1 narrow: statistics required, ldw == K (forward), "
                               "no residual and relu_y given (dgrad)");
    const void* wv = w;
    if (mode == 2) {
      if (!wt || ((uintptr_t)wt & 15)) throw std::runtime_error("conv1x1 dgrad: 16-B aligned wt workspace");
      if (w)  // (w null: wt already holds the transposed copy, transpose_bf16_batch_launch)
        hipLaunchKernelGGL(transpose_bf16_kernel, dim3((N + 31) / 32, K / 32), dim3(256), 0, s, K, N,
                           (const unsigned short*)w, ldw, (unsigned short*)wt);
      wv = wt;
    }
#define DTFX_PW_NARROW(KV, NV)                                                                  \
  do {                                                                                          \
    if (mode == 1) conv1x1_narrow_go<KV, NV, false>(M, x, wv, y, relu_y, bn_x, mean, rstd, ps, pq, s); \
    else conv1x1_narrow_go<KV, NV, true>(M, x, wv, y, relu_y, bn_x, mean, rstd, ps, pq, s);     \
  } while (0)
    if (K == 256 && N == 64) DTFX_PW_NARROW(256, 64);
    else if (K == 256) DTFX_PW_NARROW(256, 128);
    else DTFX_PW_NARROW(512, 128);
#undef DTFX_PW_NARROW
    DTFX_HIP_CHECK(hipGetLastError());
    return;
  }
  const dim3 grid(conv1x1_blocks(mode, K));
  if (mode == 1) {
    if (K == 64) conv1x1_fwd_go<64>(grid, M, N, x, w, ldw, y, ps, pq, s);
    else if (K == 128) conv1x1_fwd_go<128>(grid, M, N, x, w, ldw, y, ps, pq, s);
    else conv1x1_fwd_go<256>(grid, M, N, x, w, ldw, y, ps, pq, s);
  } else if (mode == 2) {
    if (!wt || ((uintptr_t)wt & 15)) throw std::runtime_error("conv1x1 dgrad: 16-B aligned wt workspace");
    if (w)  // (w null: wt already holds the transposed copy)
      hipLaunchKernelGGL(transpose_bf16_kernel, dim3(N / 32, K / 32), dim3(256), 0, s, K, N,
                         (const unsigned short*)w, ldw, (unsigned short*)wt);
    w = wt;
    if (K == 64) conv1x1_dgrad_pick<64>(grid, M, N, x, w, ldw, y, res, relu_y, bn_x, mean, rstd, ps, pq, s);
    else if (K == 128) conv1x1_dgrad_pick<128>(grid, M, N, x, w, ldw, y, res, relu_y, bn_x, mean, rstd, ps, pq, s);
    else conv1x1_dgrad_pick<256>(grid, M, N, x, w, ldw, y, res, relu_y, bn_x, mean, rstd, ps, pq, s);
  } else {
    throw std::runtime_error("conv1x1: mode 1 (forward) or 2 (dgrad)");
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

// The 1x1 products with a BatchNorm prologue (PRO; coef: f32 [4][K] from bn_fwd_coef /
// bn_bwd_coef in cnn.hip), op = the product's reduction operand formed per tile:
//  mode 1 (narrow forward):  op = relu((s0 a + c) + (s1 b + d)) -> xo; y = op W^T + statistics
//          rows (a bottleneck output inside the next conv1);
//  mode 2 (data gradient):   op = (s0 a + c) + (s1 b + d) -> xo (may be null); narrow: y = de
//          = (op W) * (relu_y > 0) + BN-backward rows of bn_x / mean / rstd; wide: as
//          conv1x1_launch mode 2 (+ residual, optional BN);
//  mode 3 (wide forward):    op = relu(s0 a + c) -> xo; y = op W^T + statistics rows (a BN +
//          ReLU inside the following expansion conv).
// Partial statistics rows: conv1x1_rows().  coef: the [4][K] rows of bn_fwd_coef /
// bn_bwd_coef, or (rows null) the BatchNorm's own sources, the coefficients then formed by
// every block (bn_common.h BnCoefSrc) -- no coefficient launch.
bool conv1x1_pro_applies(int mode, int M, int K, int N) {
  if (M <= 0 || M % 64) return false;
  const bool narrow = conv1x1_narrow(K, N);
  if (mode == 1) return narrow;
  if (mode == 3) return !narrow && conv1x1_applies(M, K, N);
  return mode == 2 && conv1x1_applies(M, K, N);
}
void conv1x1_pro_launch(int mode, int M, int K, int N, const void* s0, const void* s1,
                        const BnCoefSrc& coef, void* xo, const void* w, int ldw, void* y,
                        const void* res, const void* relu_y, const void* bn_x, const float* mean,
                        const float* rstd, float* ps, float* pq, void* wt, hipStream_t s,
                        int res_h, int res_w) {
  using namespace pw;
  if (res_w && (mode != 2 || !res || conv1x1_narrow(K, N) || res_h <= 0 || res_h % 2 ||
                res_w % 2 || res_w < pw::DTM || M % (res_h * res_w) || M >= (1 << 24)))
    throw std::runtime_error("conv1x1_pro: a stride-2 (compact) residual needs the wide data "
                             "gradient and even res_h / res_w dividing the pixels");
  if (!conv1x1_pro_applies(mode, M, K, N)) throw std::runtime_error("conv1x1_pro: unsupported shape");
  const bool narrow = conv1x1_narrow(K, N);
  const bool formed = !coef.rows;  // coefficients formed in the kernel from the BN's sources
  if (formed && (!coef.gamma || (coef.bwd ? (!coef.mean || !coef.rstd || !coef.sum_dy ||
                                             !coef.sum_dyxh)
                                           : (!coef.beta || !coef.st.ssum || !coef.st.ssq ||
                                              !coef.st.mean_out || !coef.st.rstd_out)) ||
                 (coef.bwd != 0) != (mode == 2)))
    throw std::runtime_error("conv1x1_pro: formed coefficients need the BatchNorm's sources "
                             "(forward: sums, affine, mean / rstd outputs; backward: mean, rstd, "
                             "gamma, reductions)");
  if (!s0 || (mode != 3 && !s1) || ((mode == 1 || mode == 3) && (!xo || !ps || !pq)) ||
      (mode == 1 && ldw != K) || (mode == 2 && !wt) ||
      (mode == 2 && narrow && res) || (mode == 2 && !ps && narrow && (relu_y || bn_x)) ||
      ((ps != nullptr) != (pq != nullptr)) || (mode == 2 && ps && (!relu_y || !bn_x || !mean || !rstd)))
    throw std::runtime_error("conv1x1_pro: sources, coefficients, statistics (and for the data "
                             "gradient wt, relu_y, bn_x, mean, rstd) required");
  if (ldw % 8 || (((uintptr_t)s0 | (uintptr_t)s1 | (uintptr_t)xo | (uintptr_t)w | (uintptr_t)y |
                   (uintptr_t)res | (uintptr_t)relu_y | (uintptr_t)bn_x | (uintptr_t)wt |
                   (uintptr_t)coef.rows) & 15))
    throw std::runtime_error("conv1x1_pro: ldw % 8, 16-B aligned tensors");
  const void* wv = w;
  if (mode == 2) {
    if (w)  // (w null: wt already holds the transposed copy)
      hipLaunchKernelGGL(transpose_bf16_kernel, dim3((N + 31) / 32, K / 32), dim3(256), 0, s, K, N,
                         (const unsigned short*)w, ldw, (unsigned short*)wt);
    wv = wt;
  }
  if (narrow) {
#define DTFX_PW_PRO(KV, NV)                                                                     \
  do {                                                                                          \
    if (mode == 1)                                                                              \
      conv1x1_narrow_go<KV, NV, false, 1>(M, s0, wv, y, nullptr, nullptr, nullptr, nullptr, ps, pq, \
                                          s, s1, coef, xo);                                     \
    else if (ps)                                                                                \
      conv1x1_narrow_go<KV, NV, true, 2>(M, s0, wv, y, relu_y, bn_x, mean, rstd, ps, pq, s, s1, \
                                         coef, xo);                                             \
    else                                                                                        \
      conv1x1_narrow_go<KV, NV, true, 4>(M, s0, wv, y, nullptr, nullptr, nullptr, nullptr,      \
                                         nullptr, nullptr, s, s1, coef, xo);                    \
  } while (0)
    if (K == 256 && N == 64) DTFX_PW_PRO(256, 64);
    else if (K == 256) DTFX_PW_PRO(256, 128);
    else DTFX_PW_PRO(512, 128);
#undef DTFX_PW_PRO
  } else {
    const dim3 grid(conv1x1_blocks(mode == 3 ? 1 : 2, K));
    if (mode == 3) {
      if (K == 64) conv1x1_fwd_go<64, 3>(grid, M, N, s0, w, ldw, y, ps, pq, s, coef, xo);
      else if (K == 128) conv1x1_fwd_go<128, 3>(grid, M, N, s0, w, ldw, y, ps, pq, s, coef, xo);
      else conv1x1_fwd_go<256, 3>(grid, M, N, s0, w, ldw, y, ps, pq, s, coef, xo);
    } else {
      if (K == 64) conv1x1_dgrad_pick<64, 2>(grid, M, N, s0, wv, ldw, y, res, relu_y, bn_x, mean, rstd, ps, pq, s, s1, coef, xo, res_h, res_w);
      else if (K == 128) conv1x1_dgrad_pick<128, 2>(grid, M, N, s0, wv, ldw, y, res, relu_y, bn_x, mean, rstd, ps, pq, s, s1, coef, xo, res_h, res_w);
      else conv1x1_dgrad_pick<256, 2>(grid, M, N, s0, wv, ldw, y, res, relu_y, bn_x, mean, rstd, ps, pq, s, s1, coef, xo, res_h, res_w);
    }
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

// (host entry points: the coefficient rows of bn_fwd_coef / bn_bwd_coef ...)
void conv1x1_pro_launch(int mode, int M, int K, int N, const void* s0, const void* s1,
                        const float* coef, void* xo, const void* w, int ldw, void* y,
                        const void* res, const void* relu_y, const void* bn_x, const float* mean,
                        const float* rstd, float* ps, float* pq, void* wt, hipStream_t s,
                        int res_h, int res_w) {
  if (!coef) throw std::runtime_error("conv1x1_pro: coefficient rows required");
  BnCoefSrc cs{};
  cs.rows = coef;
  conv1x1_pro_launch(mode, M, K, N, s0, s1, cs, xo, w, ldw, y, res, relu_y, bn_x, mean, rstd, ps,
                     pq, wt, s, res_h, res_w);
}
// ... or the forward BatchNorm's sources (modes 1 / 3: the statistics of s0 over Mst rows, its
// affine, the residual's own BN for mode 1 with sum2 set): mean / rstd / running statistics as
// bn_fwd_coef_launch writes them, by block 0 of the conv
void conv1x1_pro_fwdbn_launch(int mode, int M, int K, int N, const void* s0, const void* s1,
                              long long Mst, const float* sum, const float* sq, float eps,
                              float* mean_out, float* rstd_out, float* run_mean, float* run_var,
                              float momentum, const float* gamma, const float* beta,
                              const float* sum2, const float* sq2, const float* g2,
                              const float* b2, float* mean2, float* rstd2, float* run_mean2,
                              float* run_var2, void* xo, const void* w, int ldw, void* y,
                              float* ps, float* pq, hipStream_t s) {
  if (mode != 1 && mode != 3) throw std::runtime_error("conv1x1_pro_fwdbn: mode 1 or 3");
  if (sum2 && (mode != 1 || !sq2 || !g2 || !b2 || !mean2 || !rstd2))
    throw std::runtime_error("conv1x1_pro_fwdbn: the residual BN (mode 1) needs sq2, gamma2, "
                             "beta2, mean2, rstd2");
  const float inv_m = 1.f / (float)Mst, unbias = Mst > 1 ? (float)Mst / (float)(Mst - 1) : 1.f;
  BnCoefSrc cs{};
  cs.st = BnStats{sum, sq, inv_m, eps, unbias, momentum, mean_out, rstd_out, run_mean, run_var,
                  nullptr, nullptr};
  if (sum2)
    cs.st2 = BnStats{sum2, sq2, inv_m, eps, unbias, momentum, mean2, rstd2, run_mean2, run_var2,
                     g2, b2};
  cs.gamma = gamma;
  cs.beta = beta;
  conv1x1_pro_launch(mode, M, K, N, s0, s1, cs, xo, w, ldw, y, nullptr, nullptr, nullptr,
                     nullptr, nullptr, ps, pq, nullptr, s, 0, 0);
}
// ... or the backward BatchNorm's sources (mode 2: mean / rstd of the BN, its gamma and the
// final reductions sum_dy / sum_dyxh over Mst rows)
void conv1x1_pro_bwdbn_launch(int M, int K, int N, const void* s0, const void* s1,
                              long long Mst, const float* bmean, const float* brstd,
                              const float* gamma, const float* sum_dy, const float* sum_dyxh,
                              void* xo, const void* w, int ldw, void* y, const void* res,
                              const void* relu_y, const void* bn_x, const float* mean,
                              const float* rstd, float* ps, float* pq, void* wt, hipStream_t s,
                              int res_h, int res_w) {
  BnCoefSrc cs{};
  cs.bwd = 1;
  cs.gamma = gamma;
  cs.mean = bmean;
  cs.rstd = brstd;
  cs.sum_dy = sum_dy;
  cs.sum_dyxh = sum_dyxh;
  cs.inv_m = 1.f / (float)Mst;
  conv1x1_pro_launch(2, M, K, N, s0, s1, cs, xo, w, ldw, y, res, relu_y, bn_x, mean, rstd, ps, pq,
                     wt, s, res_h, res_w);
}

// tab: int64 [n][6] on the device (transpose_bf16_batch_kernel); tiles: the sum of every
// entry's ceil(rows / 32) * ceil(cols / 32)
void transpose_bf16_batch_launch(const long long* tab, int n, int tiles, hipStream_t s) {
  if (n <= 0 || tiles <= 0 || !tab) throw std::runtime_error("transpose_bf16_batch: empty table");
  hipLaunchKernelGGL(pw::transpose_bf16_batch_kernel, dim3(tiles), dim3(256), 0, s, tab, n);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
