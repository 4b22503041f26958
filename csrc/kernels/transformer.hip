// Transformer (BERT-base) kernels for gfx950: LayerNorm fwd/bwd, fused
// embedding-sum + LayerNorm, embedding backward, fused self-attention
// forward/backward (one workgroup per (sequence, head), everything in LDS),
// mixed-precision Adam.  North-star config 5 of BASELINE.json (BERT-base MLM
// bf16); the reference has no transformer (it runs an MLP, worker.py:47-54).
//
// Conventions: activations bf16 row-major [tokens][features]; LayerNorm
// gamma/beta, statistics and all gradients of parameters f32; attention
// reads the fused QKV projection output [T][3*Hd] in place (head h of Q at
// columns h*64, of K at Hd + h*64, of V at 2*Hd + h*64) and writes its
// gradient into the same layout, so no transpose/permute pass exists.
#include "common.h"

#include <cstdlib>
#include <stdexcept>
#include <string>

namespace dtfx {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

namespace tf {

__device__ __forceinline__ float bf(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float tobf_round(float f) { return bf(tobf(f)); }
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

// Reductions inside one 16-lane DPP row (the 16 lanes of an MFMA C/D tile that
// share a row group).
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false)));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));
  return v;
}

// MFMA 16x16x32 bf16 operand fragment from an LDS matrix with row pitch `ld`
// bytes: lane gets X[outer = o0 + (lane & 15)][k = k0 + 8 (lane >> 4) + j].
//  KC : element (outer, k) at base + outer*ld + 2k   (one ds_read_b128)
//  !KC: element (outer, k) at base + k*ld + 2*outer  (two ds_read_b64_tr_b16)
template <bool KC>
__device__ __forceinline__ bf16x8 lfrag(const char* base, int ld, int o0, int k0, int lane) {
  if (KC) {
    return *(const bf16x8*)(base + (o0 + (lane & 15)) * ld + (k0 + 8 * (lane >> 4)) * 2);
  } else {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const char* a = base + (k0 + 8 * g + q) * ld + (o0 + 4 * p) * 2;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)a);
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(a + 4 * ld));
    bf16x8 v;
    v.lo = lo;
    v.hi = hi;
    return v;
  }
}
__device__ __forceinline__ f32x4 mma(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
}  // namespace tf

using namespace tf;

// ---------------------------------------------------------------------------
// LayerNorm: one wave per row, H % 8 == 0, H <= 2048 (<= 4 16-B chunks/lane)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void layernorm_fwd_kernel(
    int T, int H, const unsigned short* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, unsigned short* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= T) return;
  const int nch = H >> 3;
  float v[4][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      unpack8(*(const bf16x8*)(x + (size_t)row * H + ch * 8), v[c]);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[c][u];
    }
  }
  const float mean = wave_sum(s) / H;
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (lane + 64 * c < nch)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float d = v[c][u] - mean;
        s2 += d * d;
      }
  const float rstd = rsqrtf(wave_sum(s2) / H + eps);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        o[u] = (v[c][u] - mean) * rstd * gamma[ch * 8 + u] + beta[ch * 8 + u];
      __builtin_nontemporal_store(pack8(o), (bf16x8*)(y + (size_t)row * H + ch * 8));
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// The same LayerNorm forward with R rows per wave, all R rows' loads issued before the first
// row is reduced (one memory round trip per R rows instead of per row) and gamma / beta held in
// registers; NC = ceil(H / 512) 8-column chunks per lane.
template <int NC, int R>
__global__ __launch_bounds__(256) void layernorm_fwd_rows_kernel(
    int T, int H, const unsigned short* __restrict__ x, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, unsigned short* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + wave) * R;
  if (row0 >= T) return;
  const int nch = H >> 3;
  bf16x8 raw[R][NC];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int rr = min(row0 + i, T - 1);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = min(lane + 64 * c, nch - 1);  // clamped: masked at use
      raw[i][c] = __builtin_nontemporal_load((const bf16x8*)(x + (size_t)rr * H + ch * 8));
    }
  }
  float gm[NC][8], bt[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = min(lane + 64 * c, nch - 1);
    *(f32x4*)&gm[c][0] = *(const f32x4*)(gamma + ch * 8);
    *(f32x4*)&gm[c][4] = *(const f32x4*)(gamma + ch * 8 + 4);
    *(f32x4*)&bt[c][0] = *(const f32x4*)(beta + ch * 8);
    *(f32x4*)&bt[c][4] = *(const f32x4*)(beta + ch * 8 + 4);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int row = row0 + i;
    if (row >= T) break;
    float v[NC][8];
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      unpack8(raw[i][c], v[c]);
      if (lane + 64 * c < nch)
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[c][u];
    }
    const float mean = wave_sum(s) / H;
    float s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (lane + 64 * c < nch)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const float d = v[c][u] - mean;
          s2 += d * d;
        }
    const float rstd = rsqrtf(wave_sum(s2) / H + eps);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nch) {
        float o[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) o[u] = (v[c][u] - mean) * rstd * gm[c][u] + bt[c][u];
        __builtin_nontemporal_store(pack8(o), (bf16x8*)(y + (size_t)row * H + ch * 8));
      }
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g * xhat)),  g = dy * gamma
// dgamma += sum dy * xhat, dbeta += sum dy (per block in registers, then atomics)
// optional dres: dx += dres (the residual branch gradient, fused)
// NC = ceil(H / 512) column chunks of 8 per lane.  Each of the NWV waves streams rows r0+wave, +NWV, ...
// with the NEXT row's x / dy / dres loads issued before the current row is reduced
// (software pipeline: one memory round trip per row instead of two) and gamma hoisted.
// NS row slots per wave (NS - 1 rows in flight while one is reduced): 2 by default, 3 with
// DTFX_LN_SLOTS=3 (H <= 1024 only: 4 slots spill at H = 768).
template <int NC, int NS = 2>
__global__ __launch_bounds__(NC <= 2 ? 512 : 256) void layernorm_bwd_kernel(
    int T, int H, int rows_per_block, const unsigned short* __restrict__ dy,
    const unsigned short* __restrict__ x, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma,
    const unsigned short* __restrict__ dres, unsigned short* __restrict__ dx,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dxsum) {
  // waves per block: 8 (2 per SIMD hide the per-row reduction latency; 26.5 -> 24.1 us at
  // the BERT shape) while the registers allow it, else 4
  constexpr int NWV = NC <= 2 ? 8 : 4;
  __shared__ float red[3][NWV][8 * 72];  // [dgamma|dbeta|dxsum][wave][u * 72 + lane], one chunk
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nch = H >> 3;
  float dg[NC][8], db[NC][8], ds[NC][8], gm[NC][8];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int ch = lane + 64 * c;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      dg[c][u] = db[c][u] = ds[c][u] = 0.f;
      gm[c][u] = ch < nch ? gamma[ch * 8 + u] : 0.f;
    }
  }
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(T, r0 + rows_per_block);
  // Two rows in flight per wave beyond the one being reduced (register double buffer, two
  // rows per trip so the buffer index stays literal): with one, every row waited out most of
  // a memory round trip (the kernel ran at ~1/2 of its HBM bound at the BERT shape).
  bf16x8 xb[NS][NC], yb[NS][NC], rb[NS][NC];
  float mb[NS] = {}, rsb[NS] = {};
  auto load = [&](int p, int row) {
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int ch = min(lane + 64 * c, nch - 1);  // clamped: masked at use
      xb[p][c] = __builtin_nontemporal_load((const bf16x8*)(x + (size_t)row * H + ch * 8));
      yb[p][c] = __builtin_nontemporal_load((const bf16x8*)(dy + (size_t)row * H + ch * 8));
      if (dres) rb[p][c] = __builtin_nontemporal_load((const bf16x8*)(dres + (size_t)row * H + ch * 8));
    }
    mb[p] = mean_in[row];
    rsb[p] = rstd_in[row];
  };
  const int first = r0 + wave;
  const int nrows = first < r1 ? (r1 - first + NWV - 1) / NWV : 0;  // rows of this wave
#pragma unroll
  for (int p = 0; p < NS; ++p)
    if (nrows > p) load(p, first + p * NWV);
  for (int i = 0; i < nrows; i += NS) {
#pragma unroll
    for (int p = 0; p < NS; ++p) {
      if (i + p >= nrows) break;
      const int row = first + (i + p) * NWV;
      float xh[NC][8], g[NC][8], dyv[NC][8], rv[NC][8];
      float s1 = 0.f, s2 = 0.f;
      const float mu = mb[p], rs = rsb[p];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bool ok = lane + 64 * c < nch;
        float xv[8];
        unpack8(xb[p][c], xv);
        unpack8(yb[p][c], dyv[c]);
        if (dres) unpack8(rb[p][c], rv[c]);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (!ok) dyv[c][u] = 0.f;
          xh[c][u] = (xv[u] - mu) * rs;
          g[c][u] = dyv[c][u] * gm[c][u];
          s1 += g[c][u];
          s2 += g[c][u] * xh[c][u];
          dg[c][u] += dyv[c][u] * xh[c][u];
          db[c][u] += dyv[c][u];
        }
      }
      if (i + p + NS < nrows) load(p, row + NS * NWV);  // in flight during the reductions
      s1 = wave_sum(s1) / H;
      s2 = wave_sum(s2) / H;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int ch = lane + 64 * c;
        if (ch < nch) {
          float o[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            o[u] = rs * (g[c][u] - s1 - xh[c][u] * s2);
            if (dres) o[u] += rv[c][u];
            ds[c][u] += o[u];
          }
          __builtin_nontemporal_store(pack8(o), (bf16x8*)(dx + (size_t)row * H + ch * 8));
        }
      }
    }
  }
  // cross-wave reduction of the parameter-gradient partials, then one atomic per column:
  // one pass per column chunk c (512 columns), LDS image [array][wave][u * 72 + lane].
  // Writes (fixed u, lanes 0..63) and reads (thread j -> column 512c + j, u = j % 8,
  // lane = j / 8: bank 8u + lane) are both bank-conflict free, and each wave's atomics
  // cover 64 CONSECUTIVE columns (2 cache lines: atomics to scattered lines serialise).
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c > 0) __syncthreads();
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      red[0][wave][u * 72 + lane] = dg[c][u];
      red[1][wave][u * 72 + lane] = db[c][u];
      red[2][wave][u * 72 + lane] = ds[c][u];
    }
    __syncthreads();
    for (int j = threadIdx.x; j < 512; j += 64 * NWV) {
      const int col = 512 * c + j;
      if (col >= H) continue;
      const int i = (j & 7) * 72 + (j >> 3);
      float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
      for (int w = 0; w < NWV; ++w) {
        a += red[0][w][i];
        b += red[1][w][i];
        d += red[2][w][i];
      }
      unsafeAtomicAdd(dgamma + col, a);
      unsafeAtomicAdd(dbeta + col, b);
      if (dxsum) unsafeAtomicAdd(dxsum + col, d);
    }
  }
}

// H = 768 (BERT-base) form of layernorm_bwd_kernel with about half the registers: 12 columns
// per lane as three 4-column chunks (lane l: columns 256 c + 4 l .. + 3, so each load
// instruction covers 512 contiguous bytes), the row slots kept as bf16 and re-read in the
// second pass instead of f32 copies of x-hat / g / dy / dres, gamma in LDS, both row sums in one
// interleaved wave reduction.  <= 128 VGPRs: two 8-wave blocks share a CU (16 waves) and each
// wave reduces 4 rows instead of 8 (the default kernel is bound by its per-wave row latency
// chain, profiles/r6/ln_slots/).  Same outputs and accumulation targets.
template <int NSL>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4))) void layernorm_bwd_h768_kernel(
    int T, int rows_per_block, const unsigned short* __restrict__ dy,
    const unsigned short* __restrict__ x, const float* __restrict__ mean_in,
    const float* __restrict__ rstd_in, const float* __restrict__ gamma,
    const unsigned short* __restrict__ dres, unsigned short* __restrict__ dx,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ dxsum) {
  constexpr int H = 768, NWV = 8;
  __shared__ f32x4 red[3][NWV][H / 4];  // [dgamma|dbeta|dxsum][wave][column quad]
  __shared__ f32x4 gms[H / 4];
  // wave index made provably uniform: row addresses then live in scalar registers (one lane
  // offset VGPR for every load) instead of a 64-bit VGPR pair per load
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (threadIdx.x < H / 4) gms[threadIdx.x] = ((const f32x4*)gamma)[threadIdx.x];
  f32x4 dg[3], db[3], ds[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) dg[c] = db[c] = ds[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(T, r0 + rows_per_block);
  bf16x4 xb[NSL][3], yb[NSL][3], rb[NSL][3];
  float mb[NSL] = {}, rsb[NSL] = {};
  auto load = [&](int p, int row) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const size_t off = (size_t)row * H + 256 * c + 4 * lane;
      xb[p][c] = __builtin_nontemporal_load((const bf16x4*)(x + off));
      yb[p][c] = __builtin_nontemporal_load((const bf16x4*)(dy + off));
      if (dres) rb[p][c] = __builtin_nontemporal_load((const bf16x4*)(dres + off));
    }
    mb[p] = mean_in[row];
    rsb[p] = rstd_in[row];
  };
  const int first = r0 + wave;
  const int nrows = first < r1 ? (r1 - first + NWV - 1) / NWV : 0;  // rows of this wave
#pragma unroll
  for (int p = 0; p < NSL; ++p)
    if (nrows > p) load(p, first + p * NWV);
  __syncthreads();  // gamma in LDS
  for (int i = 0; i < nrows; i += NSL) {
#pragma unroll
    for (int p = 0; p < NSL; ++p) {
      if (i + p >= nrows) break;
      const int row = first + (i + p) * NWV;
      const float mu = mb[p], rs = rsb[p];
      float sum[2] = {0.f, 0.f};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const f32x4 gm = gms[64 * c + lane];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float dyv = bf((unsigned short)yb[p][c][u]);
          const float xh = (bf((unsigned short)xb[p][c][u]) - mu) * rs;
          const float g = dyv * gm[u];
          sum[0] += g;
          sum[1] += g * xh;
          dg[c][u] += dyv * xh;
          db[c][u] += dyv;
        }
      }
      wave_sum_n(sum);
      const float s1 = sum[0] / H, s2 = sum[1] / H;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const f32x4 gm = gms[64 * c + lane];
        bf16x4 o4;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float xh = (bf((unsigned short)xb[p][c][u]) - mu) * rs;
          float o = rs * (bf((unsigned short)yb[p][c][u]) * gm[u] - s1 - xh * s2);
          if (dres) o += bf((unsigned short)rb[p][c][u]);
          ds[c][u] += o;
          o4[u] = (short)tobf(o);
        }
        __builtin_nontemporal_store(o4, (bf16x4*)(dx + (size_t)row * H + 256 * c + 4 * lane));
      }
      if (i + p + NSL < nrows) load(p, row + NSL * NWV);  // the slot is free after the second pass
    }
  }
  // cross-wave reduction (one 16-byte LDS store per lane and array: conflict free), then one
  // atomic per column and array
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    red[0][wave][64 * c + lane] = dg[c];
    red[1][wave][64 * c + lane] = db[c];
    red[2][wave][64 * c + lane] = ds[c];
  }
  __syncthreads();
  const float* rf = (const float*)red;
  for (int j = threadIdx.x; j < H; j += 64 * NWV) {
    float a = 0.f, b = 0.f, d = 0.f;
#pragma unroll
    for (int w = 0; w < NWV; ++w) {
      a += rf[(0 * NWV + w) * H + j];
      b += rf[(1 * NWV + w) * H + j];
      d += rf[(2 * NWV + w) * H + j];
    }
    unsafeAtomicAdd(dgamma + j, a);
    unsafeAtomicAdd(dbeta + j, b);
    if (dxsum) unsafeAtomicAdd(dxsum + j, d);
  }
}

// ---------------------------------------------------------------------------
// Embedding: x = word[ids] + pos[t % S] + type[tt]; y = LN(x).  Saves x (bf16).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void embed_ln_fwd_kernel(
    int T, int S, int H, const int* __restrict__ ids, const int* __restrict__ tt,
    const unsigned short* __restrict__ word, const unsigned short* __restrict__ pos,
    const unsigned short* __restrict__ type, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, unsigned short* __restrict__ xsum,
    unsigned short* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= T) return;
  const int nch = H >> 3;
  const int id = ids[row], ty = tt ? tt[row] : 0, ps = row % S;
  float v[4][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float a[8], b[8], d[8];
      unpack8(*(const bf16x8*)(word + (size_t)id * H + ch * 8), a);
      unpack8(*(const bf16x8*)(pos + (size_t)ps * H + ch * 8), b);
      unpack8(*(const bf16x8*)(type + (size_t)ty * H + ch * 8), d);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        v[c][u] = tobf_round(a[u] + b[u] + d[u]);
        s += v[c][u];
      }
      __builtin_nontemporal_store(pack8(v[c]), (bf16x8*)(xsum + (size_t)row * H + ch * 8));
    }
  }
  const float mean = wave_sum(s) / H;
  float s2 = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (lane + 64 * c < nch)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float d = v[c][u] - mean;
        s2 += d * d;
      }
  const float rstd = rsqrtf(wave_sum(s2) / H + eps);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nch) {
      float o[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        o[u] = (v[c][u] - mean) * rstd * gamma[ch * 8 + u] + beta[ch * 8 + u];
      __builtin_nontemporal_store(pack8(o), (bf16x8*)(y + (size_t)row * H + ch * 8));
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// word-embedding gradient: scatter-add of dx rows (f32 hardware atomics; ids are
// spread over a 30K vocabulary, so contention is low).
__global__ __launch_bounds__(256) void embed_word_bwd_kernel(int T, int H, const int* __restrict__ ids,
                                                             const unsigned short* __restrict__ dx,
                                                             float* __restrict__ dword) {
  // one row per wave; lane l owns columns l, l + 64, ...: every wave-wide atomic covers one
  // contiguous 256-B segment (four full 64-B requests at the memory side) instead of 64
  // lanes scattered 32 B apart
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= T) return;
  float* dst = dword + (size_t)ids[row] * H;
  const unsigned short* src = dx + (size_t)row * H;
  constexpr int U = 12;  // loads in flight per lane (H = 768: the whole row)
  for (int c0 = 0; c0 < H; c0 += 64 * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int col = c0 + u * 64 + lane;
      v[u] = col < H ? bf(src[col]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int col = c0 + u * 64 + lane;
      if (col < H) unsafeAtomicAdd(dst + col, v[u]);
    }
  }
}

// position / token-type gradients: one 1024-thread block per position s; 8 row streams x
// 128 threads of 8 columns (16-B loads, 4 rows in flight) fold into LDS with ds_add_f32,
// then thread i writes column i: dpos row s has a single writer (no atomics), and the
// token-type sums leave as lane-contiguous atomics (S adders per address).
__global__ __launch_bounds__(1024) void embed_pos_type_bwd_kernel(
    int Bn, int S, int H, const int* __restrict__ tt, const unsigned short* __restrict__ dx,
    float* __restrict__ dpos, float* __restrict__ dtype_) {
  __shared__ float red[3][2048];
  const int s = blockIdx.x, stream = threadIdx.x >> 7, t = threadIdx.x & 127;
  const int nch = H >> 3;
  for (int i = threadIdx.x; i < 3 * H; i += 1024) red[i / H][i % H] = 0.f;
  __syncthreads();
  for (int ch = t; ch < nch; ch += 128) {
    float acc[8], t1[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] = t1[u] = 0.f;
    for (int b0 = stream; b0 < Bn; b0 += 32) {
      bf16x8 v[4];
      bool one[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = b0 + 8 * i;
        const int row = (b < Bn ? b : 0) * S + s;
        v[i] = *(const bf16x8*)(dx + (size_t)row * H + ch * 8);
        one[i] = b < Bn && tt && tt[row];
        if (b >= Bn) v[i] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float f[8];
        unpack8(v[i], f);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          acc[u] += f[u];
          t1[u] += one[i] ? f[u] : 0.f;
        }
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      atomicAdd(&red[0][ch * 8 + u], acc[u]);
      atomicAdd(&red[2][ch * 8 + u], t1[u]);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < H; i += 1024) {
    const float a = red[0][i], one = red[2][i];
    dpos[(size_t)s * H + i] += a;
    unsafeAtomicAdd(dtype_ + i, a - one);
    unsafeAtomicAdd(dtype_ + H + i, one);
  }
}

// ---------------------------------------------------------------------------
// Self-attention, one workgroup (4 waves) per (sequence b, head h), S <= 128,
// head dim 64.  Q, K, V (and dO) tiles live in LDS with 144-B rows (16-B pad:
// conflict-free ds_read_b128 row reads); P / dS tiles 128 x 128 with 272-B rows.
// Wave w owns query rows [32w, 32w + 32) for the row-wise products and key
// rows [32w, 32w + 32) for dK / dV.
// ---------------------------------------------------------------------------
namespace at {
constexpr int SP = 128, D = 64;
constexpr int LDQ = D * 2 + 16;    // 144 B
constexpr int LDP = SP * 2 + 16;   // 272 B
constexpr int QB = SP * LDQ;       // 18432 B
constexpr int PB = SP * LDP;       // 34816 B

// XOR-swizzled [rows][64] bf16 images with unpadded 128-B rows (attn_fwd_kernel,
// attn_bwd_half_kernel): 16-B chunk c of row r sits at chunk c ^ swz(r).  Every image is read
// both as rows (ds_read_b128, lfrag_sw<true>) and transposed (ds_read_b64_tr_b16,
// lfrag_sw<false>); the 144-B padded rows were 2-way conflicted on both (the b128 group's rows
// 4 and 13 on one slot, the tr read's rows q and q + 8 likewise: 36-41 % conflict cycles in
// the BERT step's counters).  swz(r) (a linear map of r's low 4 bits, found by exhaustive
// search over them) gives conflict-free b128 row reads -- each 16-lane group's rows {0-3,
// 12-15} at chunk c and {4-11} at c ^ 1 land on 16 distinct slots -- and conflict-free tr reads
// -- the rows {R..R+3, R+8..R+11} of a 32-lane half, two chunks each, on 16 distinct slots --
// and keeps the P^T / dS^T 8-byte stores at 2-way, as before.
constexpr int LDK = D * 2;         // 128 B
constexpr int KB = SP * LDK;       // 16384 B
__device__ __forceinline__ int swz(int r) {
  return (__builtin_popcount(r & 15) & 1) | ((__builtin_popcount(r & 14) & 1) << 1) |
         (((r >> 3) & 1) << 2);
}
// byte offset of element (row r, column col) of a swizzled image
__device__ __forceinline__ int sw_off(int r, int col) {
  return r * LDK + ((((col >> 3) ^ swz(r))) << 4) + (col & 7) * 2;
}

// Load N [S][64] head slices (row stride ld[i] elements) into LDS, zero rows >= S.  All
// 4N 16-B loads of a thread are issued before the first LDS store (one memory round trip
// instead of 4N dependent load -> store pairs).
template <int N, int NT = 256, bool SWZ = false>
__device__ __forceinline__ void load_heads(char* const (&dst)[N], const unsigned short* const (&src)[N],
                                           const int (&ld)[N], int S) {
  constexpr int PER = SP * 8 / NT;  // 16-B chunks per thread per head (NT threads)
  bf16x8 v[N][PER];
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + NT * k, r = i >> 3, c = i & 7;
      v[n][k] = *(const bf16x8*)(src[n] + (size_t)min(r, S - 1) * ld[n] + c * 8);
    }
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = threadIdx.x + NT * k, r = i >> 3, c = i & 7;
      if (r >= S) v[n][k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      *(bf16x8*)(dst[n] + (SWZ ? r * LDK + ((c ^ swz(r)) << 4) : r * LDQ + c * 16)) = v[n][k];
    }
}

// lfrag over a swizzled image (same lane map as tf::lfrag).  swz is XOR-linear in the row's
// low 4 bits and every fragment's first row is a multiple of 16 (row reads) or of 8 with the
// lane's rows fixed modulo 16 (tr reads), so each lane's chunk XORs are constants computed once
// (SwLane): a row read is one immediate offset, a tr read one XOR per fragment.
struct SwLane {
  int rr;  // row reads: the lane's byte offset for k0 = 0 (k0 = 32: ^ 64, since swz(r) < 8)
  int tb;  // tr reads, lo row: row + in-chunk byte offset (k0, o0 excluded; hi row: + 4 rows)
  int ct;  // tr reads, lo row: chunk XOR (hi row: ^ swz(4) = 3, swz being linear and the lo
           // row's bit 2 clear)
};
__device__ __forceinline__ SwLane sw_lane(int lane) {
  // (recomputed at each use from the lane id, a handful of VALU: the half backward sits at its
  //  128-VGPR budget, and three long-lived registers more made it spill)
  SwLane w;
  const int l15 = lane & 15, g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  w.rr = l15 * LDK + (((lane >> 4) ^ swz(l15)) << 4);
  w.tb = (8 * g + q) * LDK + ((4 * p) & 7) * 2;
  w.ct = (p >> 1) ^ swz(8 * (g & 1) + q);
  return w;
}
template <bool KC>
__device__ __forceinline__ bf16x8 lfrag_sw(const char* base, int o0, int k0, int lane) {
  const SwLane w = sw_lane(lane);
  if (KC) {  // k0 in {0, 32} (64-column images)
    return *(const bf16x8*)(base + o0 * LDK + (w.rr ^ (k0 << 1)));
  } else {   // o0 a multiple of 16, k0 of 32
    // (the chunk XOR is formed at each read -- two VALU -- from an opaque copy of the lane's
    //  row offset: hoisted, the 8 distinct (o0, lo / hi) offsets of a loop stay live and the
    //  half backward, at its 128-VGPR budget, spilled)
    int x = w.tb + (w.ct << 4);
    asm volatile("" : "+v"(x));
    const char* b = base + k0 * LDK;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(b + (x ^ (o0 << 1))));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_bf16x4*)(b + 4 * LDK + (x ^ (o0 << 1) ^ (3 << 4))));
    bf16x8 v;
    v.lo = lo;
    v.hi = hi;
    return v;
  }
}
// The two image layouts behind one interface (SWZ: compile-time variant of the kernels below)
template <bool SWZ>
constexpr int img_pitch() { return SWZ ? LDK : LDQ; }
template <bool SWZ>
__device__ __forceinline__ int img_off(int r, int col) {
  return SWZ ? sw_off(r, col) : r * LDQ + col * 2;
}
template <bool SWZ, bool KC>
__device__ __forceinline__ bf16x8 img_frag(const char* base, int o0, int k0, int lane) {
  if constexpr (SWZ) return lfrag_sw<KC>(base, o0, k0, lane);
  else return tf::lfrag<KC>(base, LDQ, o0, k0, lane);
}
}  // namespace at

// Q never goes through LDS: each wave's 32 query rows are only its own A operands, read
// as MFMA fragments straight from global memory (issued before the K/V staging).  K, V
// and P then take 70 KB of LDS: two blocks per CU.
// SWZ (DTFX_ATTN_SWZ=1, opt-in): the K / V images XOR-swizzled (at::swz) instead of padded.
// Conflict-free, but measured slower: LDS bank-conflict cycles 21.6 M -> 4.3 M on the probe,
// 29.7 -> 31.0 us per call, BERT-base -0.3 % (profiles/r6/attn_swizzle/).
template <bool SWZ>
__global__ __launch_bounds__(256, 2) void attn_fwd_kernel(
    int S, int nh, const unsigned short* __restrict__ qkv, unsigned short* __restrict__ out,
    float* __restrict__ lse, const float* __restrict__ kmask, float scale) {
  using namespace at;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  constexpr int IB = SP * img_pitch<SWZ>();  // bytes of one K / V image
  char* Ks = sm;
  char* Vs = sm + IB;
  char* Ps = sm + 2 * IB;
  const int b = blockIdx.x / nh, h = blockIdx.x % nh;
  const int Hd = nh * D, ld = 3 * Hd;
  const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int cl = lane & 15, rg = (lane >> 4) * 4;
  bf16x8 qf[2][2];  // [row group i][k half]: rows 32 wave + 16 i + (lane & 15)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 32 * wave + 16 * i + cl;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[i][kk] = *(const bf16x8*)(base + (size_t)(row < S ? row : S - 1) * ld + 32 * kk +
                                   8 * (lane >> 4));
      if (row >= S) qf[i][kk] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  {
    char* const dst[2] = {Ks, Vs};
    const unsigned short* const src[2] = {base + Hd, base + 2 * Hd};
    const int lds[2] = {ld, ld};
    at::load_heads<2, 256, SWZ>(dst, src, lds, S);
  }
  __syncthreads();

  float km[8];  // additive key mask for this lane's key column in each key tile
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int key = 16 * j + cl;
    km[j] = key < S ? (kmask ? kmask[(size_t)b * S + key] : 0.f) : -INFINITY;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = 32 * wave + 16 * i;
    f32x4 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 a = qf[i][kk];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = mma(a, img_frag<SWZ, true>(Ks, 16 * j, 32 * kk, lane), acc[j]);
    }
    // row softmax: row r0 + rg + r lives in the 16 lanes of this row group x 8 tiles
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float m = -INFINITY;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[j][r] = acc[j][r] * scale + km[j];
        m = fmaxf(m, acc[j][r]);
      }
      m = row16_max(m);
      const float msafe = (m == -INFINITY) ? 0.f : m;
      float l = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        acc[j][r] = __expf(acc[j][r] - msafe);
        l += acc[j][r];
      }
      l = row16_sum(l);
      const float inv = l > 0.f ? 1.f / l : 0.f;
      const int row = r0 + rg + r;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *(unsigned short*)(Ps + row * LDP + (16 * j + cl) * 2) = tobf(acc[j][r] * inv);
      if (cl == 0 && row < S) lse[((size_t)b * nh + h) * SP + row] = msafe + __logf(l);
    }
  }
  __builtin_amdgcn_wave_barrier();  // P rows of this wave are read back only by this wave
  // O = P . V  (32 rows x 64 d per wave, K = 128 keys)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r0 = 32 * wave + 16 * i;
    f32x4 o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bf16x8 a = lfrag<true>(Ps, LDP, r0, 32 * kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = mma(a, img_frag<SWZ, false>(Vs, 16 * j, 32 * kk, lane), o[j]);
    }
    // through this wave's own P rows (consumed by the products above): 2 16-B stores per
    // lane instead of 16 2-byte stores
    char* stg = Ps + (size_t)r0 * LDP;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *(unsigned short*)(stg + (rg + r) * LDP + (16 * j + cl) * 2) = tobf(o[j][r]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = lane + 64 * u, row = r0 + (c >> 3), ch = c & 7;
      const bf16x8 v = *(const bf16x8*)(stg + (c >> 3) * LDP + ch * 16);
      if (row < S) *(bf16x8*)(out + ((size_t)b * S + row) * Hd + h * D + ch * 8) = v;
    }
  }
}

// Register-resident P (round 6): the scores are formed TRANSPOSED,
// S^T = K Q^T (the same two fragments as Q K^T with the MFMA operands swapped), so each lane's
// accumulators hold four consecutive keys of ONE query -- exactly the k-slots of the P . V
// A operand once the two 16-key tiles of a 32-key chunk are paired: lane (query q, group g)
// holds keys 32c + 4g + {0..3} (tile 2c) and 32c + 16 + 4g + {0..3} (tile 2c + 1) as its 8
// k-slots.  The V fragment of P . V reads the same key order with two transposed LDS reads at
// rows 32c + 4g and 32c + 16 + 4g.  P never touches LDS: K + V + the key mask are 36.5 KB,
// four blocks per CU instead of two (attn_fwd_kernel's P image took 34 KB), and the K image
// stages the output once every wave is past its scores.  Softmax over a query's keys: in-lane
// over 32 values, then across the 4 lanes of its column (xor 16, 32).
__global__ __launch_bounds__(256, 4) void attn_fwd_rp_kernel(
    int S, int nh, const unsigned short* __restrict__ qkv, unsigned short* __restrict__ out,
    float* __restrict__ lse, const float* __restrict__ kmask, float scale) {
  using namespace at;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Ks = sm;
  char* Vs = sm + QB;
  float* kms = (float*)(sm + 2 * QB);  // [SP] additive key mask, -inf past S
  const int b = blockIdx.x / nh, h = blockIdx.x % nh;
  const int Hd = nh * D, ld = 3 * Hd;
  const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int cl = lane & 15, g = lane >> 4;
  bf16x8 qf[2][2];  // [row tile i][k half]: B operand of S^T, query 32 wave + 16 i + cl
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 32 * wave + 16 * i + cl;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      qf[i][kk] = *(const bf16x8*)(base + (size_t)(row < S ? row : S - 1) * ld + 32 * kk + 8 * g);
      if (row >= S) qf[i][kk] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
  {
    char* const dst[2] = {Ks, Vs};
    const unsigned short* const src[2] = {base + Hd, base + 2 * Hd};
    const int lds[2] = {ld, ld};
    at::load_heads<2, 256, false>(dst, src, lds, S);
  }
  if (threadIdx.x < SP) {
    const int k = threadIdx.x;
    kms[k] = k < S ? (kmask ? kmask[(size_t)b * S + k] : 0.f) : -INFINITY;
  }
  __syncthreads();
  bf16x8 pf[2][4];  // P of row tile i: A fragments of the four 32-key chunks
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 acc[8];  // acc[j][r] = score(query 32 wave + 16 i + cl, key 16 j + 4 g + r)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = mma(lfrag<true>(Ks, LDQ, 16 * j, 32 * kk, lane), qf[i][kk], acc[j]);
    float m = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f32x4 km = *(const f32x4*)&kms[16 * j + 4 * g];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[j][r] = acc[j][r] * scale + km[r];
        m = fmaxf(m, acc[j][r]);
      }
    }
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    const float msafe = (m == -INFINITY) ? 0.f : m;
    float l = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[j][r] = __expf(acc[j][r] - msafe);
        l += acc[j][r];
      }
    l += __shfl_xor(l, 16);
    l += __shfl_xor(l, 32);
    const float inv = l > 0.f ? 1.f / l : 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        pf[i][c][r] = (short)tobf(acc[2 * c][r] * inv);
        pf[i][c][4 + r] = (short)tobf(acc[2 * c + 1][r] * inv);
      }
    const int row = 32 * wave + 16 * i + cl;
    if (g == 0 && row < S) lse[((size_t)b * nh + h) * SP + row] = msafe + __logf(l);
  }
  __syncthreads();  // every wave is past its scores: the K image becomes the output staging
  // the V fragment of chunk c, columns o0 .. o0 + 15: k-slots e < 4 -> key 32c + 4g + e, e >= 4
  // -> key 32c + 16 + 4g + e - 4 (the P fragment's key order)
  const int q = (lane >> 2) & 3, p4 = (lane & 3) * 4;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    f32x4 o[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const char* a = Vs + (32 * c + 4 * g + q) * LDQ + (16 * j + p4) * 2;
        bf16x8 vf;
        vf.lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)a);
        vf.hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_bf16x4*)(a + 16 * LDQ));
        o[j] = mma(pf[i][c], vf, o[j]);
      }
    // o[j][r] = O(query 32 wave + 16 i + 4 g + r, d 16 j + cl): staged in the wave's own 16
    // rows of the K image, then 16-B stores
    const int r0 = 32 * wave + 16 * i;
    char* stg = Ks + (size_t)r0 * LDQ;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        *(unsigned short*)(stg + (4 * g + r) * LDQ + (16 * j + cl) * 2) = tobf(o[j][r]);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int c = lane + 64 * u, row = r0 + (c >> 3), ch = c & 7;
      const bf16x8 v = *(const bf16x8*)(stg + (c >> 3) * LDQ + ch * 16);
      if (row < S) *(bf16x8*)(out + ((size_t)b * S + row) * Hd + h * D + ch * 8) = v;
    }
  }
}

// NW waves per (sequence, head): 4 (32 query / key rows per wave) or 8 (16 rows per wave:
// the 144 KB of LDS allow one block per CU, so 8 waves give every SIMD two waves to
// overlap LDS / global latency with the other's MFMAs).
template <int NW>
__global__ __launch_bounds__(NW * 64, 1) void attn_bwd_kernel(
    int S, int nh, const unsigned short* __restrict__ qkv, const unsigned short* __restrict__ o,
    const unsigned short* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ kmask, float scale, unsigned short* __restrict__ dqkv,
    float* __restrict__ dbias) {
  using namespace at;
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  constexpr int NT = NW * 64, RPW = SP / NW, NI = RPW / 16;  // rows per wave, 16-row tiles
  constexpr int TPR = NT / SP, CPT = 64 / TPR / 8;           // rowsum: threads / row, chunks
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Qs = sm;
  char* Ks = sm + QB;
  char* Vs = sm + 2 * QB;
  char* dOs = sm + 3 * QB;
  char* Ps = sm + 4 * QB;
  char* dSs = Ps + PB;
  float* Dr = (float*)(dSs + PB);  // [128] rowsum(dO * O)
  const int b = blockIdx.x / nh, h = blockIdx.x % nh;
  const int Hd = nh * D, ld = 3 * Hd;
  const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
  {
    char* const dst[4] = {Qs, Ks, Vs, dOs};
    const unsigned short* const src[4] = {base, base + Hd, base + 2 * Hd,
                                          dout + (size_t)b * S * Hd + h * D};
    const int lds[4] = {ld, ld, ld, Hd};
    at::load_heads<4, NT>(dst, src, lds, S);
  }
  {  // D = rowsum(dO * O): TPR threads per row, 64 / TPR columns each
    const int r = threadIdx.x / TPR, part = threadIdx.x % TPR;
    float s = 0.f;
    if (r < S) {
      const unsigned short* orow = o + ((size_t)b * S + r) * Hd + h * D + part * (64 / TPR);
      const unsigned short* drow = dout + ((size_t)b * S + r) * Hd + h * D + part * (64 / TPR);
#pragma unroll
      for (int c = 0; c < CPT; ++c) {
        float ov[8], dv[8];
        unpack8(*(const bf16x8*)(orow + c * 8), ov);
        unpack8(*(const bf16x8*)(drow + c * 8), dv);
#pragma unroll
        for (int u = 0; u < 8; ++u) s += ov[u] * dv[u];
      }
    }
#pragma unroll
    for (int w = 1; w < TPR; w <<= 1) s += __shfl_xor(s, w);
    if (part == 0) Dr[r] = s;
  }
  __syncthreads();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int cl = lane & 15, rg = (lane >> 4) * 4;
  const float* L = lse + ((size_t)b * nh + h) * SP;
  float km[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int key = 16 * j + cl;
    km[j] = key < S ? (kmask ? kmask[(size_t)b * S + key] : 0.f) : -INFINITY;
  }
  // P and dS for this wave's 32 query rows
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int r0 = RPW * wave + 16 * i;
    f32x4 s[8], dp[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] = dp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 aq = lfrag<true>(Qs, LDQ, r0, 32 * kk, lane);
      const bf16x8 ado = lfrag<true>(dOs, LDQ, r0, 32 * kk, lane);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s[j] = mma(aq, lfrag<true>(Ks, LDQ, 16 * j, 32 * kk, lane), s[j]);
        dp[j] = mma(ado, lfrag<true>(Vs, LDQ, 16 * j, 32 * kk, lane), dp[j]);
      }
    }
    // P and dS are stored TRANSPOSED ([key][query]): a lane's 4 accumulator rows are 4
    // consecutive queries of one key, one 8-B store each (the row-major 2-B stores were a
    // quarter of the kernel's LDS instructions and most of its bank-conflict cycles)
    float lr[4], dr[4];
    bool live[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = r0 + rg + r;
      live[r] = row < S;
      lr[r] = live[r] ? L[row] : 0.f;
      dr[r] = Dr[row];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf16x4 p4, d4;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = live[r] ? __expf(s[j][r] * scale + km[j] - lr[r]) : 0.f;
        p4[r] = (short)tobf(p);
        d4[r] = (short)tobf(p * (dp[j][r] - dr[r]));
      }
      *(bf16x4*)(Ps + (16 * j + cl) * LDP + (r0 + rg) * 2) = p4;
      *(bf16x4*)(dSs + (16 * j + cl) * LDP + (r0 + rg) * 2) = d4;
    }
  }
  __syncthreads();
  unsigned short* dq = dqkv + (size_t)b * S * ld + h * D;
  unsigned short* dk = dq + Hd;
  unsigned short* dv = dq + 2 * Hd;
  // dV = P^T dO, dK = scale * dS^T Q  (this wave's 32 key rows), dQ = scale * dS K (query rows)
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int k0 = RPW * wave + 16 * i;
    f32x4 av[4], ak[4], aq[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) av[j] = ak[j] = aq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const bf16x8 pT = lfrag<true>(Ps, LDP, k0, 32 * kk, lane);    // (P^T, dS^T stored)
      const bf16x8 dsT = lfrag<true>(dSs, LDP, k0, 32 * kk, lane);
      const bf16x8 dsr = lfrag<false>(dSs, LDP, k0, 32 * kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        av[j] = mma(pT, lfrag<false>(dOs, LDQ, 16 * j, 32 * kk, lane), av[j]);
        ak[j] = mma(dsT, lfrag<false>(Qs, LDQ, 16 * j, 32 * kk, lane), ak[j]);
        aq[j] = mma(dsr, lfrag<false>(Ks, LDQ, 16 * j, 32 * kk, lane), aq[j]);
      }
    }
    // each 16 x 64 tile goes through this wave's rows of the V image (no longer read after
    // the barrier above) and leaves as 16-B chunks: 6 global stores per lane instead of 48
    // 2-byte stores
    char* stg = Vs + (size_t)k0 * LDQ;
    auto put = [&](const f32x4 (&acc)[4], float mul, unsigned short* dst) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *(unsigned short*)(stg + (rg + r) * LDQ + (16 * j + cl) * 2) = tobf(acc[j][r] * mul);
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int c = lane + 64 * u, row = k0 + (c >> 3), ch = c & 7;
        const bf16x8 v = *(const bf16x8*)(stg + (c >> 3) * LDQ + ch * 16);
        if (row < S) *(bf16x8*)(dst + (size_t)row * ld + ch * 8) = v;
      }
      __builtin_amdgcn_wave_barrier();  // read back before the next tile overwrites the rows
    };
    put(av, 1.f, dv);
    put(ak, scale, dk);
    put(aq, scale, dq);
    if (dbias) {  // fused qkv bias gradient: column sums over this wave's 16 rows
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float sq = 0.f, sk = 0.f, sv = 0.f;
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // rows >= S hold exact zeros (zero dO / masked P)
          sq += aq[j][r];
          sk += ak[j][r];
          sv += av[j][r];
        }
        sq += __shfl_xor(sq, 16);
        sq += __shfl_xor(sq, 32);
        sk += __shfl_xor(sk, 16);
        sk += __shfl_xor(sk, 32);
        sv += __shfl_xor(sv, 16);
        sv += __shfl_xor(sv, 32);
        if (lane < 16) {
          const int c = h * D + 16 * j + cl;
          unsafeAtomicAdd(dbias + c, sq * scale);
          unsafeAtomicAdd(dbias + Hd + c, sk * scale);
          unsafeAtomicAdd(dbias + 2 * Hd + c, sv);
        }
      }
    }
  }
}

// Persistent attention backward: one block per CU walks (sequence, head) pairs; the NEXT
// pair's Q, K, V, dO and O are loaded into registers while the current pair computes (the
// per-block form waited out its 80 KB of loads, then computed: ~14 us per pair at BERT-base
// seq 128 for ~1 us of MFMA work, one resident block per CU).  The same math and LDS layout as
// attn_bwd_kernel<8>; rowsum(dO * O) comes from the prefetched registers.
template <int NW>
__global__ __launch_bounds__(NW * 64, 1) void attn_bwd_persist_kernel(
    int S, int nh, int npairs, const unsigned short* __restrict__ qkv,
    const unsigned short* __restrict__ o, const unsigned short* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ kmask, float scale,
    unsigned short* __restrict__ dqkv, float* __restrict__ dbias) {
  using namespace at;
  constexpr int NT = NW * 64, RPW = SP / NW, NI = RPW / 16, PER = SP * 8 / NT;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  char* Qs = sm;
  char* Ks = sm + QB;
  char* Vs = sm + 2 * QB;
  char* dOs = sm + 3 * QB;
  char* Ps = sm + 4 * QB;
  char* dSs = Ps + PB;
  float* Dr = (float*)(dSs + PB);
  const int Hd = nh * D, ld = 3 * Hd;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int cl = lane & 15, rg = (lane >> 4) * 4;
  // prefetch registers: [tensor Q K V dO O][chunk k]; thread chunk i = tid + NT k: row i >> 3,
  // 16-B column chunk i & 7
  bf16x8 pf[5][PER];
  auto prefetch = [&](int pair) {
    const int b = pair / nh, h = pair % nh;
    const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
    const unsigned short* src[5] = {base, base + Hd, base + 2 * Hd,
                                    dout + (size_t)b * S * Hd + h * D, o + (size_t)b * S * Hd + h * D};
    const int lds_[5] = {ld, ld, ld, Hd, Hd};
#pragma unroll
    for (int n = 0; n < 5; ++n)
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x + NT * k, r = i >> 3, c = i & 7;
        pf[n][k] = *(const bf16x8*)(src[n] + (size_t)min(r, S - 1) * lds_[n] + c * 8);
      }
  };
  int pair = blockIdx.x;
  if (pair < npairs) prefetch(pair);
  for (; pair < npairs; pair += gridDim.x) {
    const int b = pair / nh, h = pair % nh;
    __syncthreads();  // the previous pair's LDS reads are done
    {
      char* const dst[4] = {Qs, Ks, Vs, dOs};
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int i = threadIdx.x + NT * k, r = i >> 3, c = i & 7;
        float dsum = 0.f;
        if (r < S) {
          float ov[8], dv[8];
          unpack8(pf[4][k], ov);
          unpack8(pf[3][k], dv);
#pragma unroll
          for (int u = 0; u < 8; ++u) dsum += ov[u] * dv[u];
        }
        // the 8 chunks of a row sit in 8 consecutive lanes
        dsum += __shfl_xor(dsum, 1);
        dsum += __shfl_xor(dsum, 2);
        dsum += __shfl_xor(dsum, 4);
        if (c == 0) Dr[r] = dsum;
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          bf16x8 v = pf[n][k];
          if (r >= S) v = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
          *(bf16x8*)(dst[n] + r * LDQ + c * 16) = v;
        }
      }
    }
    if (pair + (int)gridDim.x < npairs) prefetch(pair + gridDim.x);  // in flight below
    __syncthreads();
    const float* L = lse + ((size_t)b * nh + h) * SP;
    float km[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int key = 16 * j + cl;
      km[j] = key < S ? (kmask ? kmask[(size_t)b * S + key] : 0.f) : -INFINITY;
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int r0 = RPW * wave + 16 * i;
      f32x4 sacc[8], dp[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) sacc[j] = dp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 aq = lfrag<true>(Qs, LDQ, r0, 32 * kk, lane);
        const bf16x8 ado = lfrag<true>(dOs, LDQ, r0, 32 * kk, lane);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sacc[j] = mma(aq, lfrag<true>(Ks, LDQ, 16 * j, 32 * kk, lane), sacc[j]);
          dp[j] = mma(ado, lfrag<true>(Vs, LDQ, 16 * j, 32 * kk, lane), dp[j]);
        }
      }
      float lr[4], dr[4];
      bool live[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + rg + r;
        live[r] = row < S;
        lr[r] = live[r] ? L[row] : 0.f;
        dr[r] = Dr[row];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // P^T, dS^T: one 8-B store per key (see attn_bwd_kernel)
        bf16x4 p4, d4;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float pv = live[r] ? __expf(sacc[j][r] * scale + km[j] - lr[r]) : 0.f;
          p4[r] = (short)tobf(pv);
          d4[r] = (short)tobf(pv * (dp[j][r] - dr[r]));
        }
        *(bf16x4*)(Ps + (16 * j + cl) * LDP + (r0 + rg) * 2) = p4;
        *(bf16x4*)(dSs + (16 * j + cl) * LDP + (r0 + rg) * 2) = d4;
      }
    }
    __syncthreads();
    unsigned short* dq = dqkv + (size_t)b * S * ld + h * D;
    unsigned short* dk = dq + Hd;
    unsigned short* dv = dq + 2 * Hd;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int k0 = RPW * wave + 16 * i;
      f32x4 av[4], ak[4], aq[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) av[j] = ak[j] = aq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8 pT = lfrag<true>(Ps, LDP, k0, 32 * kk, lane);
        const bf16x8 dsT = lfrag<true>(dSs, LDP, k0, 32 * kk, lane);
        const bf16x8 dsr = lfrag<false>(dSs, LDP, k0, 32 * kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          av[j] = mma(pT, lfrag<false>(dOs, LDQ, 16 * j, 32 * kk, lane), av[j]);
          ak[j] = mma(dsT, lfrag<false>(Qs, LDQ, 16 * j, 32 * kk, lane), ak[j]);
          aq[j] = mma(dsr, lfrag<false>(Ks, LDQ, 16 * j, 32 * kk, lane), aq[j]);
        }
      }
      char* stg = Vs + (size_t)k0 * LDQ;  // this wave's V rows: consumed above
      auto put = [&](const f32x4 (&acc)[4], float mul, unsigned short* dst) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            *(unsigned short*)(stg + (rg + r) * LDQ + (16 * j + cl) * 2) = tobf(acc[j][r] * mul);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int c = lane + 64 * u, row = k0 + (c >> 3), ch = c & 7;
          const bf16x8 v = *(const bf16x8*)(stg + (c >> 3) * LDQ + ch * 16);
          if (row < S) *(bf16x8*)(dst + (size_t)row * ld + ch * 8) = v;
        }
        __builtin_amdgcn_wave_barrier();
      };
      put(av, 1.f, dv);
      put(ak, scale, dk);
      put(aq, scale, dq);
      if (dbias) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float sq = 0.f, sk = 0.f, sv = 0.f;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            sq += aq[j][r];
            sk += ak[j][r];
            sv += av[j][r];
          }
          sq += __shfl_xor(sq, 16);
          sq += __shfl_xor(sq, 32);
          sk += __shfl_xor(sk, 16);
          sk += __shfl_xor(sk, 32);
          sv += __shfl_xor(sv, 16);
          sv += __shfl_xor(sv, 32);
          if (lane < 16) {
            const int c = h * D + 16 * j + cl;
            unsafeAtomicAdd(dbias + c, sq * scale);
            unsafeAtomicAdd(dbias + Hd + c, sk * scale);
            unsafeAtomicAdd(dbias + 2 * Hd + c, sv);
          }
        }
      }
    }
  }
}

// Attention backward in two query halves: the same math as attn_bwd_kernel with 72 KB of LDS
// instead of 141 KB, so two blocks share a CU (the first version's single resident block
// left every global-load and barrier latency exposed: 69 us at BERT-base's seq 128 against
// ~13 us of MFMA work).  K stays in LDS for the block; per half of 64 queries Q_h, dO_h and
// P_h^T / dS_h^T (keys x queries) are staged, V's fragments are read from L2 (each wave needs
// only its 4 key tiles); dV / dK accumulate in registers over the halves, dQ_h is final per
// half.  P = exp(S * scale + mask - lse) needs no row maximum, so any tiling works.
namespace atb {
constexpr int HQ = 64;                  // queries per half
template <bool SWZ> constexpr int QH() { return HQ * at::img_pitch<SWZ>(); }      // 9216 / 8192 B
template <bool SWZ> constexpr int PT() { return at::SP * at::img_pitch<SWZ>(); }  // [128 keys][64 q]
template <bool SWZ> constexpr int KIMG() { return at::SP * at::img_pitch<SWZ>(); }
template <bool SWZ> constexpr int LDS() { return KIMG<SWZ>() + 2 * QH<SWZ>() + 2 * PT<SWZ>() + HQ * 4; }
}  // namespace atb

// SWZ (DTFX_ATTN_SWZ=1, opt-in): every image XOR-swizzled (at::swz): LDS bank-conflict cycles
// 56.2 M -> 8.7 M and LDS-wait cycles 134 M -> 24 M on the probe, but 58.7-62.4 -> 61.1-63.2
// us per call (profiles/r6/attn_swizzle/): the kernel is not LDS-bound.
// PF (DTFX_ATTN_BWD_PF=1, opt-in; measured slower, profiles/r6/attn_pf/: 63.3-65.9 vs
// 60.5-62.3 us per call, BERT-base 8,482-8,520 vs 8,494-8,529 seq/s interleaved): the block's
// V rows are requested at the block's start with
// the K rows, as LDS-destination loads into the not-yet-used P^T / dS^T images (the data is
// never read there: the point is that phase 1's per-key-tile V fragment loads, one exposed
// round trip per key tile and half, then hit this XCD's L2 instead of HBM).  It costs no VGPR:
// the kernel sits at its 128-VGPR budget (staging the log-sum-exp values in LDS as well, so
// phase 1 would issue no global load but V's, spilled 12 bytes per lane).
template <bool SWZ, bool PF = false>
__global__ __launch_bounds__(512, 4) void attn_bwd_half_kernel(
    int S, int nh, const unsigned short* __restrict__ qkv, const unsigned short* __restrict__ o,
    const unsigned short* __restrict__ dout, const float* __restrict__ lse,
    const float* __restrict__ kmask, float scale, unsigned short* __restrict__ dqkv,
    float* __restrict__ dbias) {
  using namespace at;
  using namespace atb;
  extern __shared__ __attribute__((aligned(16))) char sm[];
  constexpr int P_ = img_pitch<SWZ>();
  char* Ks = sm;
  char* Qh = Ks + KIMG<SWZ>();
  char* dOh = Qh + QH<SWZ>();
  char* PTs = dOh + QH<SWZ>();
  char* dSTs = PTs + PT<SWZ>();
  float* Dr = (float*)(dSTs + PT<SWZ>());
  const int b = blockIdx.x / nh, h = blockIdx.x % nh;
  const int Hd = nh * D, ld = 3 * Hd;
  const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
  const unsigned short* obase = o + (size_t)b * S * Hd + h * D;
  const unsigned short* dobase = dout + (size_t)b * S * Hd + h * D;
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int cl = lane & 15, g = lane >> 4, rg = g * 4;
  {  // K: 128 rows x 8 chunks, 2 per thread (rows >= S zero)
    bf16x8 kv[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + 512 * k, r = e >> 3, c = e & 7;
      kv[k] = *(const bf16x8*)(base + Hd + (size_t)min(r, S - 1) * ld + c * 8);
      if (r >= S) kv[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    if constexpr (PF) {  // V rows -> L2 (landing in the P^T image, overwritten in phase 1)
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int e = tid + 512 * k, r = e >> 3, c = e & 7;
        __builtin_amdgcn_global_load_lds(
            (const void*)(base + 2 * Hd + (size_t)min(r, S - 1) * ld + c * 8),
            (__attribute__((address_space(3))) void*)(PTs + (e - lane) * 16), 16, 0, 0);
      }
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int e = tid + 512 * k;
      *(bf16x8*)(Ks + img_off<SWZ>(e >> 3, (e & 7) * 8)) = kv[k];
    }
  }
  const float* L = lse + ((size_t)b * nh + h) * SP;
  const int qt = wave & 3, kt0 = (wave >> 2) * 4;  // phase 1: query tile, 4 key tiles
  f32x4 av[4], ak[4];  // dV / dK of key tile `wave`, 4 d tiles, over both halves
#pragma unroll
  for (int j = 0; j < 4; ++j) av[j] = ak[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned short* dq = dqkv + (size_t)b * S * ld + h * D;
  for (int q0 = 0; q0 < S; q0 += HQ) {
    {  // Q_h, dO_h (64 rows x 8 chunks: one each per thread) and D = rowsum(dO * O)
      const int r = tid >> 3, c = tid & 7, row = q0 + r, rr = min(row, S - 1);
      bf16x8 qv = *(const bf16x8*)(base + (size_t)rr * ld + c * 8);
      bf16x8 dv = *(const bf16x8*)(dobase + (size_t)rr * Hd + c * 8);
      const bf16x8 ov = *(const bf16x8*)(obase + (size_t)rr * Hd + c * 8);
      float f0[8], f1[8], d = 0.f;
      unpack8(ov, f0);
      unpack8(dv, f1);
#pragma unroll
      for (int u = 0; u < 8; ++u) d += f0[u] * f1[u];
      d += __shfl_xor(d, 1);
      d += __shfl_xor(d, 2);
      d += __shfl_xor(d, 4);
      if (row >= S) {
        qv = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
        dv = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
      }
      __syncthreads();  // the previous half's phase 2 is done with Q_h / dO_h / P^T / dS^T
      *(bf16x8*)(Qh + img_off<SWZ>(r, c * 8)) = qv;
      *(bf16x8*)(dOh + img_off<SWZ>(r, c * 8)) = dv;
      if (c == 0) Dr[r] = row < S ? d : 0.f;
      __syncthreads();
    }
    // phase 1: S and dP tiles (query tile qt x key tiles kt0..kt0+3) -> P^T, dS^T
    {
      bf16x8 aq[2], ado[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        aq[kk] = img_frag<SWZ, true>(Qh, 16 * qt, 32 * kk, lane);
        ado[kk] = img_frag<SWZ, true>(dOh, 16 * qt, 32 * kk, lane);
      }
      float lr[4], dr[4];
      bool live[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = 16 * qt + rg + r, row = q0 + ql;
        live[r] = row < S;
        lr[r] = live[r] ? L[row] : 0.f;
        dr[r] = Dr[ql];
      }
      // the lane's P^T / dS^T store offset within a key tile (swz(16 kt + cl) = swz(cl))
      const int poff = img_off<SWZ>(cl, 16 * qt + rg);
#pragma unroll 1
      for (int j = 0; j < 4; ++j) {
        const int kt = kt0 + j, key = 16 * kt + cl;
        const float kmj = key < S ? (kmask ? kmask[(size_t)b * S + key] : 0.f) : -INFINITY;
        f32x4 sa = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          bf16x8 vb = *(const bf16x8*)(base + 2 * Hd + (size_t)min(key, S - 1) * ld + 32 * kk + 8 * g);
          if (key >= S) vb = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
          sa = mma(aq[kk], img_frag<SWZ, true>(Ks, 16 * kt, 32 * kk, lane), sa);
          dp = mma(ado[kk], vb, dp);
        }
        bf16x4 pv, dsv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = live[r] ? __expf(sa[r] * scale + kmj - lr[r]) : 0.f;
          pv[r] = (short)tobf(p);
          dsv[r] = (short)tobf(p * (dp[r] - dr[r]));
        }
        const int off = kt * (16 * P_) + poff;  // = img_off(key, 16 qt + rg)
        *(bf16x4*)(PTs + off) = pv;
        *(bf16x4*)(dSTs + off) = dsv;
      }
    }
    __syncthreads();
    // phase 2: dV += P^T dO_h, dK += dS^T Q_h (key tile `wave`); dQ_h = dS K
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 pT = img_frag<SWZ, true>(PTs, 16 * wave, 32 * kk, lane);
      const bf16x8 dsT = img_frag<SWZ, true>(dSTs, 16 * wave, 32 * kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        av[j] = mma(pT, img_frag<SWZ, false>(dOh, 16 * j, 32 * kk, lane), av[j]);
        ak[j] = mma(dsT, img_frag<SWZ, false>(Qh, 16 * j, 32 * kk, lane), ak[j]);
      }
    }
    {
      const int dt0 = 2 * (wave >> 2);
      f32x4 aq[2];
      aq[0] = aq[1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const bf16x8 dsr = img_frag<SWZ, false>(dSTs, 16 * qt, 32 * kk, lane);
#pragma unroll
        for (int jj = 0; jj < 2; ++jj)
          aq[jj] = mma(dsr, img_frag<SWZ, false>(Ks, 16 * (dt0 + jj), 32 * kk, lane), aq[jj]);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = q0 + 16 * qt + rg + r;
        if (row < S)
#pragma unroll
          for (int jj = 0; jj < 2; ++jj)
            dq[(size_t)row * ld + 16 * (dt0 + jj) + cl] = tobf(aq[jj][r] * scale);
      }
      if (dbias) {
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          float sq = aq[jj][0] + aq[jj][1] + aq[jj][2] + aq[jj][3];
          sq += __shfl_xor(sq, 16);
          sq += __shfl_xor(sq, 32);
          if (lane < 16) unsafeAtomicAdd(dbias + h * D + 16 * (dt0 + jj) + cl, sq * scale);
        }
      }
    }
  }
  // dK, dV of key tile `wave`
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = 16 * wave + rg + r;
    if (row < S)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const size_t off = (size_t)row * ld + 16 * j + cl;
        dq[off + Hd] = tobf(ak[j][r] * scale);
        dq[off + 2 * Hd] = tobf(av[j][r]);
      }
  }
  if (dbias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float sk = ak[j][0] + ak[j][1] + ak[j][2] + ak[j][3];
      float sv = av[j][0] + av[j][1] + av[j][2] + av[j][3];
      sk += __shfl_xor(sk, 16);
      sk += __shfl_xor(sk, 32);
      sv += __shfl_xor(sv, 16);
      sv += __shfl_xor(sv, 32);
      if (lane < 16) {
        const int c = h * D + 16 * j + cl;
        unsafeAtomicAdd(dbias + Hd + c, sk * scale);
        unsafeAtomicAdd(dbias + 2 * Hd + c, sv);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Mixed-precision Adam(W): f32 master p, grad g, moments m, v; writes the bf16
// working copy pb used by the GEMMs.  Grad scale folds the 1/world average.  p, m, v are
// streamed (non-temporal: next read a whole step later), the bf16 copy is stored normally
// (BERT-base +1.0 % together with the GEMMs' non-temporal f32 / split-K stores,
// profiles/r5/gemm_nt/nt2/).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adam_mixed_kernel(
    long long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, unsigned short* __restrict__ pb, float lr, float b1, float b2,
    float eps, float wd, float gscale, const int* __restrict__ step_ptr, int step) {
  const int t = step_ptr ? *step_ptr : step;
  const float bc1 = 1.f - powf(b1, (float)t), bc2 = 1.f - powf(b2, (float)t);
  const float step_size = lr / bc1, rbc2 = rsqrtf(bc2);
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    f32x4 pv = ((f32x4*)p)[i], gv = ((const f32x4*)g)[i], mv = ((f32x4*)m)[i], vv = ((f32x4*)v)[i];
    bf16x4 o;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float gg = gv[u] * gscale;
      mv[u] = b1 * mv[u] + (1.f - b1) * gg;
      vv[u] = b2 * vv[u] + (1.f - b2) * gg * gg;
      pv[u] -= lr * wd * pv[u];
      pv[u] -= step_size * mv[u] / (sqrtf(vv[u]) * rbc2 + eps);
      o[u] = (short)tobf(pv[u]);
    }
    __builtin_nontemporal_store(pv, (f32x4*)p + i);
    __builtin_nontemporal_store(mv, (f32x4*)m + i);
    __builtin_nontemporal_store(vv, (f32x4*)v + i);
    if (pb) ((bf16x4*)pb)[i] = o;
  }
}

// The same AdamW with the weight gradients of some flat ranges ("segments") left as split-K
// partial planes by their GEMMs (gemm_bf16_launch defer_reduce): the split planes are summed
// here, in split order, instead of by a reduce pass that writes the gradient only for this
// kernel to read it back.  Used when nothing sits between the weight gradient and the
// optimizer (one GPU: no all-reduce).  Segment k (int64 x 5, sorted by start, disjoint):
// {lo4, hi4 (float4 indices into the flat buffer), partial planes (f32 pointer), plane
// stride in float4s, S}.  A lane finds its segment by binary search in LDS (<= 128 entries).
constexpr int kAdamMaxSegs = 128;
__global__ __launch_bounds__(256) void adam_mixed_segs_kernel(
    long long n, float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
    float* __restrict__ v, unsigned short* __restrict__ pb, float lr, float b1, float b2,
    float eps, float wd, float gscale, const int* __restrict__ step_ptr, int step,
    const long long* __restrict__ segs, int nseg, long long base4) {
  __shared__ long long s_lo[kAdamMaxSegs], s_hi[kAdamMaxSegs], s_pl[kAdamMaxSegs];
  __shared__ const f32x4* s_w[kAdamMaxSegs];
  __shared__ int s_S[kAdamMaxSegs];
  // segment bounds are absolute float4 indices of the whole flat buffer; this launch covers
  // [base4, base4 + n / 4) of it (a bucket's range)
  for (int k = threadIdx.x; k < nseg; k += blockDim.x) {
    s_lo[k] = segs[5 * k] - base4;
    s_hi[k] = segs[5 * k + 1] - base4;
    s_w[k] = (const f32x4*)segs[5 * k + 2];
    s_pl[k] = segs[5 * k + 3];
    s_S[k] = (int)segs[5 * k + 4];
  }
  __syncthreads();
  const int t = step_ptr ? *step_ptr : step;
  const float bc1 = 1.f - powf(b1, (float)t), bc2 = 1.f - powf(b2, (float)t);
  const float step_size = lr / bc1, rbc2 = rsqrtf(bc2);
  const long long n4 = n >> 2;
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    // last segment with lo <= i
    int lo = 0, hi = nseg - 1, k = -1;
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
      // the planes four at a time, loads first (a plain loop waited out one round trip per
      // plane: 14 for the attention-output weights), added in split order
      gv = __builtin_nontemporal_load(w);
      int q = 1;
      for (; q + 3 < S; q += 4) {
        const f32x4 a0 = __builtin_nontemporal_load(w + q * pl), a1 = __builtin_nontemporal_load(w + (q + 1) * pl),
                    a2 = __builtin_nontemporal_load(w + (q + 2) * pl), a3 = __builtin_nontemporal_load(w + (q + 3) * pl);
        gv += a0;
        gv += a1;
        gv += a2;
        gv += a3;
      }
      if (q + 1 < S) {
        const f32x4 a0 = __builtin_nontemporal_load(w + q * pl), a1 = __builtin_nontemporal_load(w + (q + 1) * pl);
        gv += a0;
        gv += a1;
        q += 2;
      }
      if (q < S) gv += __builtin_nontemporal_load(w + q * pl);
    } else {
      gv = __builtin_nontemporal_load((const f32x4*)g + i);
    }
    f32x4 pv = __builtin_nontemporal_load((f32x4*)p + i), mv = __builtin_nontemporal_load((f32x4*)m + i),
          vv = __builtin_nontemporal_load((f32x4*)v + i);
    bf16x4 o;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float gg = gv[u] * gscale;
      mv[u] = b1 * mv[u] + (1.f - b1) * gg;
      vv[u] = b2 * vv[u] + (1.f - b2) * gg * gg;
      pv[u] -= lr * wd * pv[u];
      pv[u] -= step_size * mv[u] / (sqrtf(vv[u]) * rbc2 + eps);
      o[u] = (short)tobf(pv[u]);
    }
    __builtin_nontemporal_store(pv, (f32x4*)p + i);
    __builtin_nontemporal_store(mv, (f32x4*)m + i);
    __builtin_nontemporal_store(vv, (f32x4*)v + i);
    if (pb) ((bf16x4*)pb)[i] = o;
  }
}

// ---------------------------------------------------------------------------
// MLM loss: softmax cross-entropy over a large vocabulary, one 256-thread block
// per row.  Pass 1: online (max, sum-exp) + argmax over float4 loads; pass 2:
// dlogits = (softmax - onehot) * scale written directly as bf16 (the operand of
// the decoder's dgrad/wgrad GEMMs).  Columns [C, ldd) of dlogits are zeroed.
// ---------------------------------------------------------------------------
// logits f32 (LT = float) or bf16 (LT = unsigned short: half the bytes of the [Tm x vocab] product
// written by the decoder GEMM and read here; the softmax math stays f32)
__device__ __forceinline__ float xl1(const float* l, int c) { return l[c]; }
__device__ __forceinline__ float xl1(const unsigned short* l, int c) { return bf(l[c]); }
__device__ __forceinline__ f32x4 xl4(const float* l, int i) { return ((const f32x4*)l)[i]; }
__device__ __forceinline__ f32x4 xl4(const unsigned short* l, int i) {
  const bf16x4 b = ((const bf16x4*)l)[i];
  return f32x4{bf((unsigned short)b[0]), bf((unsigned short)b[1]), bf((unsigned short)b[2]),
               bf((unsigned short)b[3])};
}
template <typename LT>
__global__ __launch_bounds__(256) void mlm_xent_kernel(int C, const LT* __restrict__ logits,
                                                       int ldl, const int* __restrict__ labels,
                                                       float scale, float* __restrict__ loss,
                                                       float* __restrict__ correct,
                                                       unsigned short* __restrict__ dl, int ldd) {
  __shared__ float sm_m[4], sm_s[4];
  __shared__ int sm_a[4];
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const LT* l = logits + (size_t)row * ldl;
  const int y = labels[row];
  float m = -INFINITY, sum = 0.f, best = -INFINITY;
  int am = 0x7fffffff;
  const int C4 = C >> 2;
  // U 16-B chunks in flight per thread; the running (max, sum) is rescaled once per pass
  // of U*4 values (branch-free inner loop) instead of per element
  constexpr int U = 4;
  for (int i0 = t; i0 < C4; i0 += 256 * U) {
    f32x4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) {
      const int i = i0 + 256 * k;
      v[k] = i < C4 ? xl4(l, i) : f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    }
    float lm = -INFINITY;
#pragma unroll
    for (int k = 0; k < U; ++k)
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float x = v[k][u];
        if (x > best) { best = x; am = 4 * (i0 + 256 * k) + u; }  // first index on ties
        lm = fmaxf(lm, x);
      }
    if (lm > m) {
      sum = m == -INFINITY ? 0.f : sum * __expf(m - lm);
      m = lm;
    }
    if (m != -INFINITY)
#pragma unroll
      for (int k = 0; k < U; ++k)
#pragma unroll
        for (int u = 0; u < 4; ++u) sum += __expf(v[k][u] - m);  // -inf pads add 0
  }
  for (int c = 4 * C4 + t; c < C; c += 256) {
    const float x = xl1(l, c);
    if (x > best) { best = x; am = c; }
    if (x > m) { sum = (m == -INFINITY ? 0.f : sum * __expf(m - x)) + 1.f; m = x; }
    else sum += __expf(x - m);
  }
  // wave reduce (max, sum) pairs and (best, argmax, lowest index on ties)
  for (int o = 32; o >= 1; o >>= 1) {
    const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(sum, o);
    const float mm = fmaxf(m, m2);
    sum = (m == -INFINITY ? 0.f : sum * __expf(m - mm)) + (m2 == -INFINITY ? 0.f : s2 * __expf(m2 - mm));
    m = mm;
    const float b2 = __shfl_xor(best, o);
    const int a2 = __shfl_xor(am, o);
    if (b2 > best || (b2 == best && a2 < am)) { best = b2; am = a2; }
  }
  if (lane == 0) { sm_m[wave] = m; sm_s[wave] = sum; sm_a[wave] = am; }
  __syncthreads();
  float M = sm_m[0], Ssum = 0.f;
  for (int w = 1; w < 4; ++w) M = fmaxf(M, sm_m[w]);
  for (int w = 0; w < 4; ++w) Ssum += sm_m[w] == -INFINITY ? 0.f : sm_s[w] * __expf(sm_m[w] - M);
  // argmax across waves: recompute best value by index order
  int A = sm_a[0];
  float Bv = xl1(l, A < C ? A : 0);
  for (int w = 1; w < 4; ++w) {
    const int a = sm_a[w];
    if (a < C) {
      const float bv = xl1(l, a);
      if (bv > Bv || (bv == Bv && a < A)) { Bv = bv; A = a; }
    }
  }
  const bool valid = y >= 0 && y < C;
  const float lse = M + __logf(Ssum);
  if (t == 0) {
    loss[row] = valid ? lse - xl1(l, y) : 0.f;
    correct[row] = (valid && A == y) ? 1.f : 0.f;
  }
  unsigned short* d = dl + (size_t)row * ldd;
  const float sc = valid ? scale : 0.f;
  for (int i = t; i < (ldd >> 2); i += 256) {
    const bool vec = 4 * i + 3 < C;  // (ldl % 4 == 0: the 16-B load is aligned)
    const f32x4 lv = vec ? xl4(l, i) : f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x4 o;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = 4 * i + u;
      float g = 0.f;
      if (c < C) g = (__expf((vec ? lv[u] : xl1(l, c)) - lse) - (c == y ? 1.f : 0.f)) * sc;
      o[u] = (short)tobf(g);
    }
    ((bf16x4*)d)[i] = o;
  }
}

// The bf16 form with the row held in registers (C <= 32768, rows 16-byte aligned): each thread
// loads its <= 16 chunks of 8 logits once as 16-byte loads (all in flight together), takes the
// max / argmax and then the sum of exponentials from the registers, and forms its dlogits
// chunks from the same registers -- one read of the row instead of two (the second one an L2
// or HBM re-read of 61 KB per row at the BERT vocabulary), 16-byte loads and stores.
constexpr int kXentChunks = 16;
__global__ __launch_bounds__(256) void mlm_xent_regs_kernel(int C, const unsigned short* __restrict__ logits,
                                                            int ldl, const int* __restrict__ labels,
                                                            float scale, float* __restrict__ loss,
                                                            float* __restrict__ correct,
                                                            unsigned short* __restrict__ dl, int ldd) {
  __shared__ float sm_m[4], sm_s[4], sm_b[4];
  __shared__ int sm_a[4];
  const int row = blockIdx.x, t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const unsigned short* l = logits + (size_t)row * ldl;
  const int y = labels[row];
  const int C8 = C >> 3;
  bf16x8 v[kXentChunks];
#pragma unroll
  for (int k = 0; k < kXentChunks; ++k) {
    const int i = t + 256 * k;
    if (i < C8) v[k] = __builtin_nontemporal_load((const bf16x8*)l + i);
  }
  // max and argmax (first index on ties: chunks in increasing index order per thread)
  float best = -INFINITY;
  int am = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < kXentChunks; ++k) {
    const int i = t + 256 * k;
    if (i < C8)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float x = bf((unsigned short)v[k][u]);
        if (x > best) { best = x; am = 8 * i + u; }
      }
  }
  for (int c = 8 * C8 + t; c < C; c += 256) {  // (C % 8 tail, one element per thread at most)
    const float x = bf(l[c]);
    if (x > best) { best = x; am = c; }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const float b2 = __shfl_xor(best, o);
    const int a2 = __shfl_xor(am, o);
    if (b2 > best || (b2 == best && a2 < am)) { best = b2; am = a2; }
  }
  if (lane == 0) { sm_b[wave] = best; sm_a[wave] = am; }
  __syncthreads();
  float M = sm_b[0];
  int A = sm_a[0];
  for (int w = 1; w < 4; ++w)
    if (sm_b[w] > M || (sm_b[w] == M && sm_a[w] < A)) { M = sm_b[w]; A = sm_a[w]; }
  // sum of exponentials against the row max (exact: no rescaling)
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < kXentChunks; ++k) {
    const int i = t + 256 * k;
    if (i < C8)
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += __expf(bf((unsigned short)v[k][u]) - M);
  }
  for (int c = 8 * C8 + t; c < C; c += 256) sum += __expf(bf(l[c]) - M);
  sum = wave_sum(sum);
  if (lane == 0) sm_s[wave] = sum;
  __syncthreads();
  const float Ssum = (sm_s[0] + sm_s[1]) + (sm_s[2] + sm_s[3]);
  const bool valid = y >= 0 && y < C;
  const float lse = M + __logf(Ssum);
  if (t == 0) {
    loss[row] = valid ? lse - bf(l[y]) : 0.f;
    correct[row] = (valid && A == y) ? 1.f : 0.f;
  }
  unsigned short* d = dl + (size_t)row * ldd;
  const float sc = valid ? scale : 0.f;
  const int D8 = ldd >> 3;
#pragma unroll
  for (int k = 0; k < kXentChunks; ++k) {
    const int i = t + 256 * k;
    if (i >= D8) break;
    bf16x8 o;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int c = 8 * i + u;
      float g = 0.f;
      if (i < C8) g = (__expf(bf((unsigned short)v[k][u]) - lse) - (c == y ? 1.f : 0.f)) * sc;
      else if (c < C) g = (__expf(bf(l[c]) - lse) - (c == y ? 1.f : 0.f)) * sc;
      o[u] = (short)tobf(g);
    }
    __builtin_nontemporal_store(o, (bf16x8*)d + i);
  }
}

// dx = dy * act'(u), bf16 (gelu-tanh: act 1, relu: act 2); n % 8 == 0
__global__ __launch_bounds__(256) void act_grad_bf16_kernel(long long n8, int act,
                                                            const unsigned short* __restrict__ dy,
                                                            const unsigned short* __restrict__ u,
                                                            unsigned short* __restrict__ dx) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    float a[8], b[8];
    unpack8(((const bf16x8*)dy)[i], a);
    unpack8(((const bf16x8*)u)[i], b);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float x = b[k];
      float d;
      if (act == 1) {
        const float k0 = 0.7978845608028654f, k1 = 0.044715f;
        const float th = tanhf(k0 * (x + k1 * x * x * x));
        d = 0.5f * (1.f + th) + 0.5f * x * (1.f - th * th) * k0 * (1.f + 3.f * k1 * x * x);
      } else {
        d = x > 0.f ? 1.f : 0.f;
      }
      a[k] *= d;
    }
    __builtin_nontemporal_store(pack8(a), (bf16x8*)dx + (i));
  }
}

__global__ __launch_bounds__(256) void cast_f32_bf16_kernel(long long n, const float* __restrict__ x,
                                                            unsigned short* __restrict__ y) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = tobf(x[i]);
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static void check_h(int H) {
  if (H % 8 || H > 2048) throw std::runtime_error("transformer: H must be a multiple of 8 and <= 2048");
}

void layernorm_fwd_launch(int T, int H, const void* x, const float* gamma, const float* beta,
                          float eps, void* y, float* mean, float* rstd, hipStream_t s) {
  check_h(H);
  if (T <= 0) return;
  // rows per wave (DTFX_LN_FWD_ROWS=1: the one-row kernel, for A/B runs)
  static const int rows = [] {
    const char* e = getenv("DTFX_LN_FWD_ROWS");
    return e ? atoi(e) : 4;
  }();
  const auto* xs = (const unsigned short*)x;
  auto* ys = (unsigned short*)y;
  const int nc = (H + 511) / 512;
  if ((rows == 4 || rows == 2) && !(((uintptr_t)gamma | (uintptr_t)beta) & 15)) {  // (f32x4 gamma / beta)
    const int per_block = 4 * rows;
    const dim3 grid((T + per_block - 1) / per_block);
#define DTFX_LNF(NC_, R_) \
  hipLaunchKernelGGL((layernorm_fwd_rows_kernel<NC_, R_>), grid, dim3(256), 0, s, T, H, xs, gamma, beta, eps, ys, mean, rstd)
    if (rows == 4) {
      if (nc == 1) DTFX_LNF(1, 4); else if (nc == 2) DTFX_LNF(2, 4); else if (nc == 3) DTFX_LNF(3, 4); else DTFX_LNF(4, 4);
    } else {
      if (nc == 1) DTFX_LNF(1, 2); else if (nc == 2) DTFX_LNF(2, 2); else if (nc == 3) DTFX_LNF(3, 2); else DTFX_LNF(4, 2);
    }
#undef DTFX_LNF
  } else {
    hipLaunchKernelGGL(layernorm_fwd_kernel, dim3((T + 3) / 4), dim3(256), 0, s, T, H, xs, gamma, beta, eps,
                       ys, mean, rstd);
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

static int g_ln_slots = -1;  // -1: DTFX_LN_SLOTS (tests set both forms)
void ln_bwd_set_slots(int v) { g_ln_slots = v; }
static int g_ln_h768 = -1;  // -1: DTFX_LN_H768
void ln_bwd_set_h768(int v) { g_ln_h768 = v; }

void layernorm_bwd_launch(int T, int H, const void* dy, const void* x, const float* mean,
                          const float* rstd, const float* gamma, const void* dres, void* dx,
                          float* dgamma, float* dbeta, float* dxsum, hipStream_t s) {
  check_h(H);
  if (T <= 0) return;
  // BERT 16384 rows: 256 blocks (measured 16: 54 us, 32: 35, 64: 31, 128: 38 -- atomics vs
  // parallelism; with two rows in flight per wave 32: 33.9, 64: 26.5, 128: 29.8 us).  DTFX_LN_RPB overrides (sweeps).
  static const int rpb_env = [] {
    const char* e = getenv("DTFX_LN_RPB");
    return e ? atoi(e) : 0;
  }();
  static const int slots_env = [] {
    const char* e = getenv("DTFX_LN_SLOTS");
    return e ? std::max(1, std::min(3, atoi(e))) : 2;
  }();
  // row slots per wave of the generic kernel: 2 (default) or 3
  const int slots = g_ln_slots >= 0 ? std::max(1, std::min(3, g_ln_slots)) : slots_env;
  static const int h768_env = [] {
    const char* e = getenv("DTFX_LN_H768");
    return e ? atoi(e) : 0;
  }();
  if (H == 768 && (g_ln_h768 >= 0 ? g_ln_h768 : h768_env) == 1 && !(((uintptr_t)gamma) & 15)) {
    // 4 rows per wave at the BERT shape (512 blocks, two per CU)
    const int rpb7 = rpb_env > 0 ? rpb_env : (T >= 8192 ? 32 : 8);
    // one row slot per wave: the 16 resident waves per CU are the pipeline (two slots spill
    // at the 128 VGPRs four waves per SIMD allow)
    hipLaunchKernelGGL(layernorm_bwd_h768_kernel<1>, dim3((T + rpb7 - 1) / rpb7), dim3(512), 0, s,
                         T, rpb7, (const unsigned short*)dy, (const unsigned short*)x, mean, rstd,
                         gamma, (const unsigned short*)dres, (unsigned short*)dx, dgamma, dbeta, dxsum);
    DTFX_HIP_CHECK(hipGetLastError());
    return;
  }
  const int rpb = rpb_env > 0 ? rpb_env : (T >= 8192 ? 64 : 16);
  const int nc = (H / 8 + 63) / 64;
#define DTFX_LNB(NC_, NS_)                                                                      \
  hipLaunchKernelGGL((layernorm_bwd_kernel<NC_, NS_>), dim3((T + rpb - 1) / rpb), dim3(NC_ <= 2 ? 512 : 256), 0, s, T, H, \
                     rpb, (const unsigned short*)dy, (const unsigned short*)x, mean, rstd, gamma,  \
                     (const unsigned short*)dres, (unsigned short*)dx, dgamma, dbeta, dxsum)
  if (nc == 1 && slots >= 3) DTFX_LNB(1, 3);
  else if (nc == 2 && slots >= 3) DTFX_LNB(2, 3);
  else if (nc == 1) DTFX_LNB(1, 2);
  else if (nc == 2) DTFX_LNB(2, 2);
  else if (nc == 3) DTFX_LNB(3, 2);
  else DTFX_LNB(4, 2);
#undef DTFX_LNB
  DTFX_HIP_CHECK(hipGetLastError());
}

void embed_ln_fwd_launch(int T, int S, int H, const int* ids, const int* tt, const void* word,
                         const void* pos, const void* type, const float* gamma, const float* beta,
                         float eps, void* xsum, void* y, float* mean, float* rstd, hipStream_t s) {
  check_h(H);
  if (T <= 0) return;
  hipLaunchKernelGGL(embed_ln_fwd_kernel, dim3((T + 3) / 4), dim3(256), 0, s, T, S, H, ids, tt,
                     (const unsigned short*)word, (const unsigned short*)pos,
                     (const unsigned short*)type, gamma, beta, eps, (unsigned short*)xsum,
                     (unsigned short*)y, mean, rstd);
  DTFX_HIP_CHECK(hipGetLastError());
}

void embed_bwd_launch(int Bn, int S, int H, const int* ids, const int* tt, const void* dx,
                      float* dword, float* dpos, float* dtype_, hipStream_t s) {
  check_h(H);
  const int T = Bn * S;
  if (T <= 0) return;
  hipLaunchKernelGGL(embed_word_bwd_kernel, dim3((T + 3) / 4), dim3(256), 0, s, T, H, ids,
                     (const unsigned short*)dx, dword);
  DTFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(embed_pos_type_bwd_kernel, dim3(S), dim3(1024), 0, s, Bn, S, H, tt,
                     (const unsigned short*)dx, dpos, dtype_);
  DTFX_HIP_CHECK(hipGetLastError());
}

static void check_attn(int S, int nh) {
  if (S <= 0 || S > at::SP) throw std::runtime_error("attention: fused kernel needs 0 < S <= 128");
  if (nh <= 0) throw std::runtime_error("attention: nh must be positive");
}

// Swizzled attention images (opt-in, measured slower: see attn_fwd_kernel): -1 = from the
// environment (DTFX_ATTN_SWZ=1), 0 / 1 forced (tests run both in one process).
static int g_attn_swz = -1;
void attn_set_swizzle(int v) { g_attn_swz = v; }
static bool attn_swz() {
  static const bool env = [] {
    const char* e = std::getenv("DTFX_ATTN_SWZ");
    return e && std::atoi(e) == 1;
  }();
  return g_attn_swz >= 0 ? g_attn_swz == 1 : env;
}

template <bool SWZ>
static void attn_fwd_launch_t(int Bn, int S, int nh, const void* qkv, void* out, float* lse,
                              const float* kmask, float scale, hipStream_t s) {
  const size_t lds = 2 * (size_t)at::SP * at::img_pitch<SWZ>() + at::PB;
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_kernel<SWZ>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL(attn_fwd_kernel<SWZ>, dim3(Bn * nh), dim3(256), lds, s, S, nh,
                     (const unsigned short*)qkv, (unsigned short*)out, lse, kmask, scale);
}

// Attention forward: -1 = from DTFX_ATTN_FWD (default 1), 1: attn_fwd_rp_kernel (P in
// registers), 0: attn_fwd_kernel (P through LDS; DTFX_ATTN_SWZ picks its swizzled variant)
static int g_attn_fwd = -1;
void attn_fwd_set_variant(int v) { g_attn_fwd = v; }
static bool attn_fwd_rp() {
  if (g_attn_fwd < 0) {
    const char* e = getenv("DTFX_ATTN_FWD");
    g_attn_fwd = e && atoi(e) == 0 ? 0 : 1;
  }
  return g_attn_fwd == 1;
}

void attn_fwd_launch(int Bn, int S, int nh, const void* qkv, void* out, float* lse,
                     const float* kmask, float scale, hipStream_t s) {
  check_attn(S, nh);
  if (attn_fwd_rp()) {
    constexpr size_t lds = 2 * (size_t)at::QB + (size_t)at::SP * 4;
    static bool attr = false;
    if (!attr) {
      DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)attn_fwd_rp_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      attr = true;
    }
    hipLaunchKernelGGL(attn_fwd_rp_kernel, dim3(Bn * nh), dim3(256), lds, s, S, nh,
                       (const unsigned short*)qkv, (unsigned short*)out, lse, kmask, scale);
  } else if (attn_swz()) {
    attn_fwd_launch_t<true>(Bn, S, nh, qkv, out, lse, kmask, scale, s);
  } else {
    attn_fwd_launch_t<false>(Bn, S, nh, qkv, out, lse, kmask, scale, s);
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

template <bool SWZ, bool PF>
static void attn_bwd_half_launch_t(int Bn, int S, int nh, const void* qkv, const void* o,
                                   const void* dout, const float* lse, const float* kmask,
                                   float scale, void* dqkv, float* dbias, hipStream_t s) {
  static bool hattr = false;
  if (!hattr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_half_kernel<SWZ, PF>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, atb::LDS<SWZ>()));
    hattr = true;
  }
  hipLaunchKernelGGL((attn_bwd_half_kernel<SWZ, PF>), dim3(Bn * nh), dim3(512), atb::LDS<SWZ>(), s,
                     S, nh, (const unsigned short*)qkv, (const unsigned short*)o,
                     (const unsigned short*)dout, lse, kmask, scale, (unsigned short*)dqkv, dbias);
}
static int g_attn_bwd_pf = -1;  // -1: DTFX_ATTN_BWD_PF (tests set both forms)
void attn_bwd_set_pf(int v) { g_attn_bwd_pf = v; }
static bool attn_bwd_pf() {
  static const bool env = [] {
    const char* e = std::getenv("DTFX_ATTN_BWD_PF");
    return e && std::atoi(e) == 1;
  }();
  return g_attn_bwd_pf >= 0 ? g_attn_bwd_pf == 1 : env;
}
template <bool SWZ>
static void attn_bwd_half_launch(int Bn, int S, int nh, const void* qkv, const void* o,
                                 const void* dout, const float* lse, const float* kmask,
                                 float scale, void* dqkv, float* dbias, hipStream_t s) {
  if (attn_bwd_pf())
    attn_bwd_half_launch_t<SWZ, true>(Bn, S, nh, qkv, o, dout, lse, kmask, scale, dqkv, dbias, s);
  else
    attn_bwd_half_launch_t<SWZ, false>(Bn, S, nh, qkv, o, dout, lse, kmask, scale, dqkv, dbias, s);
}

// Attention-backward kernel: -1 = from the environment, 0: attn_bwd_kernel<8>,
// 1: attn_bwd_kernel<4>, 2: attn_bwd_half_kernel, 3: attn_bwd_persist_kernel, 4: the same on a
// 3-block grid (tests run every variant in one process).
static int g_attn_bwd_variant = -1;
void attn_bwd_set_variant(int v) { g_attn_bwd_variant = v; }

void attn_bwd_launch(int Bn, int S, int nh, const void* qkv, const void* o, const void* dout,
                     const float* lse, const float* kmask, float scale, void* dqkv, float* dbias,
                     hipStream_t s) {
  check_attn(S, nh);
  const size_t lds = 4 * at::QB + 2 * at::PB + at::SP * 4;
  static bool attr = false;
  if (!attr) {
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_kernel<4>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_kernel<8>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  static const int nw = [] {
    const char* e = std::getenv("DTFX_ATTN_BWD_WAVES");
    return e && std::atoi(e) == 4 ? 4 : 8;
  }();
  // The two-blocks-per-CU kernel (default; DTFX_ATTN_BWD_HALF=0: the 8-wave one).  Alone it is
  // 14-18 % faster (BERT-base shape, batch 128: 56.9 vs 66.3 us).  Beside the weight-gradient
  // GEMMs of a second stream it lost that (round 3: 7892 vs 7924 seq/s); with the one-GPU BERT
  // step now issuing its weight gradients in order (train/bert_trainer.py) it gains: 7,903-7,919
  // -> 8,034-8,055 seq/s interleaved (profiles/r4/bert/half_nows/).
  static const bool half = [] {
    const char* e = std::getenv("DTFX_ATTN_BWD_HALF");
    return !(e && std::atoi(e) == 0);
  }();
  // DTFX_ATTN_BWD_PERSIST=1: the persistent kernel (grid: DTFX_ATTN_BWD_BLOCKS, default one
  // block per CU).  Measured slower: 84 us standalone vs 68 for the 8-wave per-pair kernel (128
  // blocks: 144 us), BERT 7,922-7,947 vs 7,960-8,003 seq/s (profiles/r4/bert/attn_persist/):
  // the pairs are not load-latency-bound but bound inside their compute phases (~11 us per
  // pair per CU against ~1 us of MFMA work), which one wave per SIMD hides worse.
  static const bool persist = [] {
    const char* e = std::getenv("DTFX_ATTN_BWD_PERSIST");
    return e && std::atoi(e) == 1;
  }();
  const int var = g_attn_bwd_variant >= 0 ? g_attn_bwd_variant : persist ? 3 : half ? 2 : nw == 4 ? 1 : 0;
  if (var == 3 || var == 4) {
    // 4 waves: one per SIMD with up to 512 registers each -- the 8-wave form's 40 prefetch
    // registers spilled
    static bool pattr = false;
    if (!pattr) {
      DTFX_HIP_CHECK(hipFuncSetAttribute((const void*)attn_bwd_persist_kernel<4>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      pattr = true;
    }
    static const int blocks = [] {
      const char* e = std::getenv("DTFX_ATTN_BWD_BLOCKS");
      return e && std::atoi(e) > 0 ? std::atoi(e) : 256;
    }();
    const int np = Bn * nh, nb = var == 4 ? 3 : blocks;  // 4: a 3-block grid (tests: many pairs per block)
    hipLaunchKernelGGL(attn_bwd_persist_kernel<4>, dim3(std::min(np, nb)), dim3(256), lds, s, S, nh,
                       np, (const unsigned short*)qkv, (const unsigned short*)o,
                       (const unsigned short*)dout, lse, kmask, scale, (unsigned short*)dqkv, dbias);
  } else if (var == 2) {
    if (attn_swz())
      attn_bwd_half_launch<true>(Bn, S, nh, qkv, o, dout, lse, kmask, scale, dqkv, dbias, s);
    else
      attn_bwd_half_launch<false>(Bn, S, nh, qkv, o, dout, lse, kmask, scale, dqkv, dbias, s);
  } else if (var == 1)
    hipLaunchKernelGGL(attn_bwd_kernel<4>, dim3(Bn * nh), dim3(256), lds, s, S, nh,
                       (const unsigned short*)qkv, (const unsigned short*)o,
                       (const unsigned short*)dout, lse, kmask, scale, (unsigned short*)dqkv,
                       dbias);
  else
    hipLaunchKernelGGL(attn_bwd_kernel<8>, dim3(Bn * nh), dim3(512), lds, s, S, nh,
                       (const unsigned short*)qkv, (const unsigned short*)o,
                       (const unsigned short*)dout, lse, kmask, scale, (unsigned short*)dqkv,
                       dbias);
  DTFX_HIP_CHECK(hipGetLastError());
}

void adam_mixed_launch(long long n, float* p, const float* g, float* m, float* v, void* pb,
                       float lr, float b1, float b2, float eps, float wd, float gscale,
                       const int* step_ptr, int step, hipStream_t s, const long long* segs,
                       int nseg, long long base4) {
  if (n % 4) throw std::runtime_error("adam_mixed: n must be a multiple of 4");
  if (n <= 0) return;
  if (nseg < 0 || nseg > kAdamMaxSegs || (nseg && !segs))
    throw std::runtime_error("adam_mixed: 0..128 segments with a table");
  long long blocks = (n / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (nseg) {
    hipLaunchKernelGGL(adam_mixed_segs_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n, p, g,
                       m, v, (unsigned short*)pb, lr, b1, b2, eps, wd, gscale, step_ptr, step,
                       segs, nseg, base4);
    DTFX_HIP_CHECK(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(adam_mixed_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n, p, g, m, v,
                     (unsigned short*)pb, lr, b1, b2, eps, wd, gscale, step_ptr, step);
  DTFX_HIP_CHECK(hipGetLastError());
}

static int g_xent_regs = -1;  // -1: DTFX_XENT_REGS (tests set both forms)
void xent_set_regs(int v) { g_xent_regs = v; }

void mlm_xent_launch(int N, int C, const void* logits, bool logits_bf16, int ldl, const int* labels,
                     float scale, float* loss, float* correct, void* dl, int ldd, hipStream_t s) {
  if (ldl % 4 || ldd % 4 || ldd < C || ldl < C)
    throw std::runtime_error("mlm_xent: ldl/ldd must be multiples of 4 and >= C");
  if (N <= 0) return;
  static const int regs_env = [] {
    const char* e = getenv("DTFX_XENT_REGS");
    return e ? atoi(e) : 1;
  }();
  const bool regs = (g_xent_regs >= 0 ? g_xent_regs : regs_env) == 1;
  if (logits_bf16 && regs && ldl % 8 == 0 && ldd % 8 == 0 && ldd <= 256 * 8 * kXentChunks &&
      !(((uintptr_t)logits | (uintptr_t)dl) & 15)) {
    hipLaunchKernelGGL(mlm_xent_regs_kernel, dim3(N), dim3(256), 0, s, C,
                       (const unsigned short*)logits, ldl, labels, scale, loss, correct,
                       (unsigned short*)dl, ldd);
    DTFX_HIP_CHECK(hipGetLastError());
    return;
  }
  if (logits_bf16)
    hipLaunchKernelGGL(mlm_xent_kernel<unsigned short>, dim3(N), dim3(256), 0, s, C,
                       (const unsigned short*)logits, ldl, labels, scale, loss, correct,
                       (unsigned short*)dl, ldd);
  else
    hipLaunchKernelGGL(mlm_xent_kernel<float>, dim3(N), dim3(256), 0, s, C, (const float*)logits, ldl,
                       labels, scale, loss, correct, (unsigned short*)dl, ldd);
  DTFX_HIP_CHECK(hipGetLastError());
}

void act_grad_bf16_launch(long long n, int act, const void* dy, const void* u, void* dx,
                          hipStream_t s) {
  if (n % 8) throw std::runtime_error("act_grad_bf16: n must be a multiple of 8");
  if (n <= 0) return;
  long long blocks = (n / 8 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(act_grad_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n / 8, act,
                     (const unsigned short*)dy, (const unsigned short*)u, (unsigned short*)dx);
  DTFX_HIP_CHECK(hipGetLastError());
}

// Zero many f32 ranges in one launch: table int64 [n][3] = {pointer, length, first element
// (prefix of the lengths)}, thread i -> range by binary search.  The per-step zeroing of the
// gradient slots the backward accumulates into (BERT: biases, LayerNorm parameters,
// embeddings -- a handful of strided fills of ~8 us each) becomes one launch.
__global__ __launch_bounds__(256) void zero_ranges_kernel(const long long* __restrict__ tab, int n,
                                                          long long total) {
  const long long stride = (long long)gridDim.x * blockDim.x;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    int lo = 0, hi = n - 1, k = 0;
    while (lo <= hi) {
      const int mid = (lo + hi) >> 1;
      if (tab[3 * mid + 2] <= i) {
        k = mid;
        lo = mid + 1;
      } else {
        hi = mid - 1;
      }
    }
    ((float*)tab[3 * k])[i - tab[3 * k + 2]] = 0.f;
  }
}
void zero_ranges_launch(const long long* tab, int n, long long total, hipStream_t s) {
  if (n <= 0 || total <= 0) return;
  long long blocks = (total + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(zero_ranges_kernel, dim3((unsigned)blocks), dim3(256), 0, s, tab, n, total);
  DTFX_HIP_CHECK(hipGetLastError());
}

void cast_f32_bf16_launch(long long n, const float* x, void* y, hipStream_t s) {
  if (n <= 0) return;
  long long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n, x,
                     (unsigned short*)y);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
