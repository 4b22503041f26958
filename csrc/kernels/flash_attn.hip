// Flash-style fused self-attention for sequences longer than one LDS-resident tile
// (BERT phase-2 seq 512, any S; head dim 64).  Complements attn_{fwd,bwd}_kernel in
// transformer.hip (S <= 128: the whole (sequence, head) in LDS).  Same layouts: reads
// the fused QKV activations [T][3 * nh * 64] in place, writes O [T][nh * 64] and
// dQKV in the QKV layout; lse is [B * nh][ld_lse] f32.
//
//   forward   grid (ceil(S/64), B*nh): 4 waves x 16 query rows; loop over 64-key
//             tiles of K/V in LDS; online softmax in registers (rows live in the
//             16-lane groups of the MFMA C layout: DPP row reductions); P goes
//             through a per-wave LDS tile to become the A operand of P.V.
//   backward  FA2 split in two kernels, no atomics on dQ:
//             dkdv: grid (key tiles, B*nh), 4 waves x 16 keys, loop over query tiles:
//                   S^T = K Q^T, P^T, dP^T = V dO^T, dS^T, dV += P^T dO, dK += dS^T Q
//             dq:   grid (query tiles, B*nh), 4 waves x 16 queries, loop over key tiles:
//                   S, P, dP = dO V^T, dS, dQ += dS K
//             D = rowsum(dO * O) comes from flash_rowdot (one pass).
// MFMA v_mfma_f32_16x16x32_bf16 throughout (operand fragments from LDS: ds_read_b128
// for k-contiguous images, ds_read_b64_tr_b16 for k-strided ones).
#include "common.h"

#include <stdexcept>

namespace dtfx {

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4 lds_b4;

namespace fa {
constexpr int D = 64, T = 64;           // head dim, tile rows
constexpr int LD = D * 2 + 16;          // 144-B LDS rows (16-B pad)
constexpr int TILE = T * LD;            // 9216 B

__device__ __forceinline__ float bf(unsigned short h) { return __uint_as_float((unsigned)h << 16); }
__device__ __forceinline__ unsigned short tobf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float rmax16(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false)));
  return v;
}
__device__ __forceinline__ float rsum16(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x124, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x128, 0xF, 0xF, false));
  return v;
}
// (tile, batch*head) of this block: the tiles of one (batch, head) share its K/V (forward,
// dq) or Q/dO (dkdv) stream, so they are given consecutive ids of ONE XCD (bijective XCD
// remap of the linear block id) instead of the dispatcher's round robin, which put the tiles
// of every (batch, head) on 8 different XCDs -- 8 L2s each fetching the same operands.
__device__ __forceinline__ void tile_bh(int& tile, int& bh) {
  const int nt = gridDim.x;
  const int id = xcd_remap(blockIdx.y * nt + blockIdx.x, nt * gridDim.y);
  tile = id % nt;
  bh = id / nt;
}
// operand fragment from an LDS image (see transformer.hip lfrag)
template <bool KC>
__device__ __forceinline__ bf16x8 frag(const char* base, int o0, int k0, int lane) {
  if (KC) return *(const bf16x8*)(base + (o0 + (lane & 15)) * LD + (k0 + 8 * (lane >> 4)) * 2);
  const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const char* a = base + (k0 + 8 * g + q) * LD + (o0 + 4 * p) * 2;
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4*)a);
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_b4*)(a + 4 * LD));
  bf16x8 v;
  v.lo = lo;
  v.hi = hi;
  return v;
}
__device__ __forceinline__ f32x4 mma(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// A-operand fragment (k-contiguous) straight from global: rows r0 + (lane & 15) (clamped)
__device__ __forceinline__ bf16x8 gfrag(const unsigned short* base, int ld, int r0, int rmax, int k0,
                                        int lane) {
  const int r = min(r0 + (lane & 15), rmax);
  return *(const bf16x8*)(base + (size_t)r * ld + k0 + 8 * (lane >> 4));
}
// Register-staged tile load, split in two so the NEXT tile's global loads are in flight
// while the current tile is computed (one LDS image, refilled between two barriers):
// fetch_tile issues this thread's two 16-B loads (rows >= S read as zero), put_tile
// writes them to the LDS image.
__device__ __forceinline__ void fetch_tile(bf16x8 (&v)[2], const unsigned short* src, int ld,
                                           int r0, int S) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + 256 * k, r = i >> 3, c = i & 7;
    const int row = r0 + r;
    v[k] = *(const bf16x8*)(src + (size_t)(row < S ? row : S - 1) * ld + c * 8);
    if (row >= S) v[k] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
  }
}
__device__ __forceinline__ void put_tile(char* dst, const bf16x8 (&v)[2]) {
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int i = threadIdx.x + 256 * k, r = i >> 3, c = i & 7;
    *(bf16x8*)(dst + r * LD + c * 16) = v[k];
  }
}
// C-layout (16 rows x 64 cols per wave: rows 4*(lane>>4)+r, col 16j+(lane&15)) -> bf16 LDS tile
__device__ __forceinline__ void put_c(char* dst, const f32x4 (&v)[4], int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *(unsigned short*)(dst + (4 * (lane >> 4) + r) * LD + (16 * j + (lane & 15)) * 2) = tobf(v[j][r]);
}
}  // namespace fa

using namespace fa;

__global__ __launch_bounds__(256) void flash_fwd_kernel(int S, int nh,
                                                        const unsigned short* __restrict__ qkv,
                                                        unsigned short* __restrict__ out,
                                                        float* __restrict__ lse, int ld_lse,
                                                        const float* __restrict__ kmask, float scale) {
  __shared__ __attribute__((aligned(16))) char Ks[TILE], Vs[TILE], Ps[4][16 * LD];
  int tile, bh;
  tile_bh(tile, bh);
  const int b = bh / nh, h = bh % nh;
  const int Hd = nh * D, ld = 3 * Hd;
  const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int q0 = tile * T + wave * 16;
  const int cl = lane & 15, rg = 4 * (lane >> 4);
  bf16x8 qa[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) qa[kk] = gfrag(base, ld, q0, S - 1, 32 * kk, lane);
  float m[4], l[4];
  f32x4 o[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) { m[r] = -INFINITY; l[r] = 0.f; }
#pragma unroll
  for (int j = 0; j < 4; ++j) o[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkt = (S + T - 1) / T;
  bf16x8 kr[2], vr[2];
  fetch_tile(kr, base + Hd, ld, 0, S);
  fetch_tile(vr, base + 2 * Hd, ld, 0, S);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    put_tile(Ks, kr);
    put_tile(Vs, vr);
    if (kt + 1 < nkt) {  // next key tile in flight during this tile's math
      fetch_tile(kr, base + Hd, ld, (kt + 1) * T, S);
      fetch_tile(vr, base + 2 * Hd, ld, (kt + 1) * T, S);
    }
    __syncthreads();
    f32x4 s[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) s[j] = mma(qa[kk], frag<true>(Ks, 16 * j, 32 * kk, lane), s[j]);
    float km[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = kt * T + 16 * j + cl;
      km[j] = key < S ? (kmask ? kmask[(size_t)b * S + key] : 0.f) : -INFINITY;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float mx = -INFINITY;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j][r] = s[j][r] * scale + km[j];
        mx = fmaxf(mx, s[j][r]);
      }
      mx = rmax16(mx);
      const float mn = fmaxf(m[r], mx);
      const float ms = mn == -INFINITY ? 0.f : mn;
      const float alpha = __expf(m[r] - ms);  // m = -inf -> 0
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j][r] = __expf(s[j][r] - ms);
        sum += s[j][r];
      }
      sum = rsum16(sum);
      l[r] = l[r] * alpha + sum;
      m[r] = mn;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j][r] *= alpha;
    }
    put_c(Ps[wave], s, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 pa = frag<true>(Ps[wave], 0, 32 * kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = mma(pa, frag<false>(Vs, 16 * j, 32 * kk, lane), o[j]);
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int row = q0 + rg + r;
    if (row >= S) continue;
    const float inv = l[r] > 0.f ? 1.f / l[r] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) out[((size_t)b * S + row) * Hd + h * D + 16 * j + cl] = tobf(o[j][r] * inv);
    if (cl == 0) lse[(size_t)bh * ld_lse + row] = (m[r] == -INFINITY ? 0.f : m[r]) + __logf(l[r]);
  }
}

// D[bh][row] = sum_d dO[row][h*64 + d] * O[row][h*64 + d]; one thread per (row, head)
__global__ __launch_bounds__(256) void flash_rowdot_kernel(int BS, int S, int nh,
                                                           const unsigned short* __restrict__ o,
                                                           const unsigned short* __restrict__ dout,
                                                           float* __restrict__ Dv, int ld_lse) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= BS * nh) return;
  const int row = i / nh, h = i % nh, b = row / S, s = row % S;
  const unsigned short* a = o + (size_t)row * nh * D + h * D;
  const unsigned short* c = dout + (size_t)row * nh * D + h * D;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < D / 8; ++k) {
    const bf16x8 x = ((const bf16x8*)a)[k], y = ((const bf16x8*)c)[k];
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += bf((unsigned short)x[u]) * bf((unsigned short)y[u]);
  }
  Dv[((size_t)b * nh + h) * ld_lse + s] = acc;
}

__global__ __launch_bounds__(256) void flash_dkdv_kernel(
    int S, int nh, const unsigned short* __restrict__ qkv, const unsigned short* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ Dv, int ld_lse,
    const float* __restrict__ kmask, float scale, unsigned short* __restrict__ dqkv,
    float* __restrict__ dbias) {
  __shared__ __attribute__((aligned(16))) char Qs[TILE], dOs[TILE], PT[4][16 * LD], DT[4][16 * LD];
  __shared__ float Ls[T], Ds[T];
  int tile, bh;
  tile_bh(tile, bh);
  const int b = bh / nh, h = bh % nh;
  const int Hd = nh * D, ld = 3 * Hd;
  const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
  const unsigned short* dob = dout + (size_t)b * S * Hd + h * D;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int k0 = tile * T + wave * 16;
  const int cl = lane & 15, rg = 4 * (lane >> 4);
  bf16x8 ka[2], va[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    ka[kk] = gfrag(base + Hd, ld, k0, S - 1, 32 * kk, lane);
    va[kk] = gfrag(base + 2 * Hd, ld, k0, S - 1, 32 * kk, lane);
  }
  float km[4];  // this lane's keys are C-layout rows k0 + rg + r
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = k0 + rg + r;
    km[r] = key < S ? (kmask ? kmask[(size_t)b * S + key] : 0.f) : -INFINITY;
  }
  f32x4 dv[4], dk[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dv[j] = dk[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nqt = (S + T - 1) / T;
  bf16x8 qr[2], dr[2];
  float lv = 0.f, dvv = 0.f;
  auto fetch = [&](int qt) {
    fetch_tile(qr, base, ld, qt * T, S);
    fetch_tile(dr, dob, Hd, qt * T, S);
    if (threadIdx.x < T) {
      const int q = qt * T + threadIdx.x;
      lv = q < S ? lse[(size_t)bh * ld_lse + q] : INFINITY;  // P = 0 past S
      dvv = q < S ? Dv[(size_t)bh * ld_lse + q] : 0.f;
    }
  };
  fetch(0);
  for (int qt = 0; qt < nqt; ++qt) {
    __syncthreads();
    put_tile(Qs, qr);
    put_tile(dOs, dr);
    if (threadIdx.x < T) {
      Ls[threadIdx.x] = lv;
      Ds[threadIdx.x] = dvv;
    }
    if (qt + 1 < nqt) fetch(qt + 1);  // next query tile in flight during this tile's math
    __syncthreads();
    f32x4 st[4], dpt[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = dpt[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        st[j] = mma(ka[kk], frag<true>(Qs, 16 * j, 32 * kk, lane), st[j]);
        dpt[j] = mma(va[kk], frag<true>(dOs, 16 * j, 32 * kk, lane), dpt[j]);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float lq = Ls[16 * j + cl], dq = Ds[16 * j + cl];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(st[j][r] * scale + km[r] - lq);
        st[j][r] = p;
        dpt[j][r] = p * (dpt[j][r] - dq);
      }
    }
    put_c(PT[wave], st, lane);
    put_c(DT[wave], dpt, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 pa = frag<true>(PT[wave], 0, 32 * kk, lane);
      const bf16x8 da = frag<true>(DT[wave], 0, 32 * kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dv[j] = mma(pa, frag<false>(dOs, 16 * j, 32 * kk, lane), dv[j]);
        dk[j] = mma(da, frag<false>(Qs, 16 * j, 32 * kk, lane), dk[j]);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  unsigned short* dkp = dqkv + (size_t)b * S * ld + Hd + h * D;
  unsigned short* dvp = dkp + Hd;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int key = k0 + rg + r;
    if (key >= S) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dkp[(size_t)key * ld + 16 * j + cl] = tobf(dk[j][r] * scale);
      dvp[(size_t)key * ld + 16 * j + cl] = tobf(dv[j][r]);
    }
  }
  if (dbias) {  // column sums over this wave's 16 keys (rows past S hold zeros)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float sk = dk[j][0] + dk[j][1] + dk[j][2] + dk[j][3];
      float sv = dv[j][0] + dv[j][1] + dv[j][2] + dv[j][3];
      sk += __shfl_xor(sk, 16);
      sk += __shfl_xor(sk, 32);
      sv += __shfl_xor(sv, 16);
      sv += __shfl_xor(sv, 32);
      if (lane < 16) {
        unsafeAtomicAdd(dbias + Hd + h * D + 16 * j + cl, sk * scale);
        unsafeAtomicAdd(dbias + 2 * Hd + h * D + 16 * j + cl, sv);
      }
    }
  }
}

__global__ __launch_bounds__(256) void flash_dq_kernel(
    int S, int nh, const unsigned short* __restrict__ qkv, const unsigned short* __restrict__ dout,
    const float* __restrict__ lse, const float* __restrict__ Dv, int ld_lse,
    const float* __restrict__ kmask, float scale, unsigned short* __restrict__ dqkv,
    float* __restrict__ dbias) {
  __shared__ __attribute__((aligned(16))) char Ks[TILE], Vs[TILE], DS[4][16 * LD];
  int tile, bh;
  tile_bh(tile, bh);
  const int b = bh / nh, h = bh % nh;
  const int Hd = nh * D, ld = 3 * Hd;
  const unsigned short* base = qkv + (size_t)b * S * ld + h * D;
  const unsigned short* dob = dout + (size_t)b * S * Hd + h * D;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int q0 = tile * T + wave * 16;
  const int cl = lane & 15, rg = 4 * (lane >> 4);
  bf16x8 qa[2], oa[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    qa[kk] = gfrag(base, ld, q0, S - 1, 32 * kk, lane);
    oa[kk] = gfrag(dob, Hd, q0, S - 1, 32 * kk, lane);
  }
  float lr[4], dr[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + rg + r;
    lr[r] = q < S ? lse[(size_t)bh * ld_lse + q] : INFINITY;
    dr[r] = q < S ? Dv[(size_t)bh * ld_lse + q] : 0.f;
  }
  f32x4 dq[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) dq[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkt = (S + T - 1) / T;
  bf16x8 kr[2], vr[2];
  fetch_tile(kr, base + Hd, ld, 0, S);
  fetch_tile(vr, base + 2 * Hd, ld, 0, S);
  for (int kt = 0; kt < nkt; ++kt) {
    __syncthreads();
    put_tile(Ks, kr);
    put_tile(Vs, vr);
    if (kt + 1 < nkt) {  // next key tile in flight during this tile's math
      fetch_tile(kr, base + Hd, ld, (kt + 1) * T, S);
      fetch_tile(vr, base + 2 * Hd, ld, (kt + 1) * T, S);
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) s[j] = dp[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        s[j] = mma(qa[kk], frag<true>(Ks, 16 * j, 32 * kk, lane), s[j]);
        dp[j] = mma(oa[kk], frag<true>(Vs, 16 * j, 32 * kk, lane), dp[j]);
      }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int key = kt * T + 16 * j + cl;
      const float km = key < S ? (kmask ? kmask[(size_t)b * S + key] : 0.f) : -INFINITY;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = __expf(s[j][r] * scale + km - lr[r]);
        s[j][r] = p * (dp[j][r] - dr[r]);
      }
    }
    put_c(DS[wave], s, lane);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 da = frag<true>(DS[wave], 0, 32 * kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) dq[j] = mma(da, frag<false>(Ks, 16 * j, 32 * kk, lane), dq[j]);
    }
    __builtin_amdgcn_wave_barrier();
  }
  unsigned short* dqp = dqkv + (size_t)b * S * ld + h * D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + rg + r;
    if (q >= S) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) dqp[(size_t)q * ld + 16 * j + cl] = tobf(dq[j][r] * scale);
  }
  if (dbias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float sq = dq[j][0] + dq[j][1] + dq[j][2] + dq[j][3];
      sq += __shfl_xor(sq, 16);
      sq += __shfl_xor(sq, 32);
      if (lane < 16) unsafeAtomicAdd(dbias + h * D + 16 * j + cl, sq * scale);
    }
  }
}

void flash_fwd_launch(int Bn, int S, int nh, const void* qkv, void* out, float* lse, int ld_lse,
                      const float* kmask, float scale, hipStream_t st) {
  if (S <= 0 || ld_lse < (S + T - 1) / T * T) throw std::runtime_error("flash_fwd: bad S / ld_lse");
  hipLaunchKernelGGL(flash_fwd_kernel, dim3((S + T - 1) / T, Bn * nh), dim3(256), 0, st, S, nh,
                     (const unsigned short*)qkv, (unsigned short*)out, lse, ld_lse, kmask, scale);
  DTFX_HIP_CHECK(hipGetLastError());
}

// scratch_D: f32 [Bn * nh][ld_lse]
void flash_bwd_launch(int Bn, int S, int nh, const void* qkv, const void* o, const void* dout,
                      const float* lse, int ld_lse, const float* kmask, float scale, void* dqkv,
                      float* dbias, float* scratch_D, hipStream_t st) {
  if (S <= 0 || ld_lse < (S + T - 1) / T * T) throw std::runtime_error("flash_bwd: bad S / ld_lse");
  const int BS = Bn * S;
  hipLaunchKernelGGL(flash_rowdot_kernel, dim3((BS * nh + 255) / 256), dim3(256), 0, st, BS, S, nh,
                     (const unsigned short*)o, (const unsigned short*)dout, scratch_D, ld_lse);
  DTFX_HIP_CHECK(hipGetLastError());
  const dim3 grid((S + T - 1) / T, Bn * nh);
  hipLaunchKernelGGL(flash_dkdv_kernel, grid, dim3(256), 0, st, S, nh, (const unsigned short*)qkv,
                     (const unsigned short*)dout, lse, scratch_D, ld_lse, kmask, scale,
                     (unsigned short*)dqkv, dbias);
  DTFX_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(flash_dq_kernel, grid, dim3(256), 0, st, S, nh, (const unsigned short*)qkv,
                     (const unsigned short*)dout, lse, scratch_D, ld_lse, kmask, scale,
                     (unsigned short*)dqkv, dbias);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
