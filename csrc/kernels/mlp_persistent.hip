// Persistent MNIST-MLP trainer: K complete SGD steps (784 -> 100 sigmoid -> 10, softmax
// cross-entropy; reference graph worker.py:46-79, hot loop worker.py:129-159) in ONE launch.
//
// Why: the two-launch pipelined step (mlp_step.hip) runs at ~8.2 us per step and rocprof puts
// ~4-5 us on EACH launch although each does < 0.3 us of MFMA work: the step is a chain of two
// dependent kernel boundaries plus the cold load ramp after each.  Here the same two phases
// run inside one grid that lives for all K steps and hands data from workgroup to workgroup
// as data-tagged granules: one naturally aligned 8-byte word {f32 value, u32 epoch} written by
// ONE agent-scope store (sc1) and polled with agent-scope loads until the epoch matches.  No
// grid barrier, no fence, no flag: a consumer waits exactly for the words it reads.
//
// Grid (105 + B workgroups x 256 threads, all co-resident: 1 per CU needed of 256 CUs):
//   blocks [0, 98): W1 block (jt, ks) OWNS W1t[jt*16 .. +16][ks*56 .. +56] for the whole
//     launch: the tile lives in LDS (+ each lane's 4 master values in registers); the W1
//     gradient is never materialised and W1 never leaves the block until the final store.
//     step t:  (t > 0) wait for dz1 of step t-1 (rows x this block's 16 hidden units) ->
//              LDS; dW1^T tile = dz1^T . x(t-1) (f32 MFMA, K = batch); W1 -= lr * g;
//              z1 partial of every row over the block's 56 features -> SLAB granules.
//   blocks [98, 105): small block jt owns W2t[:, jt*16 .. +16], b1[jt*16 .. +16] (and b2,
//     the loss/accuracy record and global_step for jt == 0) in registers; step t:
//              (t > 0) dW2 / db1 / db2 of step t-1 from the HEAD granules of every row
//              (batch split over the 4 waves), update, publish the new values as SP
//              granules (epoch of step t).
//   blocks [105, 105 + B): head of batch row bid - 105 (4 waves): waits for its row's 14
//     SLAB partials and the SP granules, z1 -> h -> logits -> softmax / xent / argmax ->
//     dlogits -> dz1; publishes {dz1, h, dlogits, (loss, correct)} as HEAD granules.
//   Heads have workgroups of their own because a wave's load cannot be consumed before
//   every OLDER store of that wave is acknowledged (gfx9 counts loads and stores in one
//   vmcnt): a W1 wave that published its slab and then ran a head stalled ~2 us on its own
//   write-through stores before it could use the head's data (trace probe).
//
// Epochs: step t of a launch tags its words with ebase + 1 + t (the host advances ebase by
// steps + 1 per launch, so a stale word from any earlier launch never matches).  Two parity
// planes per buffer: a plane is rewritten two steps later, and every writer of step t + 2
// has waited (transitively) for every reader of step t to finish.
//
// Failure: every wait is bounded (`ticks` of s_memrealtime, 100 MHz) and also polls a sticky
// error word; a wave that times out sets it, every other waiter then gives up within a few
// polls, W1 blocks leave the step loop together (LDS flag read after a barrier), and the
// host raises (FusedMLPTrainer.check()).  The grid always drains.
//
// Numerics: the same MFMA orderings and summation orders as mlp_fwdapply_kernel /
// mlp_head_kernel<.., KS2> / wgrad_small; results match the pipelined two-launch step to f32
// rounding (the compiler may contract a different product of a short dot into an FMA;
// tests/test_kernels_gpu.py::test_persistent_trainer_*).
#include "common.h"

#include <stdexcept>

namespace dtfx {
namespace mlpp {

using u64 = unsigned long long;

constexpr int D = 784, H = 100, C = 10;
constexpr int HT = 7;             // hidden tiles of 16 (112 padded)
constexpr int KS = 14, KW = 56;   // feature slices of a hidden tile (3.5 MFMA groups of 16)
constexpr int NW1 = HT * KS;      // 98 W1 blocks
constexpr int NBLK = NW1 + HT;    // + 7 small-parameter blocks = 105
constexpr int MAXB = 128;
constexpr int OFF_W1 = 0, OFF_B1 = H * D, OFF_W2 = OFF_B1 + H, OFF_B2 = OFF_W2 + C * H;
constexpr int NPARAM = OFF_B2 + C;

// granule buffer layout (u64 words)
constexpr int SLAB_ROW = 128;                                 // words per (ks, row): j < 100
constexpr long long SLAB_PAR = (long long)KS * MAXB * SLAB_ROW;
constexpr int HEAD_ROW = 256;                                 // per row: dz1 | h | dl | stat
constexpr int HDZ = 0, HHB = 128, HDL = 232, HST = 248;
constexpr long long HEAD_PAR = (long long)MAXB * HEAD_ROW;
constexpr int SP_REP = 1152;                                  // b1 [0,100) W2t [100,1100) b2
constexpr int SP_W2 = 100, SP_B2 = 1100;
// Every head reads ALL small parameters; with one copy a hundred waves' agent-scope loads of
// the same 9 KB queued on the few memory channels holding it (trace probe: 3.7 us from the
// last publish to the heads' data), so the small blocks publish NREP copies and head row b
// reads copy b % NREP.
constexpr int NREP = 8;
constexpr int SP_PAR = NREP * SP_REP;
constexpr long long OFF_SLAB = 0;
constexpr long long OFF_HEAD = OFF_SLAB + 2 * SLAB_PAR;
constexpr long long OFF_SP = OFF_HEAD + 2 * HEAD_PAR;
constexpr long long OFF_ERR = OFF_SP + 2 * SP_PAR;
constexpr long long LL_WORDS = OFF_ERR + 32;
constexpr int TRACE_STEPS = 64;

static_assert(NPARAM == 79510, "parameter count of worker.py:50-53");
static_assert(KS * KW == D && HDL + 16 <= HST && HST + 2 <= HEAD_ROW, "layout");

struct Args {
  float* p;                 // flat parameters, updated in place (read at start, written at end)
  const float* x;           // dataset [nbatches * B][784]
  const int* labels;        // [nbatches * B]
  u64* ll;                  // granule buffer (LL_WORDS, zero-initialised once)
  int* ctr;                 // global_step
  float* stats;             // [ring][2] loss / accuracy per step
  long long ticks;          // wait bound (s_memrealtime ticks)
  u64* trace;               // optional [NBLK][TRACE_STEPS][12] s_memrealtime stamps (probe)
  float lr;
  unsigned ebase;
  int nbatches, pos0, steps, B, ring;
};

__device__ __forceinline__ void st_ll(u64* p, float v, unsigned e) {
  __hip_atomic_store(p, ((u64)e << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u64 ld_ll(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Workgroup barrier for LDS hand-offs only.  __syncthreads() also waits for every vector
// memory op in flight (s_waitcnt vmcnt(0)): after a phase that published granules with
// write-through stores it stalled ~2 us until they were acknowledged (trace probe), which no
// consumer here needs -- cross-workgroup data is tagged, cross-wave data goes through LDS.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// probe stamp k of (block, step t) by lane 0 of the calling wave
__device__ __forceinline__ void stamp(const Args& a, int t, int k) {
  if (a.trace != nullptr && t < TRACE_STEPS && (threadIdx.x & 63) == 0)
    a.trace[((size_t)blockIdx.x * TRACE_STEPS + t) * 12 + k] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ float4 f4(const float* p) {
  return *reinterpret_cast<const float4*>(p);
}

// Waits until every word addr(i) (nullptr = absent: value 0) carries epoch e: every word is
// loaded together and only stale ones are re-polled (polling one representative word first
// measured slower: it adds a round trip once the data lands, profiles/r2/persistent/).  On
// timeout or a raised error word, sets `fail` (and the error word) and returns zeros.
template <int N, class Addr>
__device__ __forceinline__ void ll_wait(Addr addr, unsigned e, const Args& a, float (&out)[N],
                                        bool& fail) {
  u64 w[N];
  const u64 ready_word = (u64)e << 32;
  long long t0 = -1;
  auto expired = [&](int it) {
    if ((it & 15) != 0) return false;
    const long long now = (long long)__builtin_amdgcn_s_memrealtime();
    if (t0 < 0) t0 = now;
    if (ld_ll(a.ll + OFF_ERR) != 0 || now - t0 > a.ticks) {
      fail = true;
      __hip_atomic_store(a.ll + OFF_ERR, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    return false;
  };
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const u64* p = addr(i);
    w[i] = p && !fail ? ld_ll(p) : ready_word;
  }
  if (!fail) {
    for (int it = 1;; ++it) {
      bool ready = true;
#pragma unroll
      for (int i = 0; i < N; ++i)
        if ((unsigned)(w[i] >> 32) != e) {
          ready = false;
          w[i] = ld_ll(addr(i));
        }
      if (ready) break;
      if (expired(it)) break;
      __builtin_amdgcn_s_sleep(1);
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i) out[i] = fail ? 0.f : __uint_as_float((unsigned)w[i]);
}

// ---------------------------------------------------------------------------------------
// head of batch row `row`, step t, by the 4 waves of a workgroup (mlp_head_kernel math):
// wave w owns hidden units j = 25w + (lane & 31) (lanes with lane & 31 >= 25 idle); half
// h2 = lane >> 5 sums slab planes ks = 7 h2 .. 7 h2 + 6 and holds W2t rows c = 5 h2 .. +4.
// A one-wave head had to pull 60 granule words per lane (30 KB per wave: ~5 us of agent-scope
// loads); split four ways a wave pulls 23.  The 10 partial logits of each wave meet in LDS
// (red, double-buffered by step parity).  Called by every wave of the block (barrier inside).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ float swap32_add(float v) {  // v + v of lane ^ 32
  const int x = __float_as_int(v);
  auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}

__device__ __forceinline__ void head_row(const Args& a, int row, int t, int wave, int lane,
                                         float (*red)[16], bool& fail) {
  const unsigned e = a.ebase + 1u + (unsigned)t;
  const int bidx = (a.pos0 + t) % a.nbatches;
  const int y = a.labels[(size_t)bidx * a.B + row];
  const int h2 = lane >> 5, jl = lane & 31;
  const bool jv = jl < 25;
  const int j = 25 * wave + (jv ? jl : 0);
  const u64* slab = a.ll + OFF_SLAB + (e & 1) * SLAB_PAR + (size_t)row * SLAB_ROW + j;
  const u64* sp = a.ll + OFF_SP + (e & 1) * SP_PAR + (row % NREP) * SP_REP;
  // words: [0, 7) slab[7 h2 + k][j], [7, 12) W2t[5 h2 + k][j], [12] b1[j], [13, 23) b2[c]
  if (wave == 3) stamp(a, t, 5);
  float v[23];
  ll_wait<23>(
      [&](int i) -> const u64* {
        if (i < 7) return jv ? slab + (size_t)(7 * h2 + i) * MAXB * SLAB_ROW : nullptr;
        if (i < 12) return jv ? sp + SP_W2 + (5 * h2 + i - 7) * H + j : nullptr;
        if (i == 12) return jv ? sp + j : nullptr;
        return sp + SP_B2 + (i - 13);
      },
      e, a, v, fail);
  stamp(a, t, wave == 3 ? 6 : 8 + wave);
  float zp = 0.f;
#pragma unroll
  for (int k = 0; k < 7; ++k) zp += v[k];
  const float z = swap32_add(zp);  // planes 0..6 + planes 7..13
  const float hv = jv ? sigmoidf_(z + v[12]) : 0.f;
  float lg[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const bool mine = (c >= 5 * h2) && (c < 5 * h2 + 5);
    const float w2 = v[7 + (c - 5 * h2 >= 0 && c - 5 * h2 < 5 ? c - 5 * h2 : 0)];
    lg[c] = mine ? hv * w2 : 0.f;
  }
  wave_sum_n(lg);
  float* rw = red[(t & 1) * 4 + wave];
  float mine_l = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) mine_l = lane == c ? lg[c] : mine_l;
  if (lane < C) rw[lane] = mine_l;
  lds_barrier();
  if (wave == 3) stamp(a, t, 11);
  const float (*rr)[16] = red + (t & 1) * 4;
#pragma unroll
  for (int c = 0; c < C; ++c) lg[c] = ((rr[0][c] + rr[1][c]) + (rr[2][c] + rr[3][c])) + v[13 + c];
  float m = lg[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < C; ++c)
    if (lg[c] > m) { m = lg[c]; am = c; }  // first max, like tf.argmax
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) se += __expf(lg[c] - m);
  const float inv = fast_rcp(se), invB = 1.f / (float)a.B;
  float dl[C], ly = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    dl[c] = (__expf(lg[c] - m) * inv - (c == y ? 1.f : 0.f)) * invB;
    ly = (c == y) ? lg[c] : ly;
  }
  float dhp = 0.f;
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    float dlc = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) dlc = (c == 5 * h2 + k) ? dl[c] : dlc;
    dhp += dlc * v[7 + k];
  }
  const float dh = swap32_add(dhp);
  u64* hd = a.ll + OFF_HEAD + (e & 1) * HEAD_PAR + (size_t)row * HEAD_ROW;
  if (jv) {
    if (h2 == 0) st_ll(hd + HDZ + j, dh * hv * (1.f - hv), e);
    else st_ll(hd + HHB + j, hv, e);
  }
  if (wave == 0) {
    float mydl = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) mydl = (lane == c) ? dl[c] : mydl;
    if (lane < C) st_ll(hd + HDL + lane, mydl, e);
    if (lane == 0) {
      st_ll(hd + HST, m + __logf(se) - ly, e);  // xent of this row
      st_ll(hd + HST + 1, (am == y) ? 1.f : 0.f, e);
    }
  }
  if (wave == 3) stamp(a, t, 7);
}

// ---------------------------------------------------------------------------------------
// the persistent kernel
// ---------------------------------------------------------------------------------------
template <int NGT>
__global__ __launch_bounds__(256) void mlp_persistent_kernel(Args a) {
  const int B = a.B;
  const int BP = NGT > 0 ? NGT * 16 : ((B + 15) >> 4) * 16;
  const int NG = BP / 16, RT = (B + 15) >> 4;
  constexpr int MAXG = NGT > 0 ? NGT : MAXB / 16;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, r = lane & 15, q = lane >> 4;
  const int bid = blockIdx.x;
  bool fail = false;

  if (bid >= NBLK) {
    // ===================== head block: batch row bid - NBLK ===========================
    __shared__ float red[8][16];  // per-wave partial logits, [step parity][wave][c]
    for (int t = 0; t < a.steps; ++t) head_row(a, bid - NBLK, t, wave, lane, red, fail);
    return;
  }

  if (bid >= NW1) {
    // ===================== small-parameter block jt ===================================
    const int jt = bid - NW1;
    const bool upd = wave < 2 || (wave == 2 && jt == 0);  // waves owning parameters
    // owned values: wave 0 W2t[c = q*4+i][j = jt*16+r]; wave 1 b1[j = jt*16+q*4+i] (r == 0);
    // wave 2 (jt == 0) b2[c = q*4+i] (r == 0).  sp index: position in the SP plane
    int spi[4];
    bool own[4];
    float pv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (wave == 0) {
        const int c = q * 4 + i, j = jt * 16 + r;
        own[i] = c < C && j < H;
        spi[i] = SP_W2 + (own[i] ? c * H + j : 0);
      } else if (wave == 1) {
        const int j = jt * 16 + q * 4 + i;
        own[i] = r == 0 && j < H;
        spi[i] = own[i] ? j : 0;
      } else if (wave == 2) {
        const int c = q * 4 + i;
        own[i] = r == 0 && c < C;
        spi[i] = SP_B2 + (own[i] ? c : 0);
      } else {
        own[i] = false;
        spi[i] = 0;
      }
      pv[i] = own[i] ? a.p[OFF_B1 + spi[i]] : 0.f;  // SP index + OFF_B1 = flat index
    }
    const int ctr0 = (wave == 3 && jt == 0 && lane == 0) ? *a.ctr : 0;
    {
      const unsigned e0 = a.ebase + 1u;
      u64* sp = a.ll + OFF_SP + (e0 & 1) * SP_PAR;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (own[i])
#pragma unroll
          for (int c = 0; c < NREP; ++c) st_ll(sp + c * SP_REP + spi[i], pv[i], e0);
    }
    // The batch (K of every product) is split over the 4 waves -- wave w takes row groups
    // g = w, w + 4 -- so each wave pulls at most 28 granule words per lane instead of one wave
    // pulling 56 (its ~28 KB of agent-scope loads sat on the critical path: every head waits
    // for these parameters).  Products per wave (MFMA 16x16x4, lane l: A[l&15][k], B[k][l&15]):
    //   P0 dW2^T[c][j] = sum_b dl[b][c] h[b][jt*16+j]   P1 db1[jt*16+i] = sum_b dz1[b][jt*16+i]
    //   P2 db2[c] = sum_b dl[b][c] (jt == 0)
    // Partials meet in LDS (double-buffered by step parity) and the owners add them in wave
    // order.  Wave 3 of jt == 0 also folds the loss / accuracy record of the step.
    __shared__ f32x4 part[2][4][3][64];
    const bool hv_ok = jt * 16 + r < H;
    for (int t = 1; t <= a.steps; ++t) {
      const unsigned ep = a.ebase + (unsigned)t;  // HEAD granules of step t-1
      const u64* hd = a.ll + OFF_HEAD + (ep & 1) * HEAD_PAR;
      if (wave == 0) stamp(a, t, 0);
      // words: [0, 8) dl[b][r], [8, 16) h[b][jt*16+r], [16, 24) dz1[b][jt*16+r] for the 2 x 4
      // rows b = g*16 + q*4 + e of groups g = wave, wave + 4; [24, 28) stat words (rows lane,
      // lane + 64) for wave 3 of jt == 0
      float v[28];
      ll_wait<28>(
          [&](int i) -> const u64* {
            if (i >= 24) {
              const int b = lane + 64 * ((i - 24) >> 1);
              return wave == 3 && jt == 0 && b < B ? hd + (size_t)b * HEAD_ROW + HST + (i & 1)
                                                   : nullptr;
            }
            const int k = i & 7, g = wave + 4 * (k >> 2);
            const int b = g * 16 + q * 4 + (k & 3);
            if (g >= NG || b >= B) return nullptr;
            const u64* row = hd + (size_t)b * HEAD_ROW;
            if (i < 8) return r < C ? row + HDL + r : nullptr;
            if (i < 16) return hv_ok ? row + HHB + jt * 16 + r : nullptr;
            return hv_ok ? row + HDZ + jt * 16 + r : nullptr;
          },
          ep, a, v, fail);
      if (wave == 0) stamp(a, t, 1);
      f32x4 p0 = {0, 0, 0, 0}, p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0};
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (wave + 4 * h < NG) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            p0 = mfma16x16x4(v[h * 4 + e], v[8 + h * 4 + e], p0);
            p1 = mfma16x16x4(v[16 + h * 4 + e], 1.f, p1);
            if (jt == 0) p2 = mfma16x16x4(v[h * 4 + e], 1.f, p2);
          }
        }
      }
      f32x4(&pp)[4][3][64] = part[t & 1];
      pp[wave][0][lane] = p0;
      pp[wave][1][lane] = p1;
      pp[wave][2][lane] = p2;
      lds_barrier();
      if (upd) {
        f32x4 g = {0, 0, 0, 0};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const f32x4 o = pp[w][wave][lane];
#pragma unroll
          for (int i = 0; i < 4; ++i) g[i] += o[i];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (!fail) pv[i] = pv[i] - a.lr * g[i];
        if (t < a.steps) {
          const unsigned e = a.ebase + 1u + (unsigned)t;
          u64* sp = a.ll + OFF_SP + (e & 1) * SP_PAR;
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (own[i])
#pragma unroll
              for (int c = 0; c < NREP; ++c) st_ll(sp + c * SP_REP + spi[i], pv[i], e);
          if (wave == 0) stamp(a, t, 2);
        }
      } else if (wave == 3 && jt == 0) {  // loss / accuracy record of step t-1
        const float l = wave_sum(v[24] + v[26]), ac = wave_sum(v[25] + v[27]);
        if (lane == 0 && a.stats) {
          float* st = a.stats + (size_t)((ctr0 + t - 1) % a.ring) * 2;
          st[0] = l / (float)B;
          st[1] = ac / (float)B;
        }
      }
    }
    if (upd) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (own[i]) a.p[OFF_B1 + spi[i]] = pv[i];
    } else if (wave == 3 && jt == 0 && lane == 0) {
      *a.ctr = ctr0 + a.steps;
    }
    return;
  }

  // ======================= W1 block (jt, ks) ============================================
  constexpr int LW = KW + 4;          // LDS row pitch (floats)
  constexpr int LZ = MAXB + 4;        // dz1 slice pitch
  __shared__ float Wt[16][LW];
  __shared__ float Dz[16][LZ];
  __shared__ int abort_flag;
  const int jt = bid / KS, ks = bid % KS;
  const int f0 = ks * KW;
  const int fl = wave * 16 + r;       // phase A: this lane's feature within the slice
  const bool cv = fl < KW;            // wave 3: 8 live columns
  const int fc = f0 + (cv ? fl : KW - 1);
  float pw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = jt * 16 + q * 4 + i;
    pw[i] = j < H ? a.p[OFF_W1 + (size_t)j * D + fc] : 0.f;
    if (cv) Wt[q * 4 + i][fl] = pw[i];
  }
  if (tid == 0) abort_flag = 0;
  // (the first barrier of the loop orders these LDS writes before any read)

  for (int t = 0; t <= a.steps; ++t) {
    const bool last = t == a.steps;
    // phase B's x rows (independent of everything this step waits for): requested first
    constexpr int RTW = 2;
    float4 xa[RTW][4];
    if (!last) {
      const float* xb = a.x + (size_t)((a.pos0 + t) % a.nbatches) * B * D;
#pragma unroll
      for (int tt = 0; tt < RTW; ++tt) {
        const int row = (wave + 4 * tt) * 16 + r;
        const float* xr = xb + (size_t)(row < B ? row : B - 1) * D + f0;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int k = 16 * g + 4 * q;
          xa[tt][g] = f4(xr + (k < KW ? k : 0));
        }
      }
    }
    if (t > 0) {
      // ---- phase A: W1 tile update with step t-1's factors ------------------------------
      const float* xp = a.x + (size_t)((a.pos0 + t - 1) % a.nbatches) * B * D + fc;
      float xv[MAXG][4];
#pragma unroll
      for (int g = 0; g < MAXG; ++g)
        if (g < NG)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int b = g * 16 + q * 4 + e;  // rows >= B: dz1 is zero there
            xv[g][e] = xp[(size_t)(b < B ? b : B - 1) * D];
          }
      const unsigned ep = a.ebase + (unsigned)t;
      const u64* hd = a.ll + OFF_HEAD + (ep & 1) * HEAD_PAR + HDZ + jt * 16;
      // the block's dz1 slice [16 hidden][BP rows]: thread (jl = tid & 15, b = tid >> 4 + 16k)
      constexpr int NL = 16 * MAXB / 256;
      float dz[NL];
      if (wave == 0) stamp(a, t, 0);
      const int jl = tid & 15;
      const bool jvalid = jt * 16 + jl < H;
      ll_wait<NL>(
          [&](int k) -> const u64* {
            const int b = (tid >> 4) + 16 * k;
            return b < B && jvalid ? hd + (size_t)b * HEAD_ROW + jl : nullptr;
          },
          ep, a, dz, fail);
      if (wave == 0) stamp(a, t, 1);
#pragma unroll
      for (int k = 0; k < NL; ++k) Dz[jl][(tid >> 4) + 16 * k] = dz[k];
      if (fail) abort_flag = 1;
      lds_barrier();
      if (abort_flag) break;
      if (wave == 0) stamp(a, t, 2);
      f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
      for (int g = 0; g < MAXG; ++g) {
        if (g < NG) {
          const float4 av = *reinterpret_cast<const float4*>(&Dz[r][g * 16 + q * 4]);
          acc0 = mfma16x16x4(av.x, xv[g][0], acc0);
          acc1 = mfma16x16x4(av.y, xv[g][1], acc1);
          acc0 = mfma16x16x4(av.z, xv[g][2], acc0);
          acc1 = mfma16x16x4(av.w, xv[g][3], acc1);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hl = q * 4 + i, j = jt * 16 + hl;
        pw[i] = pw[i] - a.lr * (acc0[i] + acc1[i]);
        if (cv) Wt[hl][fl] = j < H ? pw[i] : 0.f;  // padded hidden rows contribute zeros
      }
      if (last) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int j = jt * 16 + q * 4 + i;
          if (cv && j < H) a.p[OFF_W1 + (size_t)j * D + f0 + fl] = pw[i];
        }
        break;
      }
    }
    lds_barrier();  // Wt of step t complete
    if (abort_flag) break;
    if (wave == 0) stamp(a, t, 3);
    // ---- phase B: z1 partial of row tiles rt = wave, wave + 4 over the block's features ---
    const unsigned e = a.ebase + 1u + (unsigned)t;
    u64* slab = a.ll + OFF_SLAB + (e & 1) * SLAB_PAR + (size_t)ks * MAXB * SLAB_ROW;
    float4 wb[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int k = 16 * g + 4 * q;
      wb[g] = k < KW ? *reinterpret_cast<const float4*>(&Wt[r][k]) : float4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int tt = 0; tt < RTW; ++tt) {
      const int rt = wave + 4 * tt;
      if (rt < RT) {
        const float rm = rt * 16 + r < B ? 1.f : 0.f;
        f32x4 o0 = {0, 0, 0, 0}, o1 = {0, 0, 0, 0};
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          o0 = mfma16x16x4(xa[tt][g].x * rm, wb[g].x, o0);
          o1 = mfma16x16x4(xa[tt][g].y * rm, wb[g].y, o1);
          o0 = mfma16x16x4(xa[tt][g].z * rm, wb[g].z, o0);
          o1 = mfma16x16x4(xa[tt][g].w * rm, wb[g].w, o1);
        }
        const int col = jt * 16 + r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rt * 16 + q * 4 + i;
          if (row < B && col < H) st_ll(slab + (size_t)row * SLAB_ROW + col, o0[i] + o1[i], e);
        }
      }
    }
    if (wave == 0) stamp(a, t, 4);
  }
}

}  // namespace mlpp

long long mlp_persistent_ll_words() { return mlpp::LL_WORDS; }

int mlp_persistent_blocks() { return mlpp::NBLK; }

int mlp_persistent_trace_steps() { return mlpp::TRACE_STEPS; }

void mlp_persistent_launch(float* p, const float* x, const int* labels, int nbatches, int pos,
                           int steps, float lr, unsigned ebase, unsigned long long* ll, int* ctr,
                           float* stats, int ring, int B, long long ticks,
                           unsigned long long* trace, hipStream_t stream) {
  using namespace mlpp;
  if (B < 1 || B > MAXB) throw std::runtime_error("mlp_persistent: batch must be in [1, 128]");
  if (!p || !x || !labels || !ll || !ctr || nbatches < 1 || pos < 0 || pos >= nbatches ||
      steps < 1 || ticks < 1)
    throw std::runtime_error("mlp_persistent: bad buffers / position / count");
  if (stats && ring < 1) throw std::runtime_error("mlp_persistent: stats ring < 1");
  if (reinterpret_cast<uintptr_t>(x) % 16 || (size_t)B * D % 4)
    throw std::runtime_error("mlp_persistent: x must be 16-byte aligned");
  Args a{p, x, labels, ll, ctr, stats, ticks, trace, lr, ebase, nbatches, pos, steps, B, ring};
  if ((B + 15) / 16 == 7)
    hipLaunchKernelGGL(mlp_persistent_kernel<7>, dim3(NBLK + B), dim3(256), 0, stream, a);
  else
    hipLaunchKernelGGL(mlp_persistent_kernel<0>, dim3(NBLK + B), dim3(256), 0, stream, a);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
