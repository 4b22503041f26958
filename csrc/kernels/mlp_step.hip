// Fused training step for the reference's MNIST MLP (784 -> 100 sigmoid -> 10,
// softmax cross-entropy, plain SGD).  Reference graph: worker.py:46-79.
//
// Design rule (measured, profiles/): at this size the step is bound by how
// many bytes EACH CU must pull and by dependent kernel boundaries (~1.5 us),
// not by FLOPs (32 MFLOP = 0.2 us of f32 MFMA).  A first version that gave
// each of 49 workgroups a full-K 16x16 tile moved ~150 KB per CU and took
// ~10 us per kernel.  This version keeps every workgroup at 7-21 KB and
// spreads each phase over ~100-350 workgroups:
//
//   K1 mlp_fwd   grid (row tile 16) x (hidden tile 16) x (K slice of 112):
//                partial z1 = x . W1 over its K slice -> slab[ks]
//                (deferred-apply mode: W1 <- W1 - lr * G on the fly,
//                 published to the ping-pong buffer by the rt == 0 blocks)
//   K2 mlp_head  one wave per batch row: z1 = sum of 7 slabs + b1,
//                h = sigmoid, logits = h . W2 + b2, softmax, xent, accuracy,
//                dlogits = (p - y)/B, dz1 = (dlogits . W2^T) * h * (1 - h)
//                -> hbuf [b][j], dz1T [j][b], dlT [c][b], rowstat [b]
//   K3 mlp_wgrad 343 blocks: dW1^T tile = dz1^T . x   (f32 MFMA, K = batch)
//                  7 blocks: dW2^T = dl^T . h, db1, db2 (MFMA against ones),
//                            mean loss / accuracy -> stats ring
//                direct mode: the SGD apply is fused into the epilogue
//                (each parameter element is owned by exactly one lane);
//                grad mode: writes the flat gradient for an all-reduce.
//
// All MFMA work is v_mfma_f32_16x16x4_f32 (exact f32).  Lane l supplies
// A[i = l&15][k = l>>4], B[k = l>>4][j = l&15]; C[row = (l>>4)*4 + r][col = l&15].
// A float4 load of k = 16g + 4q .. 16g + 4q + 3 feeds 4 MFMAs (element e is
// k = 16g + 4q + e on BOTH operands: a consistent permutation of the K sum).
//
// Parameter layout (flat f32, 79,510 elements; gradients use the same layout
// so one all-reduce covers everything):
//   [0, 78400)      W1t [100][784]   (W1t[j][i] = TF kernel W1[i][j])
//   [78400, 78500)  b1  [100]
//   [78500, 79500)  W2t [10][100]    (W2t[c][j] = TF kernel W2[j][c])
//   [79500, 79510)  b2  [10]
//
// Batch selection: every launch takes the batch's own x / label pointer.  A
// captured hipGraph therefore freezes one batch per captured step; the
// trainer captures a whole epoch (one graph = nbatches steps), so replaying
// it walks the device-resident dataset exactly like next_batch does.  No
// kernel starts with a dependent "which batch?" load (measured: ~0.5 us per
// dependent round trip on this chip).
//
// global_step (worker.py:29-32,141) is a device int advanced by ONE thread of
// mlp_wgrad after it has used the value as the stats-ring index; no other
// thread of any launch touches it.
#include "common.h"
#include <mutex>
#include <map>
#include "xgmi_ll.h"

#include <cstdlib>
#include <stdexcept>
#include <string>

namespace dtfx {
namespace mlp {

constexpr int D = 784, H = 100, C = 10;
constexpr int HT = 7;          // hidden tiles of 16 (112 padded)
constexpr int HP = HT * 16;    // padded hidden width
constexpr int KS = 7;          // K slices of K1
constexpr int KW = D / KS;     // 112 = 7 groups of 16
constexpr int FT = D / 16;     // 49 feature tiles (dW1)
constexpr int KS2 = 14;        // K slices of the pipelined step's fused apply+forward launch
constexpr int KW2 = D / KS2;   // 56 features = 3.5 MFMA groups of 16
constexpr int KS3 = 28;        // ... the single-GPU form: 28 slices of 28 features (203 blocks)
// 16-byte LL layout of the one-shot split exchange (mlp_fwdapply_kernel<.., XW, .., TWO =
// false> with DTFX_XG_SPLIT bit 0): word pair of (exchange slot, K-split wave, lane) at
// XG_W1_BASE + ((eslot * 2 + sp) * 64 + lane) * 2 -- past the parameter-offset region of
// the small parameters; a communicator needs XG_SLOT_WORDS words per slot for it.
constexpr long long XG_W1_BASE = 79616;
constexpr long long XG_SLOT_WORDS = XG_W1_BASE + (long long)HT * KS3 * 2 * 2 * 64 * 2;
constexpr int NSLAB_MAX = KS3; // slab planes in the workspace
constexpr int OFF_W1 = 0;
constexpr int OFF_B1 = H * D;
constexpr int OFF_W2 = OFF_B1 + H;
constexpr int OFF_B2 = OFF_W2 + C * H;
constexpr int NPARAM = OFF_B2 + C;
constexpr int MAXB = 256;

static_assert(KW % 16 == 0 && KS * KW == D, "K slicing of 784");
static_assert(KS2 * KW2 == D && KW2 % 8 == 0, "K slicing of the pipelined step");
static_assert(NPARAM == 79510, "parameter count of worker.py:50-53");

struct Bufs {            // workspace (zero-initialised once; padding stays 0)
  float* slab;           // [NSLAB_MAX][BP][HP]  partial z1 (KS or KS2 planes used)
  float* hbuf;           // [BP][HP]      h
  float* dz1T;           // [HP][BP]      dz1 transposed
  float* dlT;            // [16][BP]      dlogits transposed
  float* rowstat;        // [BP][2]       per-row (loss, correct)
  int* sync;             // [4] handoff words of mlp_head_flush_kernel (0 between launches):
                         //     [0] head rows done, [1] apply blocks done, [2] sticky timeout
};

__device__ __forceinline__ float4 f4(const float* p) { return *reinterpret_cast<const float4*>(p); }

// ---------------------------------------------------------------------------
// K1: partial z1 over one K slice (+ deferred W1 apply)
// ---------------------------------------------------------------------------
template <bool APPLY, bool TRACE>
__global__ __launch_bounds__(64) void mlp_fwd_kernel(
    const float* __restrict__ p_old, const float* __restrict__ grad, float lr,
    float* __restrict__ p_new, const float* __restrict__ x, Bufs w, int B,
    unsigned long long* __restrict__ tr) {
  if (TRACE) trace_stamp(tr, blockIdx.x * 4 + 0);
  const int RT = (B + 15) >> 4, BP = RT * 16;
  const int rt = blockIdx.x % RT, jt = (blockIdx.x / RT) % HT, ks = blockIdx.x / (RT * HT);
  const int lane = threadIdx.x, r = lane & 15, q = lane >> 4;

  const int row = rt * 16 + r, col = jt * 16 + r;
  const bool rv = row < B, cv = col < H;
  const int k0 = ks * KW + q * 4;
  const float* xr = x + (size_t)(rv ? row : 0) * D + k0;
  const size_t woff = OFF_W1 + (size_t)(cv ? col : 0) * D + k0;

  // Loads are unconditional (clamped rows/cols) and masked after the fact:
  // a guarded load becomes its own exec-masked branch in the ISA.
  const float rm = rv ? 1.f : 0.f, cm = cv ? 1.f : 0.f;
  float4 xa[KW / 16], wa[KW / 16];
#pragma unroll
  for (int g = 0; g < KW / 16; ++g) {
    xa[g] = f4(xr + g * 16);
    wa[g] = f4(p_old + woff + g * 16);
  }
  float4 ga[KW / 16];
  if (APPLY) {
#pragma unroll
    for (int g = 0; g < KW / 16; ++g) ga[g] = f4(grad + woff + g * 16);
  }
  // Keep every load above this point in flight together: without the fence
  // hipcc sinks them into the MFMA chain as 3-4 serial vmcnt(0) round trips.
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int g = 0; g < KW / 16; ++g) {
    xa[g].x *= rm; xa[g].y *= rm; xa[g].z *= rm; xa[g].w *= rm;
    wa[g].x *= cm; wa[g].y *= cm; wa[g].z *= cm; wa[g].w *= cm;
  }
  if (APPLY) {
#pragma unroll
    for (int g = 0; g < KW / 16; ++g) {
      float4 gg = ga[g];
      gg.x *= cm; gg.y *= cm; gg.z *= cm; gg.w *= cm;
      wa[g].x -= lr * gg.x;
      wa[g].y -= lr * gg.y;
      wa[g].z -= lr * gg.z;
      wa[g].w -= lr * gg.w;
      if (rt == 0 && cv) *reinterpret_cast<float4*>(p_new + woff + g * 16) = wa[g];
    }
  }
  if (TRACE) trace_stamp(tr, blockIdx.x * 4 + 1);
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
  for (int g = 0; g < KW / 16; ++g) {
    acc0 = mfma16x16x4(xa[g].x, wa[g].x, acc0);
    acc1 = mfma16x16x4(xa[g].y, wa[g].y, acc1);
    acc0 = mfma16x16x4(xa[g].z, wa[g].z, acc0);
    acc1 = mfma16x16x4(xa[g].w, wa[g].w, acc1);
  }
  float* out = w.slab + ((size_t)ks * BP + rt * 16 + q * 4) * HP + jt * 16 + r;
  if (TRACE) {
    asm volatile("" ::"v"(acc0[0]), "v"(acc1[0]));
    trace_stamp(tr, blockIdx.x * 4 + 2);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) out[(size_t)i * HP] = acc0[i] + acc1[i];
  if (TRACE) trace_stamp(tr, blockIdx.x * 4 + 3);
}

// ---------------------------------------------------------------------------
// K2: per-row head (one wave per batch row)
// ---------------------------------------------------------------------------
// The factor engines' dz1 all-gather of one head row (mlp_head_kernel<.., XW>): BL = polls as
// 16-byte buffer loads and pushes as global stores (DTFX_XG_SPLIT bit 4, as xg_exchange2p).
template <int XW, bool BL>
__device__ __forceinline__ void head_allgather(const MlpXg& xg, unsigned ep, int row, int lane,
                                               int BP, const float (&dzv)[2],
                                               float* __restrict__ dz1A, bool& fail) {
  {
    // the row's 100 factors travel as 50 16-byte word pairs {dz(2l), ep, dz(2l+1), ep} at
    // word row * HP + 2l of slot (parity, me) -- a wave's pushes and polls are contiguous
    // 800-B runs, one store / load per lane and peer -- and land in dz1A [XW][BP][HP] row-major
    // (one 8-byte store per lane and rank).  Each 8-byte half carries the epoch (as
    // xg_exchange16); every poll is issued before the pushes (xgll::first_loads).
    using xgll::u64;
    using xgll::u32x4;
    const long long par = ep & 1u, plane = (long long)HP * BP;
    const int me = xgll::uniform(xg.rank);
    const bool act = lane < H / 2;
    const long long woff = (long long)row * HP + 2 * (act ? lane : 0);
    auto slot = [&](int dst, int src) {
      return xgll::uniform_ptr((u64*)xg.peers.data[dst]) + (par * XW + src) * xg.S + woff;
    };
    const xgll::OwnPoll pr(BL ? xgll::uniform_ptr((const u64*)xg.peers.data[me]) : nullptr);
    auto poll = [&](int q) {
      if constexpr (BL) return pr.pair((par * XW + q) * xg.S, woff);
      else return xgll::load_pair(slot(me, q));
    };
    u32x4 wq[XW];
#pragma unroll
    for (int q = 0; q < XW; ++q)
      if (act && q != me) wq[q] = poll(q);
    if (act) {
      const u32x4 out = {__float_as_uint(dzv[0]), ep, __float_as_uint(dzv[1]), ep};
#pragma unroll
      for (int d = 0; d < XW; ++d)
        if (d != me) {
          if constexpr (BL) xgll::store_pair_g(slot(d, me), out);
          else *(u32x4*)slot(d, me) = out;
        }
    }
    if (act) {
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      for (;;) {
        bool ready = true;
#pragma unroll
        for (int q = 0; q < XW; ++q)
          if (q != me && (wq[q].y != ep || wq[q].w != ep)) {
            ready = false;
            wq[q] = poll(q);
          }
        if (ready) break;
        if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > xg.ticks) {
          fail = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
#pragma unroll
      for (int q = 0; q < XW; ++q) {
        const float2 v = q == me ? make_float2(dzv[0], dzv[1])
                                 : make_float2(__uint_as_float(wq[q].x), __uint_as_float(wq[q].z));
        *reinterpret_cast<float2*>(&dz1A[q * plane + woff]) = v;
      }
    }
  }
}

// XW > 0 (factor exchange, MlpXg in xgmi.h): the row's dz1 values are also pushed as LL
// words into slot (parity, me) of every peer and every peer's values for the same (j, row)
// are gathered from local memory into dz1A [XW][BP][HP] -- the all-gather of the backprop
// factors that mlp_wgrad_factor_kernel turns into the global weight gradient.
// (the body of one row's wave: mlp_head_kernel runs it as a one-wave block, the terminal
// head + apply kernel of a launched region as one of four waves of a block)
template <bool APPLY, bool TRACE, int XW = 0, int NSLAB = KS>
__device__ __forceinline__ void head_row(
    const int row, const int lane, const float* __restrict__ p_old,
    const float* __restrict__ grad, float lr, float* __restrict__ p_new,
    const int* __restrict__ labels, const Bufs& w, int B, unsigned long long* __restrict__ tr,
    const MlpXg& xg, float* __restrict__ dz1A) {
  static_assert(XW == 0 || (!APPLY && !TRACE), "the factor exchange runs the direct step");
  if (TRACE) trace_stamp(tr, row * 4 + 0);
  const int BP = ((B + 15) >> 4) * 16;
  const int y = labels[row];
  const unsigned ep = XW > 0 ? xg.epochs[MLP_XG_HEAD_EPOCH + row] + 1 : 0u;
  const bool publish = APPLY && row == 0;

  // All loads first, unconditional (clamped), masked afterwards.  Lane l owns the ADJACENT
  // hidden units 2l, 2l + 1 (lanes 0..49), so every per-unit operand -- the NSLAB partial
  // z1 slabs, b1, the 10 W2 columns -- arrives as one 8-B load per pair: 49 load
  // instructions per lane instead of 88 (more than the 63 a wave can keep in flight:
  // the 28-slab step waited out a second round trip here).
  float hv[2], w2[2][C], zs[2], b1v[2], b2v[C];
  int jj[2];
  bool jv[2];
  const int j0 = min(2 * lane, H - 2);  // (H even: j0, j0 + 1 always a valid, aligned pair)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    jv[u] = 2 * lane + u < H;
    jj[u] = j0 + u;
    zs[u] = 0.f;
  }
#pragma unroll
  for (int s = 0; s < NSLAB; ++s) {
    const float2 v = *reinterpret_cast<const float2*>(&w.slab[((size_t)s * BP + row) * HP + j0]);
    zs[0] += v.x;
    zs[1] += v.y;
  }
  {
    const float2 v = *reinterpret_cast<const float2*>(&p_old[OFF_B1 + j0]);
    b1v[0] = v.x;
    b1v[1] = v.y;
  }
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float2 v = *reinterpret_cast<const float2*>(&p_old[OFF_W2 + c * H + j0]);
    w2[0][c] = v.x;
    w2[1][c] = v.y;
  }
#pragma unroll
  for (int c = 0; c < C; ++c) b2v[c] = p_old[OFF_B2 + c];
  float gb1[2], gw2[2][C], gb2[C];
  if (APPLY) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      gb1[u] = grad[OFF_B1 + jj[u]];
#pragma unroll
      for (int c = 0; c < C; ++c) gw2[u][c] = grad[OFF_W2 + c * H + jj[u]];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) gb2[c] = grad[OFF_B2 + c];
  }
  __builtin_amdgcn_sched_barrier(0);  // all loads in flight together
  if (APPLY) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      b1v[u] -= lr * gb1[u];
#pragma unroll
      for (int c = 0; c < C; ++c) w2[u][c] -= lr * gw2[u][c];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) b2v[c] -= lr * gb2[c];
    if (publish) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (jv[u]) {
          p_new[OFF_B1 + jj[u]] = b1v[u];
#pragma unroll
          for (int c = 0; c < C; ++c) p_new[OFF_W2 + c * H + jj[u]] = w2[u][c];
        }
      if (lane < C) {
        float b2l = 0.f;
#pragma unroll
        for (int c = 0; c < C; ++c) b2l = (lane == c) ? b2v[c] : b2l;
        p_new[OFF_B2 + lane] = b2l;
      }
    }
  }
  if (TRACE) trace_stamp(tr, row * 4 + 1);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    hv[u] = jv[u] ? sigmoidf_(zs[u] + b1v[u]) : 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) w2[u][c] = jv[u] ? w2[u][c] : 0.f;
    if (jv[u]) w.hbuf[(size_t)row * HP + jj[u]] = hv[u];
  }
  // logits = h . W2 + b2 (10 interleaved DPP wave reductions; every lane ends with all 10)
  float lg[C];
#pragma unroll
  for (int c = 0; c < C; ++c) lg[c] = hv[0] * w2[0][c] + hv[1] * w2[1][c];
  wave_sum_n(lg);
#pragma unroll
  for (int c = 0; c < C; ++c) lg[c] += b2v[c];

  float m = lg[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < C; ++c)
    if (lg[c] > m) { m = lg[c]; am = c; }  // first max, like tf.argmax
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) se += __expf(lg[c] - m);
  const float inv = fast_rcp(se), invB = 1.f / (float)B;
  float dl[C], ly = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    dl[c] = (__expf(lg[c] - m) * inv - (c == y ? 1.f : 0.f)) * invB;
    ly = (c == y) ? lg[c] : ly;
  }
  float dzv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int j = 2 * lane + u;
    dzv[u] = 0.f;
    if (j < H) {
      float dh = 0.f;
#pragma unroll
      for (int c = 0; c < C; ++c) dh += dl[c] * w2[u][c];
      dzv[u] = dh * hv[u] * (1.f - hv[u]);
      w.dz1T[(size_t)j * BP + row] = dzv[u];
    }
  }
  if constexpr (XW > 0) {
    bool fail = false;
    if (xg.split & 16) head_allgather<XW, true>(xg, ep, row, lane, BP, dzv, dz1A, fail);
    else head_allgather<XW, false>(xg, ep, row, lane, BP, dzv, dz1A, fail);
    if (lane == 0) xg.epochs[MLP_XG_HEAD_EPOCH + row] = ep;
    if (fail) atomicExch(xg.err, 1);
  }
  if (TRACE) trace_stamp(tr, row * 4 + 2);
  float mydl = 0.f;
#pragma unroll
  for (int c = 0; c < C; ++c) mydl = (lane == c) ? dl[c] : mydl;
  if (lane < C) w.dlT[(size_t)lane * BP + row] = mydl;
  if (lane == 0) {
    w.rowstat[2 * row] = m + __logf(se) - ly;  // xent of this row
    w.rowstat[2 * row + 1] = (am == y) ? 1.f : 0.f;
  }
  if (TRACE) trace_stamp(tr, row * 4 + 3);
}

template <bool APPLY, bool TRACE, int XW = 0, int NSLAB = KS>
__global__ __launch_bounds__(64) void mlp_head_kernel(
    const float* __restrict__ p_old, const float* __restrict__ grad, float lr,
    float* __restrict__ p_new, const int* __restrict__ labels, Bufs w, int B,
    unsigned long long* __restrict__ tr, MlpXg xg, float* __restrict__ dz1A) {
  head_row<APPLY, TRACE, XW, NSLAB>(blockIdx.x, threadIdx.x, p_old, grad, lr, p_new, labels, w,
                                     B, tr, xg, dz1A);
}

// ---------------------------------------------------------------------------
// K3: weight gradients (+ fused SGD apply in direct mode)
// ---------------------------------------------------------------------------
// NGT > 0: batch padded to NGT*16 rows at compile time (branch-free loads);
// NGT == 0: generic (runtime NG, guarded loops).
// XW > 0: fused xGMI gradient exchange over XW ranks before the (direct) apply.
template <int XW, int N = 4>
__device__ __forceinline__ void xg_exchange(const MlpXg& xg, unsigned ep, const size_t (&off)[N],
                                            const bool (&ok)[N], float (&v)[N], bool& fail) {
  using xgll::u64;
  const long long par = ep & 1u;
  const int me = xgll::uniform(xg.rank);
  auto local = [&](int j) { return (const u64*)xg.peers.data[me] + (par * XW + j) * xg.S; };
  u64 w[N][XW];  // first polls before the pushes (xgll::first_loads: one vmcnt for both)
  xgll::first_loads<XW, N>(local, off, ok, me, ep, w);
#pragma unroll
  for (int i = 0; i < N; ++i) {
    if (!ok[i]) continue;
    const u64 wd = xgll::word(v[i], ep);
#pragma unroll
    for (int d = 0; d < XW; ++d)
      if (d != me) xgll::store((u64*)xg.peers.data[d] + (par * XW + me) * xg.S + off[i], wd);
  }
  if (!fail) xgll::finish_sum_n<XW, N>(local, off, ok, me, ep, w, v, xg.ticks, fail);
}

// Two-shot form of xg_exchange (reduce-scatter + all-gather inside the wave): element i of
// lane l (hidden row 4 q + i of the tile, q = l / 16) is owned by rank (q + 4 i) % XW -- the
// same on every rank, and one owner per 16-lane row segment, so every push below writes whole
// 128-byte runs.  (1) a non-owned value goes to its owner only (slot (par, me) of the owner),
// (2) the owner sums the XW contributions in rank order and pushes the sum into every peer's
// result region (2 XW + par) -- the push layout's last two slots --, (3) a non-owned element
// waits for its owner's sum.  Per rank 2 (XW-1)/XW words per element cross the links instead
// of XW-1 (at 8 ranks 1.75 vs 7), for one more dependent hop.  Every rank pushes before it
// waits in each phase: no wait cycle.
// Tried (round 4, tools/probes/engine_trace.py): wave-uniform owners ((eslot * 4 + i) % XW,
// every owned set's gather in full 64-lane instructions, 4x fewer load instructions).  The
// median wave's exchange at 8 ranks fell 4.7 -> 1.8 us, but the owning waves then carried all
// of the gather transactions, the launch's span grew 8.2 -> 9.0 us and the step's local cost
// 11.8 -> 12.6 us (W = 4: 10.1 -> 10.7): the per-lane owners keep every wave's share of the
// uncached-memory transactions equal, which is what bounds the phase.
// One-shot exchange of a lane's TWO elements as one 16-byte word pair {v0, epoch, v1, epoch}
// per peer (a single dwordx4 store / load instead of two 8-byte LL accesses: half the memory
// instructions and requests of the wave, and 16-byte fabric writes on real xGMI).  Each 8-byte
// half still carries its own epoch, so a reader never accepts a value of another epoch even if
// the pair were observed as two 8-byte halves.  `woff`: this (slot, wave, lane)'s pair in the
// XG_W1_BASE layout -- the same on every rank.  `live` = false (a pair of padding columns /
// hidden rows, the same on every rank): neither pushed nor gathered -- 22 % of the layout's
// pairs, so the links carry live parameters only (78,400 of 100,352 words).
// BL: polls as 16-byte buffer loads, pushes as global stores (as xg_exchange2p<XW, true>).
template <int XW, bool BL = false>
__device__ __forceinline__ void xg_exchange16(const MlpXg& xg, unsigned ep, long long woff,
                                              float (&v)[2], bool& fail, bool live = true) {
  using xgll::u64;
  using xgll::u32x4;
  const long long par = ep & 1u;
  const int me = xgll::uniform(xg.rank);
  const u64* mine = xgll::uniform_ptr((const u64*)xg.peers.data[me]) + woff;
  const xgll::OwnPoll pr(BL ? mine - woff : nullptr);
  auto poll = [&](int j) {
    if constexpr (BL) return pr.pair((par * XW + j) * xg.S, woff);
    else return xgll::load_pair(mine + (par * XW + j) * xg.S);
  };
  const u32x4 out = {__float_as_uint(v[0]), ep, __float_as_uint(v[1]), ep};
  u32x4 w[XW];  // first polls before the pushes (xgll::first_loads: one vmcnt for both)
#pragma unroll
  for (int j = 0; j < XW; ++j) {
    w[j] = u32x4{0u, ep, 0u, ep};
    if (live && j != me) w[j] = poll(j);
  }
#pragma unroll
  for (int d = 0; d < XW; ++d)
    if (live && d != me) {
      u64* dst = xgll::uniform_ptr((u64*)xg.peers.data[d]) + (par * XW + me) * xg.S + woff;
      if constexpr (BL) xgll::store_pair_g(dst, out);
      else *(u32x4*)dst = out;
    }
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int j = 0; j < XW; ++j)
      if (j != me && (w[j].y != ep || w[j].w != ep)) {
        ready = false;
        w[j] = poll(j);
      }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > xg.ticks) {
      fail = true;
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  float a0 = 0.f, a1 = 0.f;  // rank-ordered sums: the same bits on every rank
#pragma unroll
  for (int j = 0; j < XW; ++j) {
    a0 += j == me ? v[0] : __uint_as_float(w[j].x);
    a1 += j == me ? v[1] : __uint_as_float(w[j].z);
  }
  v[0] = a0;
  v[1] = a1;
}

// Two-shot form of xg_exchange16 (fused2x, round 5): a lane's TWO elements travel as one
// 16-byte word pair in the XG_W1_BASE layout (`woff`, as the one-shot) and the PAIR has one
// owner rank, (q + 4 sp) % XW -- the same on every rank; at 8 ranks the 8 (q, sp) classes of a
// column group are the 8 owners.  (1) a non-owner lane pushes its pair to the owner's slot
// (parity, me); (2) an owner lane gathers the XW - 1 peers' pairs, sums each element in rank
// order and pushes the sums into every peer's result region (2 XW + parity); (3) a non-owner
// lane waits for its owner's sums.  Per hop one 16-byte store / load per lane and peer instead
// of two 8-byte LL accesses to two owners (per-element owners, xg_exchange2), and every poll
// is issued before the hop's own pushes (xgll::first_loads: stores and loads share one
// in-order vmcnt).  Each 8-byte half carries the epoch, as in xg_exchange16.
// `live` as in xg_exchange16: a dead pair is neither pushed, gathered nor broadcast.
// BL (DTFX_XG_SPLIT bit 4, round 6): the polls of the own slot region as 16-byte raw buffer
// loads and the pushes as GLOBAL stores (xgll::OwnPoll / store_pair_g) instead of FLAT
// accesses -- same words, same coherence bits.
template <int XW, bool BL = false>
__device__ __forceinline__ void xg_exchange2p(const MlpXg& xg, unsigned ep, long long woff,
                                              float (&v)[2], bool& fail, int lane, int sp,
                                              unsigned long long* trw = nullptr,
                                              bool live = true) {
  using xgll::u64;
  using xgll::u32x4;
  const long long par = ep & 1u;
  const int me = xgll::uniform(xg.rank);
  // owner class of the pair: (q + 4 sp) % XW -- at 8 ranks one rank owns one (q, sp) row of
  // a column group.  DTFX_XG_SPLIT bit 3 (A/B runs): (q + 4 (sp ^ h)) % XW, h = the lane's half
  // of its 16-lane row, so a rank owns half a row in EACH of the two waves
  const int h = (xg.split & 8) ? ((lane >> 3) & 1) : 0;
  const int own = ((lane >> 4) + 4 * (sp ^ h)) % XW;
  const bool mine = live && own == me, other = live && own != me;
  auto base = [&](int dst) { return xgll::uniform_ptr((u64*)xg.peers.data[dst]); };
  auto slot = [&](int dst, int src) { return base(dst) + (par * XW + src) * xg.S + woff; };
  auto result = [&](int dst) { return base(dst) + (2 * XW + par) * xg.S + woff; };
  auto ready2 = [&](const u32x4& w) { return w.y == ep && w.w == ep; };
  const xgll::OwnPoll pr(BL ? base(me) : nullptr);
  auto poll_slot = [&](int j) {
    if constexpr (BL) return pr.pair((par * XW + j) * xg.S, woff);
    else return xgll::load_pair(slot(me, j));
  };
  auto poll_result = [&]() {
    if constexpr (BL) return pr.pair((2 * XW + par) * xg.S, woff);
    else return xgll::load_pair(result(me));
  };
  auto put = [&](u64* p, const u32x4& w) {
    if constexpr (BL) xgll::store_pair_g(p, w);
    else *(u32x4*)p = w;
  };
  // ---- hop 1: owners' first polls, then the non-owners' push to their owner
  u32x4 w[XW];
#pragma unroll
  for (int j = 0; j < XW; ++j)
    if (mine && j != me) w[j] = poll_slot(j);
  const u32x4 out = {__float_as_uint(v[0]), ep, __float_as_uint(v[1]), ep};
  // uniform loop over destinations, per-lane predicate: a per-lane peer index would turn the
  // kernel-argument pointer table into a private (scratch) array
#pragma unroll
  for (int d = 0; d < XW; ++d)
    if (other && own == d) put(slot(d, me), out);
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  if (mine) {
    for (;;) {
      bool ready = true;
#pragma unroll
      for (int j = 0; j < XW; ++j)
        if (j != me && !ready2(w[j])) {
          ready = false;
          w[j] = poll_slot(j);
        }
      if (ready) break;
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > xg.ticks) {
        fail = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    float a0 = 0.f, a1 = 0.f;  // rank-ordered sums: the same bits on every rank
#pragma unroll
    for (int j = 0; j < XW; ++j) {
      a0 += j == me ? v[0] : __uint_as_float(w[j].x);
      a1 += j == me ? v[1] : __uint_as_float(w[j].z);
    }
    v[0] = a0;
    v[1] = a1;
  }
  if (trw) trace_stamp(trw, 5);  // probe builds: the owned sums are complete
  // ---- hop 2: non-owners' first poll of the result, then the owners' broadcast
  u32x4 r = {0u, 0u, 0u, 0u};
  if (other) r = poll_result();
  if (mine && !fail) {
    const u32x4 sum = {__float_as_uint(v[0]), ep, __float_as_uint(v[1]), ep};
#pragma unroll
    for (int d = 0; d < XW; ++d)
      if (d != me) put(result(d), sum);
  }
  if (other) {
    const long long t1 = (long long)__builtin_amdgcn_s_memrealtime();
    while (!ready2(r)) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - t1 > xg.ticks) {
        fail = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      r = poll_result();
    }
    v[0] = __uint_as_float(r.x);
    v[1] = __uint_as_float(r.z);
  }
}

// N < 4: the lane's elements i0 .. i0 + N - 1 of the four (the exchange split over the
// K-split waves of mlp_fwdapply_kernel); ownership is by the element index i either way.
template <int XW, int N = 4>
__device__ __forceinline__ void xg_exchange2(const MlpXg& xg, unsigned ep, const size_t (&off)[N],
                                             const bool (&ok)[N], float (&v)[N], bool& fail,
                                             int lane, unsigned long long* trw = nullptr,
                                             int i0 = 0) {
  using xgll::u64;
  const long long par = ep & 1u;
  const int me = xgll::uniform(xg.rank);
  const int q = lane >> 4;
  int own[N];
  bool mine[N], other[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    own[i] = (q + 4 * (i0 + i)) % XW;
    mine[i] = ok[i] && own[i] == me;
    other[i] = ok[i] && own[i] != me;
  }
  auto slot = [&](int dst, int src) {
    return xgll::uniform_ptr((u64*)xg.peers.data[dst]) + (par * XW + src) * xg.S;
  };
  auto result = [&](int dst) {
    return xgll::uniform_ptr((u64*)xg.peers.data[dst]) + (2 * XW + par) * xg.S;
  };
  auto local = [&](int j) { return (const u64*)slot(me, j); };
  // each hop issues its first polls before its pushes (xgll::first_loads: one vmcnt for both)
  u64 w1[N][XW];
  xgll::first_loads<XW, N>(local, off, mine, me, ep, w1);
  // uniform loop over destinations, per-lane predicate: a per-lane peer index would turn the
  // kernel-argument pointer table into a private (scratch) array
#pragma unroll
  for (int d = 0; d < XW; ++d) {
    if (d == me) continue;
    u64* dst = slot(d, me);
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (other[i] && own[i] == d) xgll::store(dst + off[i], xgll::word(v[i], ep));
  }
  if (!fail) xgll::finish_sum_n<XW, N>(local, off, mine, me, ep, w1, v, xg.ticks, fail);
  if (trw) trace_stamp(trw, 5);  // probe builds: the owned sums are complete
  u64 w2[N];
  xgll::first_loads1<N>(result(me), off, other, ep, w2);
#pragma unroll
  for (int d = 0; d < XW; ++d) {
    if (d == me) continue;
    u64* dst = result(d);
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (mine[i]) xgll::store(dst + off[i], xgll::word(v[i], ep));
  }
  if (!fail) xgll::finish_wait_n<N>(result(me), off, other, ep, w2, v, xg.ticks, fail);
}

// Small parameters of hidden tile jt (one product per wave), shared by mlp_wgrad_kernel and
// mlp_wgrad_factor_kernel; eidx = this wave's exchange-epoch slot.
// p_src: where the current parameter values are read (== p except in the pipelined step,
// which reads the old ping-pong buffer and writes the new one); stats_on = 0 skips the
// loss/accuracy record and the global_step increment.
template <bool DIRECT, int NGT, int XW>
__device__ __forceinline__ void wgrad_small(int jt, int wave, int lane, int eidx,
                                            float* __restrict__ p, float lr,
                                            float* __restrict__ grad, const Bufs& w,
                                            int* __restrict__ ctr, float* __restrict__ stats,
                                            int stats_ring, int B, const MlpXg& xg,
                                            const float* __restrict__ p_src = nullptr,
                                            int stats_on = 1) {
  if (p_src == nullptr) p_src = p;
  const int BP = NGT > 0 ? NGT * 16 : ((B + 15) >> 4) * 16;
  const int NG = NGT > 0 ? NGT : BP / 16;
  const int r = lane & 15, q = lane >> 4;
  constexpr int MAXG = NGT > 0 ? NGT : MAXB / 16;
  // ---- small parameters of hidden tile jt: one product per wave -----------
  //   wave 0: dW2^T[:, jt] = dlT . h[:, jt]   wave 1: db1[jt] = dz1T[jt] . 1
  //   wave 2: db2 = dlT . 1 (jt == 0)         wave 3: loss/accuracy (jt == 0)
  // With an exchange (XW > 0), the dW2 product is formed by waves 0 AND 2, each exchanging
  // and applying half of every lane's elements (the exchange's uncached-memory transactions
  // bound these blocks, as in mlp_fwdapply_kernel's split exchange), and db2 moves to wave 3
  // after the loss / accuracy record.
  const bool SPLIT = XW > 0 && (xg.split & 2);
  int role = wave;  // 0 / 2 (SPLIT): dW2 (halves), 1: db1, 2 (!SPLIT): db2, 3: stats (+ db2)
  if (wave == 3) {
    if (jt != 0) return;
    if (stats_on) {
      float l = 0.f, a = 0.f;
      for (int b = lane; b < B; b += 64) {
        l += w.rowstat[2 * b];
        a += w.rowstat[2 * b + 1];
      }
      l = wave_sum(l);
      a = wave_sum(a);
      if (lane == 0) {
        const int step = *ctr;  // this thread is the only reader/writer of ctr
        if (stats) {
          float* st = stats + (size_t)(step % stats_ring) * 2;
          st[0] = l / (float)B;
          st[1] = a / (float)B;
        }
        *ctr = step + 1;
      }
    }
    if (!SPLIT) return;
    role = 4;  // db2
  }
  if (!SPLIT && wave == 2 && jt != 0) return;
  const bool dw2 = role == 0 || (SPLIT && role == 2);
  const bool db2 = role == 4 || (!SPLIT && role == 2);
  const float* A = (role == 1) ? w.dz1T + (size_t)(jt * 16 + r) * BP + q * 4
                               : w.dlT + (size_t)r * BP + q * 4;
  const float* hb = w.hbuf + jt * 16 + r;
  const unsigned ep = XW > 0 ? xg.epochs[eidx] + 1 : 0u;
  float4 av[MAXG];
  float bv[MAXG][4];
#pragma unroll
  for (int g = 0; g < MAXG; ++g)
    if (g < NG) av[g] = f4(A + g * 16);
  if (dw2) {  // one uniform branch around the whole B-operand load block
#pragma unroll
    for (int g = 0; g < MAXG; ++g)
      if (g < NG)
#pragma unroll
        for (int e = 0; e < 4; ++e) bv[g][e] = hb[(size_t)(g * 16 + q * 4 + e) * HP];
  } else {
#pragma unroll
    for (int g = 0; g < MAXG; ++g)
#pragma unroll
      for (int e = 0; e < 4; ++e) bv[g][e] = 1.f;
  }
  __builtin_amdgcn_sched_barrier(0);  // all loads in flight together
  // Destination offsets (and, in direct mode, the current values) resolved
  // before the MFMAs so the epilogue is a pure store.
  size_t off[4];
  bool ok[4];
  float pv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (dw2) {  // C[c = q*4+i][j = jt*16 + r] -> dW2t[c][j]; SPLIT: wave 0 i < 2, wave 2 i >= 2
      const int c = q * 4 + i, j = jt * 16 + r;
      ok[i] = c < C && j < H && (!SPLIT || (i >> 1) == (role >> 1));
      off[i] = OFF_W2 + (c < C && j < H ? c * H + j : 0);
    } else if (role == 1) {  // C[j = jt*16 + q*4+i][*] -> db1[j]
      const int j = jt * 16 + q * 4 + i;
      ok[i] = r == 0 && j < H;
      off[i] = OFF_B1 + (j < H ? j : 0);
    } else {  // db2: C[c = q*4+i][*] -> db2[c]
      const int c = q * 4 + i;
      ok[i] = r == 0 && c < C;
      off[i] = OFF_B2 + (c < C ? c : 0);
    }
    if (DIRECT) pv[i] = p_src[off[i]];
  }
  (void)db2;
  __builtin_amdgcn_sched_barrier(0);
  // NB: padded batch columns of dz1T/dlT are zero, so multiplying by 1 is exact.
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
  for (int g = 0; g < MAXG; ++g) {
    if (g < NG) {
      acc0 = mfma16x16x4(av[g].x, bv[g][0], acc0);
      acc1 = mfma16x16x4(av[g].y, bv[g][1], acc1);
      acc0 = mfma16x16x4(av[g].z, bv[g][2], acc0);
      acc1 = mfma16x16x4(av[g].w, bv[g][3], acc1);
    }
  }
  float v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = acc0[i] + acc1[i];
  bool fail = false;
  if constexpr (XW > 0) {
    if (SPLIT && (role == 1 || role == 4)) {
      // db1 / db2: the product against ones replicates every value over the 16 lanes of its
      // row group, so lane r < 4 of group q takes element i = r alone -- ONE element per lane
      // (W-1 stores, W-1 loads) instead of four with one live lane in sixteen (the traced
      // tail of these blocks: 6.4 us at 8 ranks, profiles/r4/engine_trace/)
      const int is = r & 3;
      auto sel = [&](auto (&a)[4]) { return is == 0 ? a[0] : is == 1 ? a[1] : is == 2 ? a[2] : a[3]; };
      const bool live = r < 4 && (role == 1 ? (jt * 16 + q * 4 + is < H) : (q * 4 + is < C));
      size_t o1[1] = {sel(off)};
      bool k1[1] = {live};
      float v1[1] = {sel(v)};
      xg_exchange<XW, 1>(xg, ep, o1, k1, v1, fail);
      if (live && !fail) {
        if (DIRECT) p[o1[0]] = sel(pv) - lr * v1[0];
        else grad[o1[0]] = v1[0];
      }
      if (lane == 0) xg.epochs[eidx] = ep;
      if (fail) atomicExch(xg.err, 1);
      return;
    }
    if (SPLIT && dw2) {  // this wave's half: elements 2 (role / 2) + e of every lane
      const bool hi = role == 2;  // (selects: no dynamically indexed register arrays)
      size_t o2[2] = {hi ? off[2] : off[0], hi ? off[3] : off[1]};
      bool k2[2] = {hi ? ok[2] : ok[0], hi ? ok[3] : ok[1]};
      float v2[2] = {hi ? v[2] : v[0], hi ? v[3] : v[1]};
      xg_exchange<XW, 2>(xg, ep, o2, k2, v2, fail);
      if (hi) {
        v[2] = v2[0];
        v[3] = v2[1];
      } else {
        v[0] = v2[0];
        v[1] = v2[1];
      }
    } else {
      xg_exchange<XW>(xg, ep, off, ok, v, fail);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (ok[i] && !fail) {
      if (DIRECT) p[off[i]] = pv[i] - lr * v[i];
      else grad[off[i]] = v[i];
    }
  }
  if constexpr (XW > 0) {
    if (lane == 0) xg.epochs[eidx] = ep;
    if (fail) atomicExch(xg.err, 1);
  }
}

template <bool DIRECT, bool TRACE, int NGT, int XW = 0>
__global__ __launch_bounds__(256) void mlp_wgrad_kernel(
    float* __restrict__ p, float lr, float* __restrict__ grad, const float* __restrict__ x,
    Bufs w, int* __restrict__ ctr, float* __restrict__ stats, int stats_ring, int B,
    unsigned long long* __restrict__ tr, MlpXg xg) {
  static_assert(XW == 0 || DIRECT, "the fused exchange applies the update directly");
  const int BP = NGT > 0 ? NGT * 16 : ((B + 15) >> 4) * 16;
  const int NG = NGT > 0 ? NGT : BP / 16;
  // readfirstlane: make the wave id provably uniform (scalar branches, not exec masks)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  constexpr int MAXG = NGT > 0 ? NGT : MAXB / 16;
  constexpr int FG = (FT + 3) / 4;  // 13 feature groups of 4 waves
  const int bid = blockIdx.x;

  if (bid < HT * FG) {
    // ---- dW1^T tile (jt, kt) = dz1T[jt] . x[:, kt], one tile per wave ------
    const int jt = bid / FG, kt = (bid % FG) * 4 + wave;
    if (kt >= FT) return;
    unsigned long long* trw = tr + (size_t)(bid * 4 + wave) * 4;
    if (TRACE) trace_stamp(trw, 0);
    const float* xc = x + kt * 16 + r;
    const float* a = w.dz1T + (size_t)(jt * 16 + r) * BP + q * 4;
    float4 av[MAXG];
    float xv[MAXG][4];
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
      if (g < NG) {
        av[g] = f4(a + g * 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int b = g * 16 + q * 4 + e;  // rows >= B: dz1T is zero there
          xv[g][e] = xc[(size_t)(b < B ? b : B - 1) * D];
        }
      }
    }
    const unsigned ep = XW > 0 ? xg.epochs[bid * 4 + wave] + 1 : 0u;
    float pw[4];
    if (DIRECT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = jt * 16 + q * 4 + i;
        pw[i] = p[OFF_W1 + (size_t)(j < H ? j : H - 1) * D + kt * 16 + r];
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // all loads in flight together
    if (TRACE) trace_stamp(trw, 1);
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < MAXG; ++g) {
      if (g < NG) {
        acc0 = mfma16x16x4(av[g].x, xv[g][0], acc0);
        acc1 = mfma16x16x4(av[g].y, xv[g][1], acc1);
        acc0 = mfma16x16x4(av[g].z, xv[g][2], acc0);
        acc1 = mfma16x16x4(av[g].w, xv[g][3], acc1);
      }
    }
    if (TRACE) {
      asm volatile("" ::"v"(acc0[0]), "v"(acc1[0]));
      trace_stamp(trw, 2);
    }
    size_t offw[4];
    bool okw[4];
    float gv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = jt * 16 + q * 4 + i;
      okw[i] = j < H;
      offw[i] = OFF_W1 + (size_t)(j < H ? j : 0) * D + kt * 16 + r;
      gv[i] = acc0[i] + acc1[i];
    }
    bool fail = false;
    if constexpr (XW > 0) xg_exchange<XW>(xg, ep, offw, okw, gv, fail);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (okw[i] && !fail) {
        if (DIRECT) p[offw[i]] = pw[i] - lr * gv[i];
        else grad[offw[i]] = gv[i];
      }
    }
    if constexpr (XW > 0) {
      if (lane == 0) xg.epochs[bid * 4 + wave] = ep;
      if (fail) atomicExch(xg.err, 1);
    }
    if (TRACE) trace_stamp(trw, 3);
    return;
  }

  wgrad_small<DIRECT, NGT, XW>(bid - HT * FG, wave, lane, bid * 4 + wave, p, lr, grad, w, ctr,
                               stats, stats_ring, B, xg);
}



// ---------------------------------------------------------------------------
// Pipelined single-GPU step (2 launches): K1' applies step t-1's SGD update and runs
// step t's forward in ONE launch, then mlp_head_kernel<.., KS2> finishes step t.
//   blocks [0, HT*KS2): block (jt, ks) OWNS the W1 tile [16 hidden][56 features]:
//     wave w forms dW1^T[jt][ks*56 + 16w .. +16) = dz1T[jt] . x_prev (f32 MFMA,
//     K = batch; wave 3 has 8 live columns), W1new = W1old - lr * g -> LDS + p_new;
//     barrier; then z1 partial of row tiles rt = w, w+4, .. over the block's 56 features
//     with W1new from LDS -> slab[ks].  No tile is computed twice and no W1 gradient is
//     ever stored.
//   blocks [HT*KS2, +HT): wgrad_small (dW2 / db1 / db2 of step t-1, p_old -> p_new; the
//     loss/accuracy record and global_step += 1 of step t-1).
// lr = 0 / stats_on = 0 (the first step after a flush): a pure copy p_old -> p_new.
// Removes one dependent kernel boundary and one cold-load phase per step vs the 3-launch
// step (fwd / head / wgrad).
// XW > 0 (pipelined FUSED data-parallel engine, launched with KSX = KS3): each 16x16 local
// gradient slice (summed over the two K-split waves) is exchanged by its K-split-0 wave in LL
// words with the XW - 1 peers (xg_exchange, epoch slot bid * NCG + column group) and summed
// in rank order before the apply -- the all-reduce of the 3-launch fused engine,
// moved into the next step's first launch (2 launches per data-parallel step).
// TRACE (probe builds, tools/probes/mlp_pipelined_trace.py): per wave, s_memrealtime stamps
// 0 entry, 1 phase-A operands landed, 2 W1 tile applied (after the barrier), 3 slab stored;
// small-parameter blocks: 0 entry, 3 done.  tr: [blocks * 4 waves][4].
// KSX: K slices (blocks per hidden tile).  KS2 = 14 (56 features, 105 blocks: the factor
// engine's layout); KS3 = 28 for the single-GPU step and the fused engines: 203 blocks on the 256 CUs instead of
// 105, phase A's K (the batch) split over two waves per 16-column group (partials added
// through LDS) and phase B's z1 partial over 28 features -- per wave 14 + 8..16 f32 MFMAs
// instead of 28 + 16..32.  f32 MFMAs issue at 32 cycles each on one SIMD, so with one wave
// per SIMD the MFMA issue itself set the two phases' length (profiles/r3/mlp_trace/pmc.md:
// 41 % of the waves' cycles were issue stalls).
// FWD = false (mlp_apply_launch: the pending update of the last pipelined step, the flush):
// phase A and the small parameters only -- no forward, no x loads.
// (the body of block `bid`: mlp_fwdapply_kernel runs it with bid = blockIdx.x, the terminal
// head + apply kernel of a launched region with FWD = false on its apply blocks)
template <int NGT, int XW = 0, bool TRACE = false, bool TWO = false, int KSX = KS2, bool FWD = true>
__device__ __forceinline__ void fwdapply_block(
    const int bid, const float* __restrict__ p_old, float* __restrict__ p_new, float lr,
    const float* __restrict__ x_prev, const float* __restrict__ x, const Bufs& w,
    int* __restrict__ ctr, float* __restrict__ stats, int stats_ring, int B, int stats_on,
    const MlpXg& xg, unsigned long long* __restrict__ tr) {
  // stamps per wave: 0 entry, 1 phase-A operands landed, 2 W1 tile applied + barrier, 3 slab
  // stored; with XW > 0 also 4 local gradient slice ready (exchange starts), 5 two-shot: the
  // owned sums done (first hop), 6 exchange done -- 8 slots per wave then
  constexpr int TRN = XW > 0 ? 8 : 4;
  unsigned long long* trw = TRACE ? tr + (size_t)(bid * 4 + (threadIdx.x >> 6)) * TRN : nullptr;
  if (TRACE) trace_stamp(trw, 0);
  const int BP = NGT > 0 ? NGT * 16 : ((B + 15) >> 4) * 16;
  const int NG = NGT > 0 ? NGT : BP / 16;
  const int RT = (B + 15) >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  constexpr int MAXG = NGT > 0 ? NGT : MAXB / 16;
  constexpr int KWX = D / KSX;            // features per block
  constexpr int NCG = (KWX + 15) / 16;     // 16-column groups of the W1 tile (4 or 2)
  constexpr int KSP = 4 / NCG;             // phase-A K splits (waves per column group)
  constexpr int G2 = (KWX + 15) / 16;      // phase-B 16-feature groups
  static_assert(KSX * KWX == D && KWX % 4 == 0 && NCG * KSP == 4, "K slicing");
  if (bid >= HT * KSX) {
    const int jt = bid - HT * KSX;
    wgrad_small<true, NGT, XW>(jt, wave, lane, MLP_XG_SMALL_EPOCH + jt * 4 + wave, p_new, lr,
                               nullptr, w, ctr, stats, stats_ring, B, xg, p_old, stats_on);
    if (TRACE) trace_stamp(trw, 3);
    return;
  }
  constexpr int LW = KWX + 4;  // LDS row pitch (floats)
  __shared__ float Wt[16][LW];
  __shared__ float Kred[KSP > 1 ? NCG : 1][64][4];  // phase-A K-split partials
  const int jt = bid / KSX, ks = bid % KSX;
  const int f0 = ks * KWX;
  // phase B's x rows are independent of phase A: requested first, so the whole launch
  // makes one memory round trip (B <= 128 -> at most 2 row tiles per wave held here)
  constexpr int RTW = 2;
  float4 xa[RTW][G2];
  float rmv[RTW];
#pragma unroll
  for (int t = 0; t < (FWD ? RTW : 0); ++t) {
    const int row = (wave + 4 * t) * 16 + r;
    const float* xr = x + (size_t)(row < B ? row : B - 1) * D + f0;
    rmv[t] = row < B ? 1.f : 0.f;
#pragma unroll
    for (int g = 0; g < G2; ++g) {
      const int k = 16 * g + 4 * q;
      xa[t][g] = f4(xr + (k < KWX ? k : 0));
    }
  }

  // ---- phase A: this wave's 16 x 16 slice of the updated W1 tile (K split sp of KSP) -----
  {
    const int cgp = wave % NCG, sp = wave / NCG;
    const int fl = cgp * 16 + r;            // feature within the block's slice
    const bool cv = fl < KWX;               // (14 slices: wave 3 has 8 live columns)
    const int fc = f0 + (cv ? fl : KWX - 1);
    const float* a = w.dz1T + (size_t)(jt * 16 + r) * BP + q * 4;
    const float* xc = x_prev + fc;
    constexpr int GPS = (MAXG + KSP - 1) / KSP;  // batch groups per K split
    const int g0 = sp * GPS;
    float4 av[GPS];
    float xv[GPS][4];
    float pw[4] = {0.f, 0.f, 0.f, 0.f};
    // exchange-epoch slot of this 16 x 16 slice (the K split 0 wave exchanges the summed tile)
    const int eslot = bid * NCG + cgp;
    const unsigned ep = XW > 0 ? xg.epochs[eslot] + 1 : 0u;
#pragma unroll
    for (int gg = 0; gg < GPS; ++gg) {
      const int g = g0 + gg;
      if (g < NG) {
        av[gg] = f4(a + g * 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int b = g * 16 + q * 4 + e;  // rows >= B: dz1T is zero there
          xv[gg][e] = xc[(size_t)(b < B ? b : B - 1) * D];
        }
      }
    }
    // SPLITX (exchange engines, two K-split waves per column group): BOTH waves finish half of
    // the slice -- wave sp joins, exchanges and applies elements 2 sp, 2 sp + 1 of each lane --
    // so the exchange's uncached-memory transactions are spread over all 4 waves of the block
    // (the exchange bounds the phase at 4-8 ranks, tools/probes/engine_trace.py)
    const bool SPLITX = XW > 0 && KSP == 2 && (xg.split & 1);
    if (SPLITX || sp == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (SPLITX && (i >> 1) != sp) continue;
        const int j = jt * 16 + q * 4 + i;
        pw[i] = p_old[OFF_W1 + (size_t)(j < H ? j : H - 1) * D + fc];
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // all loads in flight together
    if (TRACE) trace_stamp(trw, 1);
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
    for (int gg = 0; gg < GPS; ++gg) {
      if (g0 + gg < NG) {
        acc0 = mfma16x16x4(av[gg].x, xv[gg][0], acc0);
        acc1 = mfma16x16x4(av[gg].y, xv[gg][1], acc1);
        acc0 = mfma16x16x4(av[gg].z, xv[gg][2], acc0);
        acc1 = mfma16x16x4(av[gg].w, xv[gg][3], acc1);
      }
    }
    float gv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) gv[i] = acc0[i] + acc1[i];
    if (SPLITX) {  // hand the other wave its half: element i goes to wave i / 2
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((i >> 1) != sp) Kred[cgp][lane][i] = gv[i];
      __syncthreads();
      // split 0 + split 1 either way (IEEE addition commutes: the same bits on every rank)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if ((i >> 1) == sp) gv[i] += Kred[cgp][lane][i];
    } else if constexpr (KSP > 1) {  // the later K split's partial joins split 0 (fixed order)
      if (sp > 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) Kred[cgp][lane][i] = gv[i];
      __syncthreads();
      if (sp == 0)
#pragma unroll
        for (int i = 0; i < 4; ++i) gv[i] += Kred[cgp][lane][i];
    }
    bool fail = false;
    if constexpr (XW > 0) {
    if (SPLITX) {
      size_t offw[2];
      bool okw[2];
      float g2[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int i = 2 * sp + e;
        const int j = jt * 16 + q * 4 + i;
        okw[e] = cv && j < H;
        offw[e] = OFF_W1 + (size_t)(j < H ? j : 0) * D + fc;
        g2[e] = sp == 0 ? gv[e] : gv[2 + e];
      }
      if (TRACE) trace_stamp(trw, 4);
      // the pair's two hidden rows j, j + 1 (j even, H even: both live or both padding)
      const bool plive = cv && jt * 16 + q * 4 + 2 * sp < H;
      if constexpr (TWO) {
        if (xg.split & 4)  // (DTFX_XG_SPLIT bit 2: the round-4 per-element owners, A/B runs)
          xg_exchange2<XW, 2>(xg, ep, offw, okw, g2, fail, lane, TRACE ? trw : nullptr, 2 * sp);
        else if (xg.split & 16)
          xg_exchange2p<XW, true>(xg, ep, XG_W1_BASE + ((long long)(eslot * 2 + sp) * 64 + lane) * 2,
                                  g2, fail, lane, sp, TRACE ? trw : nullptr, plive);
        else
          xg_exchange2p<XW>(xg, ep, XG_W1_BASE + ((long long)(eslot * 2 + sp) * 64 + lane) * 2,
                            g2, fail, lane, sp, TRACE ? trw : nullptr, plive);
      } else if (xg.split & 16)
        xg_exchange16<XW, true>(xg, ep, XG_W1_BASE + ((long long)(eslot * 2 + sp) * 64 + lane) * 2,
                                g2, fail, plive);
      else
        xg_exchange16<XW>(xg, ep, XG_W1_BASE + ((long long)(eslot * 2 + sp) * 64 + lane) * 2,
                          g2, fail, plive);
      if (TRACE) trace_stamp(trw, 6);
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int i = 2 * sp + e;
        const int hl = q * 4 + i, j = jt * 16 + hl;
        const float pv = sp == 0 ? pw[e] : pw[2 + e];
        const float v = fail ? pv : pv - lr * g2[e];  // timed out: keep W1 (err raised)
        if (cv) {
          if (FWD) Wt[hl][fl] = j < H ? v : 0.f;  // padded hidden rows contribute exact zeros
          if (j < H) p_new[OFF_W1 + (size_t)j * D + f0 + fl] = v;
        }
      }
      if (sp == 0 && lane == 0) xg.epochs[eslot] = ep;
      if (fail) atomicExch(xg.err, 1);
    } else if (sp == 0) {
      size_t offw[4];
      bool okw[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j = jt * 16 + q * 4 + i;
        okw[i] = cv && j < H;
        offw[i] = OFF_W1 + (size_t)(j < H ? j : 0) * D + fc;
      }
      if (TRACE) trace_stamp(trw, 4);
      if constexpr (TWO) xg_exchange2<XW>(xg, ep, offw, okw, gv, fail, lane, TRACE ? trw : nullptr);
      else xg_exchange<XW>(xg, ep, offw, okw, gv, fail);
      if (TRACE) trace_stamp(trw, 6);
    }
    }  // XW > 0
    if (!SPLITX && sp == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hl = q * 4 + i, j = jt * 16 + hl;
        const float v = fail ? pw[i] : pw[i] - lr * gv[i];  // timed out: keep W1 (err raised)
        if (cv) {
          if (FWD) Wt[hl][fl] = j < H ? v : 0.f;  // padded hidden rows contribute exact zeros
          if (j < H) p_new[OFF_W1 + (size_t)j * D + f0 + fl] = v;
        }
      }
    }
    if (XW > 0 && !SPLITX && sp == 0) {
      if (lane == 0) xg.epochs[eslot] = ep;
      if (fail) atomicExch(xg.err, 1);
    }
  }
  if constexpr (!FWD) return;
  __syncthreads();
  if (TRACE) trace_stamp(trw, 2);

  // ---- phase B: z1 partial over the block's KWX features, row tiles rt = wave, wave + 4,
  // ..  lane (r, q): A = x[rt*16 + r][f0 + 16g + 4q + e], B = Wt[r][16g + 4q + e]; the last
  // group is partly live (14 slices: 8 features, q < 2; 28 slices: 12, q < 3)
  float4 wb[G2];
#pragma unroll
  for (int g = 0; g < G2; ++g) {
    const int k = 16 * g + 4 * q;
    wb[g] = k < KWX ? *reinterpret_cast<const float4*>(&Wt[r][k]) : float4{0.f, 0.f, 0.f, 0.f};
  }
  for (int rt = wave, t = 0; rt < RT; rt += 4, ++t) {
    float4 xg[G2];
    float rm;
    if (t < RTW) {  // prefetched (wave-uniform)
#pragma unroll
      for (int g = 0; g < G2; ++g) xg[g] = t == 0 ? xa[0][g] : xa[1][g];
      rm = t == 0 ? rmv[0] : rmv[1];
    } else {        // B > 128: later row tiles load here
      const int row = rt * 16 + r;
      const float* xr = x + (size_t)(row < B ? row : B - 1) * D + f0;
      rm = row < B ? 1.f : 0.f;
#pragma unroll
      for (int g = 0; g < G2; ++g) {
        const int k = 16 * g + 4 * q;
        xg[g] = f4(xr + (k < KWX ? k : 0));
      }
    }
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < G2; ++g) {
      // (wb is zero for the dead part of the last group, so no mask is needed on xg there)
      acc0 = mfma16x16x4(xg[g].x * rm, wb[g].x, acc0);
      acc1 = mfma16x16x4(xg[g].y * rm, wb[g].y, acc1);
      acc0 = mfma16x16x4(xg[g].z * rm, wb[g].z, acc0);
      acc1 = mfma16x16x4(xg[g].w * rm, wb[g].w, acc1);
    }
    float* out = w.slab + ((size_t)ks * BP + rt * 16 + q * 4) * HP + jt * 16 + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) out[(size_t)i * HP] = acc0[i] + acc1[i];
  }
  if (TRACE) trace_stamp(trw, 3);
}

template <int NGT, int XW = 0, bool TRACE = false, bool TWO = false, int KSX = KS2, bool FWD = true>
__global__ __launch_bounds__(256) void mlp_fwdapply_kernel(
    const float* __restrict__ p_old, float* __restrict__ p_new, float lr,
    const float* __restrict__ x_prev, const float* __restrict__ x, Bufs w, int* __restrict__ ctr,
    float* __restrict__ stats, int stats_ring, int B, int stats_on, MlpXg xg,
    unsigned long long* __restrict__ tr = nullptr) {
  fwdapply_block<NGT, XW, TRACE, TWO, KSX, FWD>(blockIdx.x, p_old, p_new, lr, x_prev, x, w, ctr,
                                                stats, stats_ring, B, stats_on, xg, tr);
}

// Terminal step of a launched region with the flush folded in (opt-in,
// measured slower: see mlp_flush_fused): the head of
// the region's last step AND the apply of that step's update -- what mlp_head_kernel + the
// apply-only mlp_fwdapply_kernel<.., FWD = false> (mlp_apply_launch) do as two dependent
// launches -- in ONE launch, so the region ends on the step's own second launch.
//   blocks [0, NHB): head rows 4 * bid + wave (one wave per batch row, as mlp_head_kernel);
//     each row's wave publishes with ONE agent-scope release add on sync[0] (its stores to
//     hbuf / dz1T / dlT / rowstat retired and written back first).
//   blocks [NHB, NHB + HT * KSX + HT): apply blocks: thread 0 waits (agent-scope acquire)
//     until sync[0] == B, then the block runs the apply-only body on the step's parameters
//     p_cur -> p_next (the same code, operands and summation order as the flush launch: the
//     result is bit-identical).
// Every wait is bounded (`ticks` of s_memrealtime): a timed-out block sets sync[2] and skips
// its apply (the host raises: FusedMLPTrainer.check()).  The grid (25 + 203 blocks of 256
// threads at batch 100) is a fraction of one wave slot per CU, so every head block is resident
// while the apply blocks wait.  The last apply block to finish zeroes sync[0..1] for the next
// region (stream order: no launch reads them before this one has ended).
template <int NGT, int KSX>
__global__ __launch_bounds__(256) void mlp_head_flush_kernel(
    const float* __restrict__ p_cur, float* __restrict__ p_next, float lr,
    const float* __restrict__ x, const int* __restrict__ labels, Bufs w, int* __restrict__ ctr,
    float* __restrict__ stats, int stats_ring, int B, long long ticks) {
  const int nhb = (B + 3) >> 2;
  const int bid = blockIdx.x, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (bid < nhb) {
    const int row = bid * 4 + wave;
    if (row >= B) return;
    head_row<false, false, 0, KSX>(row, lane, p_cur, p_cur, 0.f, nullptr, labels, w, B, nullptr,
                                   MlpXg{}, nullptr);
    // release at agent scope: the wave's stores are complete and written back past this
    // XCD's L2 before the count moves (one add per row)
    if (lane == 0) __hip_atomic_fetch_add(w.sync, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  __shared__ int ok_s;
  if (threadIdx.x == 0) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    int ok = 1;
    while (__hip_atomic_load(w.sync, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < B) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks ||
          __hip_atomic_load(w.sync + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        ok = 0;
        __hip_atomic_store(w.sync + 2, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    ok_s = ok;
  }
  __syncthreads();
  if (ok_s)
    fwdapply_block<NGT, 0, false, false, KSX, false>(bid - nhb, p_cur, p_next, lr, x, x, w, ctr,
                                                     stats, stats_ring, B, 1, MlpXg{}, nullptr);
  __syncthreads();
  if (threadIdx.x == 0) {
    const int napply = (int)gridDim.x - nhb;
    if (__hip_atomic_fetch_add(w.sync + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == napply - 1) {
      __hip_atomic_store(w.sync, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(w.sync + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}


// ---------------------------------------------------------------------------
// Pipelined FACTOR engine (world XW, 2 launches per data-parallel step): the
// mlp_fwdapply_kernel structure with the W1 update formed from EVERY rank's factors:
//   g = sum_q dz1A[q][jt]^T . x_q(t-1)   (K = XW * BP, the all-gathered factors of step
//   t-1 and every rank's resident batch), W1new = W1old - lr * g,
// then step t's forward on W1new.  The single-GPU step's 28-feature K slices (196 W1
// blocks): 1024-thread blocks, wave (c, s) owns column group c (16 + 12 live features) and
// K split s of fx_kspl = 8 (generic batches: 512 threads, 4 splits); the partial slices are
// added in split order through LDS
// (identical order on every rank: bit-identical replicas).  At 8 ranks the global W1 gradient
// is 8 x the 1-GPU step's MFMA work (K = 800), so it must be spread over the chip and issue
// all of its loads in ONE round trip: a wave's K share (XW * 7 / 8 batch groups of 16 rows, 7
// at 8 ranks) is requested at once (CH groups per round), and the seven hidden tiles of a K slice
// -- which read the same x columns of every rank's batch, the one large fresh read -- run on
// one XCD (block b on XCD b % 8; speed only), so each XCD's L2 fetches its slices' x once.
// The first version (14 slices, 98 blocks, 4 load rounds, slices scattered over the XCDs)
// cost 21.2 us per step at 8 ranks against 7.3 for the 1-GPU step (round-4 local cost).
// Measured and not kept (round 5): the block's x slab of all ranks staged in LDS with 16-byte
// loads instead of per-lane 4-byte gathers (first launch + plain head 10.9-11.1 -> 11.8-12.1
// us at 8 ranks: the staging round trip then sits in front of every MFMA).
// Small-parameter blocks exchange dW2/db1/db2 partials of step t-1 as in the 3-launch factor
// engine (waves 0..3 of the block).  The head of step t all-gathers dz1 into dz1A
// (mlp_head_kernel<.., XW, KS3>).
constexpr int FX_SLOTS = (KS3 + 7) / 8 * HT;  // block slots per XCD (4 slice rows x 7 tiles)
// phase-A K splits: 8 (1024-thread blocks, 16 waves, 4 per SIMD) for the batch <= 112
// instantiations; the generic ones keep 4 (512 threads: their small-parameter waves hold
// 16 batch groups of operands, which 4 waves per SIMD would spill)
template <int NGT> constexpr int fx_kspl() { return NGT > 0 ? 8 : 4; }
// Phase A of mlp_fwdapply_factor_kernel in row-quad form (DTFX_XG_SPLIT bit 5, round 6): each
// of the block's 16 waves covers ALL 28 features of the slice for its 1/16 of the K = XW x BP
// rows.  Per quad of 4 rows a lane loads ONE float2 of x (features 2r, 2r + 1 of row base + q;
// lanes r >= 14 are dead) and ONE dz1A value (hidden r of row base + q), and feeds two
// 16x16x4 MFMAs (accumulator e: features 2r + e).  The column-group form loads four scalar x
// and four dz1A values per 16 rows and column group -- twice the load instructions per
// element, the one cost that grows with K = XW x BP (the global W1 gradient is 8x the 1-GPU
// step's MFMA work at 8 ranks).  The 16 partials are added in split order (the same bits on
// every rank); wave e in {0, 1} applies accumulator e.
template <int XW, int NGT>
__device__ __forceinline__ void fx_phase_a_quads(
    const float* __restrict__ p_old, float* __restrict__ p_new, float lr,
    const float* __restrict__ x_prev, long long xstride, const float* __restrict__ dz1A, int B,
    int BP, int jt, int f0, int me, int wave, int lane, float (&Wt)[16][D / KS3 + 4],
    f32x4* red) {
  constexpr int KWX = D / KS3;         // 28 features
  constexpr int NQ = NGT * 4;          // row quads per rank
  constexpr int GQ = XW * NQ;          // row quads in all
  constexpr int QPW = (GQ + 15) / 16;  // per wave (14 at 8 ranks x 112 rows)
  const int r = lane & 15, q = lane >> 4;
  const bool lv = r < KWX / 2;
  const int fo = 2 * (lv ? r : KWX / 2 - 1);
  float pw[4];
  if (wave < 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = jt * 16 + q * 4 + i;
      pw[i] = p_old[OFF_W1 + (size_t)(j < H ? j : H - 1) * D + f0 + fo + wave];
    }
  }
  float av[QPW];
  float2 xv[QPW];
  const int u0 = wave * QPW;
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    const int g = u0 + u;
    if (g < GQ) {  // wave-uniform
      const int qq = g / NQ, row = (g - qq * NQ) * 4 + q;
      av[u] = dz1A[((size_t)qq * BP + row) * HP + jt * 16 + r];  // rows >= B: zero
      xv[u] = *reinterpret_cast<const float2*>(
          x_prev + (long long)(qq - me) * xstride + (size_t)(row < B ? row : B - 1) * D + f0 + fo);
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // the wave's loads in flight together
  f32x4 a0 = {0, 0, 0, 0}, a1 = {0, 0, 0, 0};
#pragma unroll
  for (int u = 0; u < QPW; ++u) {
    if (u0 + u < GQ) {
      a0 = mfma16x16x4(av[u], xv[u].x, a0);
      a1 = mfma16x16x4(av[u], xv[u].y, a1);
    }
  }
  red[(wave * 2 + 0) * 64 + lane] = a0;
  red[(wave * 2 + 1) * 64 + lane] = a1;
  __syncthreads();
  if (wave < 2) {
    f32x4 part = red[wave * 64 + lane];
#pragma unroll
    for (int k = 1; k < 16; ++k) {  // split order: the same bits on every rank
      const f32x4 o = red[(k * 2 + wave) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; ++i) part[i] += o[i];
    }
    const int fl = fo + wave;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hl = q * 4 + i, j = jt * 16 + hl;
      const float v = pw[i] - lr * part[i];
      if (lv) {
        Wt[hl][fl] = j < H ? v : 0.f;
        if (j < H) p_new[OFF_W1 + (size_t)j * D + f0 + fl] = v;
      }
    }
  }
}

template <int XW, int NGT>
__global__ __launch_bounds__(128 * fx_kspl<NGT>()) void mlp_fwdapply_factor_kernel(
    const float* __restrict__ p_old, float* __restrict__ p_new, float lr,
    const float* __restrict__ x_prev, const float* __restrict__ x, long long xstride,
    const float* __restrict__ dz1A, Bufs w, int* __restrict__ ctr, float* __restrict__ stats,
    int stats_ring, int B, int stats_on, MlpXg xg) {
  constexpr int FX_KSPL = fx_kspl<NGT>();
  const int BP = NGT > 0 ? NGT * 16 : ((B + 15) >> 4) * 16;
  const int NG = NGT > 0 ? NGT : BP / 16;
  const int RT = (B + 15) >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, q = lane >> 4;
  const int bid = blockIdx.x;
  if (bid >= 8 * FX_SLOTS) {
    const int jt = bid - 8 * FX_SLOTS;
    if (wave < 4)
      wgrad_small<true, NGT, XW>(jt, wave, lane, MLP_XG_SMALL_EPOCH + jt * 4 + wave, p_new, lr,
                                 nullptr, w, ctr, stats, stats_ring, B, xg, p_old, stats_on);
    return;
  }
  // block -> (hidden tile jt, K slice ks) with ks % 8 == the block's XCD
  const int xcd = bid & 7, s8 = bid >> 3;
  const int jt = s8 % HT, ks = (s8 / HT) * 8 + xcd;
  if (ks >= KS3) return;  // (whole block: the slots past the 28 slices)
  constexpr int KWX = D / KS3;  // 28 features
  constexpr int LW = KWX + 4;
  __shared__ float Wt[16][LW];
  // K-split partials: [c][k][lane] (column-group form) or [s][e][lane] (row-quad form)
  __shared__ f32x4 red[32 * 64];
  const int f0 = ks * KWX;
  const int me = xgll::uniform(xg.rank);
  // phase B's x rows (wave w < RT owns row tile w; B <= 128): requested first
  float4 xa[2];
  const int rowB = wave * 16 + r;
  const float rmB = rowB < B ? 1.f : 0.f;
  if (wave < RT) {
    const float* xr = x + (size_t)(rowB < B ? rowB : B - 1) * D + f0;
#pragma unroll
    for (int g = 0; g < 2; ++g) {
      const int k = 16 * g + 4 * q;
      xa[g] = f4(xr + (k < KWX ? k : 0));
    }
  }
  if (NGT > 0 && (xg.split & 32)) {
    if constexpr (NGT > 0)
      fx_phase_a_quads<XW, NGT>(p_old, p_new, lr, x_prev, xstride, dz1A, B, BP, jt, f0, me,
                                wave, lane, Wt, red);
  } else {
  // ---- phase A: column group c, K split sp (FX_KSPL splits) ------------------------------
  const int c = wave & 1, sp = wave >> 1;
  const int fl = c * 16 + r;
  const bool cv = fl < KWX;
  const int fc = f0 + (cv ? fl : KWX - 1);
  const int G = XW * NG, per = (G + FX_KSPL - 1) / FX_KSPL;
  const int g0 = sp * per, g1 = min(G, g0 + per);
  float pw[4];
  if (sp == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = jt * 16 + q * 4 + i;
      pw[i] = p_old[OFF_W1 + (size_t)(j < H ? j : H - 1) * D + fc];
    }
  }
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
  // one round at 8 ranks x 7 groups (7 per split); more only for batches > 112 rows
  constexpr int CH = (XW * (NGT > 0 ? NGT : 7) + FX_KSPL - 1) / FX_KSPL;
  for (int c0 = g0; c0 < g1; c0 += CH) {
    float4 av[CH];
    float xv[CH][4];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int g = c0 + i;
      if (g < g1) {  // wave-uniform
        const int qq = g / NG, gg = g - qq * NG;
        const float* a = dz1A + ((size_t)qq * BP + gg * 16 + q * 4) * HP + jt * 16 + r;
        av[i] = make_float4(a[0], a[HP], a[2 * HP], a[3 * HP]);
        const float* xq = x_prev + (long long)(qq - me) * xstride + fc;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int b = gg * 16 + q * 4 + e;  // rows >= B: dz1A is zero there
          xv[i][e] = xq[(size_t)(b < B ? b : B - 1) * D];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // the round's loads in flight together
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (c0 + i < g1) {
        acc0 = mfma16x16x4(av[i].x, xv[i][0], acc0);
        acc1 = mfma16x16x4(av[i].y, xv[i][1], acc1);
        acc0 = mfma16x16x4(av[i].z, xv[i][2], acc0);
        acc1 = mfma16x16x4(av[i].w, xv[i][3], acc1);
      }
    }
  }
  f32x4 part;
#pragma unroll
  for (int i = 0; i < 4; ++i) part[i] = acc0[i] + acc1[i];
  if (sp > 0) red[(c * (FX_KSPL - 1) + sp - 1) * 64 + lane] = part;
  __syncthreads();
  if (sp == 0) {
#pragma unroll
    for (int k = 0; k < FX_KSPL - 1; ++k) {  // split order: the same bits on every rank
      const f32x4 o = red[(c * (FX_KSPL - 1) + k) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; ++i) part[i] += o[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hl = q * 4 + i, j = jt * 16 + hl;
      const float v = pw[i] - lr * part[i];
      if (cv) {
        Wt[hl][fl] = j < H ? v : 0.f;
        if (j < H) p_new[OFF_W1 + (size_t)j * D + f0 + fl] = v;
      }
    }
  }
  }
  __syncthreads();
  // ---- phase B: z1 partial of row tile `wave` over the block's 28 features -------------
  if (wave >= RT) return;
  float4 wb[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int k = 16 * g + 4 * q;
    wb[g] = k < KWX ? *reinterpret_cast<const float4*>(&Wt[r][k]) : float4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 o0 = {0, 0, 0, 0}, o1 = {0, 0, 0, 0};
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    // (wb is zero for the dead part of the last group, so no mask is needed on xa there)
    o0 = mfma16x16x4(xa[g].x * rmB, wb[g].x, o0);
    o1 = mfma16x16x4(xa[g].y * rmB, wb[g].y, o1);
    o0 = mfma16x16x4(xa[g].z * rmB, wb[g].z, o0);
    o1 = mfma16x16x4(xa[g].w * rmB, wb[g].w, o1);
  }
  float* out = w.slab + ((size_t)ks * BP + wave * 16 + q * 4) * HP + jt * 16 + r;
#pragma unroll
  for (int i = 0; i < 4; ++i) out[(size_t)i * HP] = o0[i] + o1[i];
}

// ---------------------------------------------------------------------------
// K3, factor engine (sufficient-factor exchange, world XW): the backprop factors dz1 of
// every rank were all-gathered by mlp_head_kernel<.., XW> into dz1A [XW][BP][HP], and every
// rank holds every rank's (deterministic, device-resident) batch, so each rank computes the
// GLOBAL dW1^T = sum_q dz1_q^T . x_q itself (K = XW * BP) and applies it -- the 313 KB W1
// gradient never crosses xGMI; only the 1,110 small-parameter gradients are exchanged
// (wgrad_small, LL push).  Identical inputs + a fixed summation order keep the replicas
// bit-identical.
//   blocks [0, 8 * FT): one 16x16 dW1^T tile per block, the K range split over 4 waves and
//     the 4 partial tiles added in wave order through LDS.  Block b runs on XCD b % 8
//     (round-robin dispatch; speed only): feature tile kt = 8 * s + b % 8 keeps each
//     XCD's x columns to ~1/8 of every rank's batch (x is the one large fresh read).
//   blocks [8 * FT, 8 * FT + HT): wgrad_small (dW2 / db1 / db2 partials exchanged).
// xstride: elements between consecutive ranks' datasets (x of rank q = x + (q - me) * xstride).
template <int XW, int NGT>
__global__ __launch_bounds__(256) void mlp_wgrad_factor_kernel(
    float* __restrict__ p, float lr, const float* __restrict__ x, long long xstride,
    const float* __restrict__ dz1A, Bufs w, int* __restrict__ ctr, float* __restrict__ stats,
    int stats_ring, int B, MlpXg xg) {
  const int BP = NGT > 0 ? NGT * 16 : ((B + 15) >> 4) * 16;
  const int NG = NGT > 0 ? NGT : BP / 16;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, r = lane & 15, q4 = lane >> 4;
  const int bid = blockIdx.x;
  constexpr int NSLOT = (FT + 7) / 8;  // 7 feature-tile slots per XCD
  if (bid >= 8 * HT * NSLOT) {
    const int jt = bid - 8 * HT * NSLOT;
    wgrad_small<true, NGT, XW>(jt, wave, lane, MLP_XG_SMALL_EPOCH + jt * 4 + wave, p, lr,
                               nullptr, w, ctr, stats, stats_ring, B, xg);
    return;
  }
  const int xcd = bid & 7, s = bid >> 3;
  const int jt = s / NSLOT, kt = (s % NSLOT) * 8 + xcd;
  if (kt >= FT) return;  // whole block: uniform
  __shared__ f32x4 red[3][64];
  const int G = XW * NG, per = (G + 3) / 4;
  const int g0 = wave * per, g1 = min(G, g0 + per);
  const int me = xgll::uniform(xg.rank);
  float pw[4];
  if (wave == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = jt * 16 + q4 * 4 + i;
      pw[i] = p[OFF_W1 + (size_t)(j < H ? j : H - 1) * D + kt * 16 + r];
    }
  }
  f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
  constexpr int CH = 7;  // groups of 16 batch rows per load round (all in flight together)
  for (int c0 = g0; c0 < g1; c0 += CH) {
    float4 av[CH];
    float xv[CH][4];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int g = c0 + i;
      if (g < g1) {  // wave-uniform
        const int qq = g / NG, gg = g - qq * NG;
        const float* a = dz1A + ((size_t)qq * BP + gg * 16 + q4 * 4) * HP + jt * 16 + r;
        av[i] = make_float4(a[0], a[HP], a[2 * HP], a[3 * HP]);
        const float* xq = x + (long long)(qq - me) * xstride + kt * 16 + r;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int b = gg * 16 + q4 * 4 + e;  // rows >= B: dz1A is zero there
          xv[i][e] = xq[(size_t)(b < B ? b : B - 1) * D];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // the round's loads in flight together
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (c0 + i < g1) {
        acc0 = mfma16x16x4(av[i].x, xv[i][0], acc0);
        acc1 = mfma16x16x4(av[i].y, xv[i][1], acc1);
        acc0 = mfma16x16x4(av[i].z, xv[i][2], acc0);
        acc1 = mfma16x16x4(av[i].w, xv[i][3], acc1);
      }
    }
  }
  f32x4 part;
#pragma unroll
  for (int i = 0; i < 4; ++i) part[i] = acc0[i] + acc1[i];
  if (wave > 0) red[wave - 1][lane] = part;
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const f32x4 o = red[k][lane];
#pragma unroll
    for (int i = 0; i < 4; ++i) part[i] += o[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int j = jt * 16 + q4 * 4 + i;
    if (j < H) p[OFF_W1 + (size_t)j * D + kt * 16 + r] = pw[i] - lr * part[i];
  }
}

}  // namespace mlp

// ---------------------------------------------------------------------------
// host launchers
// ---------------------------------------------------------------------------
static mlp::Bufs make_bufs(float* ws, int B) {
  using namespace mlp;
  const int BP = ((B + 15) / 16) * 16;
  Bufs b;
  b.slab = ws;
  b.hbuf = b.slab + (size_t)NSLAB_MAX * BP * HP;
  b.dz1T = b.hbuf + (size_t)BP * HP;
  b.dlT = b.dz1T + (size_t)HP * BP;
  b.rowstat = b.dlT + (size_t)16 * BP;
  b.sync = reinterpret_cast<int*>(b.rowstat + (size_t)2 * BP);
  return b;
}

// TF checkpoint layout <-> the kernels' flat layout of the MLP parameters / gradients (the
// async-PS wire format is TF's: worker.py:27-31 kernels [in, out]).  The four segments sit at
// the same offsets in both (78400 | 100 | 1000 | 10); only the kernels are transposed.
// to_tf = 1: flat -> TF (+ `extra` floats copied from `xsrc` after NPARAM: the step's loss /
// accuracy record rides along in the same D2H copy); 0: TF -> flat.
__global__ __launch_bounds__(256) void mlp_tf_layout_kernel(const float* __restrict__ src,
                                                            float* __restrict__ dst, int to_tf,
                                                            const float* __restrict__ xsrc,
                                                            int extra) {
  using namespace mlp;
  const int i = blockIdx.x * 256 + threadIdx.x;  // destination index
  if (i < NPARAM) {
    int j = i;  // source index
    if (i < OFF_B1) {  // W1: TF [784][100] <-> flat [100][784]
      j = to_tf ? (i % H) * D + i / H : (i % D) * H + i / D;
    } else if (i >= OFF_W2 && i < OFF_B2) {  // W2: TF [100][10] <-> flat [10][100]
      const int k = i - OFF_W2;
      j = OFF_W2 + (to_tf ? (k % C) * H + k / C : (k % H) * C + k / H);
    }
    dst[i] = src[j];
  } else if (to_tf && i < NPARAM + extra) {
    dst[i] = xsrc[i - NPARAM];
  }
}

// TF layout -> flat layout iterating over the SOURCE (TF) index: consecutive threads read
// consecutive words (the source may be host memory read over the host link, where the
// destination-major walk of mlp_tf_layout_kernel would issue 4-byte reads 400 bytes apart)
// and scatter into device memory.
__global__ __launch_bounds__(256) void mlp_from_tf_src_major_kernel(const float* __restrict__ src,
                                                                    float* __restrict__ dst) {
  using namespace mlp;
  const int k = blockIdx.x * 256 + threadIdx.x;  // source (TF) index
  if (k >= NPARAM) return;
  int i = k;  // destination (flat) index
  if (k < OFF_B1) {  // TF W1 [784][100] -> flat W1t [100][784]
    i = (k % H) * D + k / H;
  } else if (k >= OFF_W2 && k < OFF_B2) {  // TF W2 [100][10] -> flat W2t [10][100]
    const int m = k - OFF_W2;
    i = OFF_W2 + (m % C) * H + m / C;
  }
  dst[i] = src[k];
}

void mlp_tf_layout_launch(const float* src, float* dst, int to_tf, const float* xsrc, int extra,
                          hipStream_t stream) {
  using namespace mlp;
  if (extra < 0 || extra > 64 || (extra && !xsrc))
    throw std::runtime_error("mlp_tf_layout: 0..64 extra floats with a source");
  const int n = NPARAM + (to_tf ? extra : 0);
  hipLaunchKernelGGL(mlp_tf_layout_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, src, dst,
                     to_tf, xsrc, to_tf ? extra : 0);
  DTFX_HIP_CHECK(hipGetLastError());
}

long long mlp_workspace_floats(int B) {
  using namespace mlp;
  const long long BP = ((B + 15) / 16) * 16;
  return (long long)NSLAB_MAX * BP * HP + BP * HP + HP * BP + 16 * BP + 2 * BP + 4;
}

static void check_b(int B) {
  if (B < 1 || B > mlp::MAXB) throw std::runtime_error("fused MLP step: batch must be in [1, 256]");
}

// K1: grad != nullptr => deferred apply (p_new must differ from p_old)
void mlp_fwd_launch(const float* p_old, const float* grad, float lr, float* p_new, const float* x,
                    float* ws, int B, hipStream_t stream, unsigned long long* tr) {
  using namespace mlp;
  check_b(B);
  const Bufs w = make_bufs(ws, B);
  const int RT = (B + 15) / 16;
  dim3 grid(RT * HT * KS), block(64);
  if (grad) {
    if (!p_new || p_new == p_old) throw std::runtime_error("mlp_fwd: apply needs ping-pong p_new");
    hipLaunchKernelGGL((mlp_fwd_kernel<true, false>), grid, block, 0, stream, p_old, grad, lr,
                       p_new, x, w, B, tr);
  } else if (tr) {
    hipLaunchKernelGGL((mlp_fwd_kernel<false, true>), grid, block, 0, stream, p_old, p_old, 0.f,
                       nullptr, x, w, B, tr);
  } else {
    hipLaunchKernelGGL((mlp_fwd_kernel<false, false>), grid, block, 0, stream, p_old, p_old, 0.f,
                       nullptr, x, w, B, tr);
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

void mlp_head_launch(const float* p_old, const float* grad, float lr, float* p_new,
                     const int* labels, float* ws, int B, hipStream_t stream,
                     unsigned long long* tr) {
  using namespace mlp;
  check_b(B);
  const Bufs w = make_bufs(ws, B);
  if (grad) {
    if (!p_new || p_new == p_old) throw std::runtime_error("mlp_head: apply needs ping-pong p_new");
    hipLaunchKernelGGL((mlp_head_kernel<true, false>), dim3(B), dim3(64), 0, stream, p_old, grad,
                       lr, p_new, labels, w, B, tr, MlpXg{}, nullptr);
  } else if (tr) {
    hipLaunchKernelGGL((mlp_head_kernel<false, true>), dim3(B), dim3(64), 0, stream, p_old, p_old,
                       0.f, nullptr, labels, w, B, tr, MlpXg{}, nullptr);
  } else {
    hipLaunchKernelGGL((mlp_head_kernel<false, false>), dim3(B), dim3(64), 0, stream, p_old, p_old,
                       0.f, nullptr, labels, w, B, tr, MlpXg{}, nullptr);
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

// K3: grad == nullptr => direct mode (p -= lr * g fused); else writes grad
void mlp_wgrad_launch(float* p, float lr, float* grad, const float* x, float* ws, int* ctr,
                      float* stats, int stats_ring, int B, hipStream_t stream,
                      unsigned long long* tr) {
  using namespace mlp;
  check_b(B);
  if (stats && stats_ring < 1) throw std::runtime_error("mlp_wgrad: stats_ring < 1");
  if (!ctr) throw std::runtime_error("mlp_wgrad: needs the global_step counter");
  const Bufs w = make_bufs(ws, B);
  dim3 grid(HT * ((FT + 3) / 4) + HT), block(256);
  const int NG = (B + 15) / 16;
  if (!grad && !p) throw std::runtime_error("mlp_wgrad: direct mode needs parameters");
  const MlpXg noxg{};
#define DTFX_WG(DIR, TR, NGT)                                                                 \
  hipLaunchKernelGGL((mlp_wgrad_kernel<DIR, TR, NGT>), grid, block, 0, stream, p,          \
                     DIR ? lr : 0.f, DIR ? nullptr : grad, x, w, ctr, stats, stats_ring, B, tr, \
                     noxg)
  if (grad) {
    if (NG == 7) DTFX_WG(false, false, 7);
    else DTFX_WG(false, false, 0);
  } else if (tr) {
    if (NG == 7) DTFX_WG(true, true, 7);
    else DTFX_WG(true, true, 0);
  } else {
    if (NG == 7) DTFX_WG(true, false, 7);
    else DTFX_WG(true, false, 0);
  }
#undef DTFX_WG
  DTFX_HIP_CHECK(hipGetLastError());
}

// K3 with the fused xGMI gradient exchange (direct apply with lr = lr / world).
void mlp_wgrad_xg_launch(float* p, float lr, const float* x, float* ws, int* ctr, float* stats,
                         int stats_ring, int B, hipStream_t stream, const MlpXg& xg, int world) {
  using namespace mlp;
  check_b(B);
  if (stats && stats_ring < 1) throw std::runtime_error("mlp_wgrad: stats_ring < 1");
  if (!ctr || !p) throw std::runtime_error("mlp_wgrad_xg: needs parameters and the step counter");
  if (xg.S < NPARAM) throw std::runtime_error("mlp_wgrad_xg: exchange slots smaller than the model");
  const Bufs w = make_bufs(ws, B);
  const int nblk = HT * ((FT + 3) / 4) + HT;
  if (nblk * 4 > MLP_XG_EPOCHS) throw std::runtime_error("mlp_wgrad_xg: epoch array too small");
  dim3 grid(nblk), block(256);
  const int NG = (B + 15) / 16;
#define DTFX_WGX(WW, NGT)                                                                    \
  hipLaunchKernelGGL((mlp_wgrad_kernel<true, false, NGT, WW>), grid, block, 0, stream, p, lr, \
                     nullptr, x, w, ctr, stats, stats_ring, B, nullptr, xg)
#define DTFX_WGW(WW)             \
  case WW:                       \
    if (NG == 7) DTFX_WGX(WW, 7); \
    else DTFX_WGX(WW, 0);        \
    break;
  switch (world) {
    DTFX_WGW(2) DTFX_WGW(3) DTFX_WGW(4) DTFX_WGW(5) DTFX_WGW(6) DTFX_WGW(7) DTFX_WGW(8)
    default:
      throw std::runtime_error("mlp_wgrad_xg: world must be 2..8");
  }
#undef DTFX_WGW
#undef DTFX_WGX
  DTFX_HIP_CHECK(hipGetLastError());
}


// Factor engine launches (see mlp_wgrad_factor_kernel).
void mlp_head_xg_launch(const float* p, const int* labels, float* ws, float* dz1A, int B,
                        hipStream_t stream, const MlpXg& xg, int world, int nslab) {
  using namespace mlp;
  check_b(B);
  if (nslab != KS && nslab != KS3) throw std::runtime_error("mlp_head_xg: nslab must be 7 or 28");
  if (xg.S < (long long)HP * (((B + 15) / 16) * 16))
    throw std::runtime_error("mlp_head_xg: exchange slots smaller than the factor plane");
  const Bufs w = make_bufs(ws, B);
#define DTFX_HX(WW)                                                                            \
  case WW:                                                                                     \
    if (nslab == KS)                                                                           \
      hipLaunchKernelGGL((mlp_head_kernel<false, false, WW>), dim3(B), dim3(64), 0, stream, p, \
                         p, 0.f, nullptr, labels, w, B, nullptr, xg, dz1A);                    \
    else                                                                                       \
      hipLaunchKernelGGL((mlp_head_kernel<false, false, WW, KS3>), dim3(B), dim3(64), 0, stream, \
                         p, p, 0.f, nullptr, labels, w, B, nullptr, xg, dz1A);                 \
    break;
  switch (world) {
    DTFX_HX(2) DTFX_HX(3) DTFX_HX(4) DTFX_HX(5) DTFX_HX(6) DTFX_HX(7) DTFX_HX(8)
    default:
      throw std::runtime_error("mlp_head_xg: world must be 2..8");
  }
#undef DTFX_HX
  DTFX_HIP_CHECK(hipGetLastError());
}

void mlp_wgrad_factor_launch(float* p, float lr, const float* x, long long xstride,
                             const float* dz1A, float* ws, int* ctr, float* stats, int stats_ring,
                             int B, hipStream_t stream, const MlpXg& xg, int world) {
  using namespace mlp;
  check_b(B);
  if (stats && stats_ring < 1) throw std::runtime_error("mlp_wgrad: stats_ring < 1");
  if (!ctr || !p || !dz1A) throw std::runtime_error("mlp_wgrad_factor: null buffer");
  if (xg.S < NPARAM) throw std::runtime_error("mlp_wgrad_factor: exchange slots smaller than the model");
  const Bufs w = make_bufs(ws, B);
  dim3 grid(8 * HT * ((FT + 7) / 8) + HT), block(256);
  const int NG = (B + 15) / 16;
#define DTFX_WF(WW, NGT)                                                                       \
  hipLaunchKernelGGL((mlp_wgrad_factor_kernel<WW, NGT>), grid, block, 0, stream, p, lr, x,     \
                     xstride, dz1A, w, ctr, stats, stats_ring, B, xg)
#define DTFX_WFW(WW)             \
  case WW:                       \
    if (NG == 7) DTFX_WF(WW, 7); \
    else DTFX_WF(WW, 0);         \
    break;
  switch (world) {
    DTFX_WFW(2) DTFX_WFW(3) DTFX_WFW(4) DTFX_WFW(5) DTFX_WFW(6) DTFX_WFW(7) DTFX_WFW(8)
    default:
      throw std::runtime_error("mlp_wgrad_factor: world must be 2..8");
  }
#undef DTFX_WFW
#undef DTFX_WF
  DTFX_HIP_CHECK(hipGetLastError());
}


// K slices of the single-GPU pipelined step (fwdapply + head agree on it): KS3 = 28, or
// DTFX_MLP_KS=14 for the layout of the data-parallel engines (A/B runs).
static int mlp_single_ks() {
  static const int ks = [] {
    const char* e = std::getenv("DTFX_MLP_KS");
    return e && std::atoi(e) == 14 ? 14 : 28;
  }();
  return ks;
}

// Pipelined single-GPU step (see mlp_fwdapply_kernel): K1' then the head over the K slabs.
void mlp_fwdapply_launch(const float* p_old, float* p_new, float lr, const float* x_prev,
                         const float* x, float* ws, int* ctr, float* stats, int stats_ring, int B,
                         int stats_on, hipStream_t stream, int ks) {
  using namespace mlp;
  check_b(B);
  if (!p_old || !p_new || p_old == p_new || !x_prev || !x || !ctr)
    throw std::runtime_error("mlp_fwdapply: needs distinct ping-pong buffers, both batches, ctr");
  if (stats && stats_ring < 1) throw std::runtime_error("mlp_fwdapply: stats_ring < 1");
  const Bufs w = make_bufs(ws, B);
  const bool rt7 = (B + 15) / 16 == 7;
  if (ks == 0) ks = mlp_single_ks();
  if (ks != KS2 && ks != KS3) throw std::runtime_error("mlp_fwdapply: ks must be 0, 14 or 28");
  if (ks == KS3) {
    dim3 grid(HT * KS3 + HT), block(256);
    if (rt7)
      hipLaunchKernelGGL((mlp_fwdapply_kernel<7, 0, false, false, KS3>), grid, block, 0, stream, p_old,
                         p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B, stats_on, MlpXg{},
                         nullptr);
    else
      hipLaunchKernelGGL((mlp_fwdapply_kernel<0, 0, false, false, KS3>), grid, block, 0, stream, p_old,
                         p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B, stats_on, MlpXg{},
                         nullptr);
  } else {
    dim3 grid(HT * KS2 + HT), block(256);
    if (rt7)
      hipLaunchKernelGGL((mlp_fwdapply_kernel<7>), grid, block, 0, stream, p_old, p_new, lr, x_prev,
                         x, w, ctr, stats, stats_ring, B, stats_on, MlpXg{});
    else
      hipLaunchKernelGGL((mlp_fwdapply_kernel<0>), grid, block, 0, stream, p_old, p_new, lr, x_prev,
                         x, w, ctr, stats, stats_ring, B, stats_on, MlpXg{});
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

// The pending update of the last single-GPU pipelined step (the flush): W1 from step t's
// factors and its small parameters, p_old -> p_new, with step t's loss / accuracy record and
// global_step += 1 -- the first launch's apply half alone (mlp_fwdapply_kernel<.., FWD =
// false>, the single-GPU K slicing), ~half the MFMAs per wave of the 3-launch step's
// mlp_wgrad_kernel.
void mlp_apply_launch(const float* p_old, float* p_new, float lr, const float* x_prev, float* ws,
                      int* ctr, float* stats, int stats_ring, int B, hipStream_t stream) {
  using namespace mlp;
  check_b(B);
  if (!p_old || !p_new || p_old == p_new || !x_prev || !ctr)
    throw std::runtime_error("mlp_apply: needs distinct ping-pong buffers, the batch, ctr");
  if (stats && stats_ring < 1) throw std::runtime_error("mlp_apply: stats_ring < 1");
  const Bufs w = make_bufs(ws, B);
  const bool rt7 = (B + 15) / 16 == 7;
  // DTFX_MLP_FLUSH_FWD=1: the flush runs the steps' own instantiation (FWD = true, its forward
  // over x_prev into the workspace slab, which the next step overwrites) instead of the
  // apply-only one: A/B of whether the flush pays for a code object no step keeps hot
  static const bool ffwd = [] {
    const char* e = std::getenv("DTFX_MLP_FLUSH_FWD");
    return e && std::atoi(e) == 1;
  }();
  if (ffwd) {
    if (mlp_single_ks() == KS3) {
      if (rt7)
        hipLaunchKernelGGL((mlp_fwdapply_kernel<7, 0, false, false, KS3>), dim3(HT * KS3 + HT),
                           dim3(256), 0, stream, p_old, p_new, lr, x_prev, x_prev, w, ctr, stats,
                           stats_ring, B, 1, MlpXg{}, nullptr);
      else
        hipLaunchKernelGGL((mlp_fwdapply_kernel<0, 0, false, false, KS3>), dim3(HT * KS3 + HT),
                           dim3(256), 0, stream, p_old, p_new, lr, x_prev, x_prev, w, ctr, stats,
                           stats_ring, B, 1, MlpXg{}, nullptr);
      DTFX_HIP_CHECK(hipGetLastError());
      return;
    }
  }
#define DTFX_AP(NGT, KSV)                                                                       \
  hipLaunchKernelGGL((mlp_fwdapply_kernel<NGT, 0, false, false, KSV, false>), dim3(HT * KSV + HT), \
                     dim3(256), 0, stream, p_old, p_new, lr, x_prev, x_prev, w, ctr, stats,        \
                     stats_ring, B, 1, MlpXg{}, nullptr)
  if (mlp_single_ks() == KS3) {
    if (rt7) DTFX_AP(7, KS3);
    else DTFX_AP(0, KS3);
  } else {
    if (rt7) DTFX_AP(7, KS2);
    else DTFX_AP(0, KS2);
  }
#undef DTFX_AP
  DTFX_HIP_CHECK(hipGetLastError());
}

// Pipelined fused data-parallel step, first launch (mlp_fwdapply_kernel<.., XW>); the head is
// mlp_head2_launch.  lr already divided by the world size.
void mlp_fwdapply_xg_launch(const float* p_old, float* p_new, float lr, const float* x_prev,
                            const float* x, float* ws, int* ctr, float* stats, int stats_ring,
                            int B, int stats_on, hipStream_t stream, const MlpXg& xg, int world,
                            int two_shot, unsigned long long* trace) {
  using namespace mlp;
  check_b(B);
  if (!p_old || !p_new || p_old == p_new || !x_prev || !x || !ctr)
    throw std::runtime_error("mlp_fwdapply_xg: needs distinct ping-pong buffers, both batches, ctr");
  if (stats && stats_ring < 1) throw std::runtime_error("mlp_fwdapply_xg: stats_ring < 1");
  if (xg.S < NPARAM) throw std::runtime_error("mlp_fwdapply_xg: exchange slots smaller than the model");
  if ((xg.split & 1) && !(two_shot && (xg.split & 4)) && xg.S < XG_SLOT_WORDS)
    throw std::runtime_error("mlp_fwdapply_xg: the split exchange's 16-byte pair layout needs "
                             "slots of mlp_step.XG_SLOT_WORDS words (create the communicator "
                             "with that max_numel)");
  // 28 K slices (as the single-GPU step): 196 W1 blocks x 2 column groups of epoch slots
  static_assert(HT * KS3 * 2 <= MLP_XG_SMALL_EPOCH, "W1 epoch slots overlap the small ones");
  const Bufs w = make_bufs(ws, B);
  dim3 grid(HT * KS3 + HT), block(256);
  if (trace) {  // probe builds (tools/probes/engine_trace.py): [blocks * 4 waves][8] stamps
    if ((B + 15) / 16 != 7) throw std::runtime_error("mlp_fwdapply_xg trace: batch 97..112 only");
#define DTFX_FXT(WW)                                                                            \
  case WW:                                                                                      \
    if (two_shot)                                                                               \
      hipLaunchKernelGGL((mlp_fwdapply_kernel<7, WW, true, true, KS3>), grid, block, 0, stream,  \
                         p_old, p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B, stats_on, xg, \
                         trace);                                                                \
    else                                                                                        \
      hipLaunchKernelGGL((mlp_fwdapply_kernel<7, WW, true, false, KS3>), grid, block, 0, stream, \
                         p_old, p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B, stats_on, xg, \
                         trace);                                                                \
    break;
    switch (world) {
      DTFX_FXT(2) DTFX_FXT(4) DTFX_FXT(8)
      default:
        throw std::runtime_error("mlp_fwdapply_xg trace: world 2, 4 or 8");
    }
#undef DTFX_FXT
    DTFX_HIP_CHECK(hipGetLastError());
    return;
  }
#define DTFX_FX(WW, NGT)                                                                      \
  if (two_shot)                                                                               \
    hipLaunchKernelGGL((mlp_fwdapply_kernel<NGT, WW, false, true, KS3>), grid, block, 0,       \
                       stream, p_old, p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B,      \
                       stats_on, xg, nullptr);                                                \
  else                                                                                        \
    hipLaunchKernelGGL((mlp_fwdapply_kernel<NGT, WW, false, false, KS3>), grid, block, 0,      \
                       stream, p_old, p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B,      \
                       stats_on, xg, nullptr)
#define DTFX_FXW(WW)                        \
  case WW:                                  \
    if ((B + 15) / 16 == 7) DTFX_FX(WW, 7); \
    else DTFX_FX(WW, 0);                    \
    break;
  switch (world) {
    DTFX_FXW(2) DTFX_FXW(3) DTFX_FXW(4) DTFX_FXW(5) DTFX_FXW(6) DTFX_FXW(7) DTFX_FXW(8)
    default:
      throw std::runtime_error("mlp_fwdapply_xg: world must be 2..8");
  }
#undef DTFX_FXW
#undef DTFX_FX
  DTFX_HIP_CHECK(hipGetLastError());
}

// Probe: one pipelined step with in-kernel stamps in both launches (trf: (7 * ks + 7) * 4 * 4
// with ks = mlp_single_ks_query(), trh: B * 4 entries); batch 100 only.
int mlp_single_ks_query() { return mlp_single_ks(); }
void mlp_pipelined_trace_launch(const float* p_old, float* p_new, float lr, const float* x_prev,
                                const float* x, const int* labels, float* ws, int* ctr,
                                float* stats, int stats_ring, int B, hipStream_t stream,
                                unsigned long long* trf, unsigned long long* trh) {
  using namespace mlp;
  check_b(B);
  if ((B + 15) / 16 != 7) throw std::runtime_error("mlp_pipelined_trace: batch 97..112 only");
  const Bufs w = make_bufs(ws, B);
  if (mlp_single_ks() == KS3) {
    hipLaunchKernelGGL((mlp_fwdapply_kernel<7, 0, true, false, KS3>), dim3(HT * KS3 + HT), dim3(256),
                       0, stream, p_old, p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B, 1,
                       MlpXg{}, trf);
    hipLaunchKernelGGL((mlp_head_kernel<false, true, 0, KS3>), dim3(B), dim3(64), 0, stream, p_new,
                       p_new, 0.f, nullptr, labels, w, B, trh, MlpXg{}, nullptr);
  } else {
    hipLaunchKernelGGL((mlp_fwdapply_kernel<7, 0, true>), dim3(HT * KS2 + HT), dim3(256), 0, stream,
                       p_old, p_new, lr, x_prev, x, w, ctr, stats, stats_ring, B, 1, MlpXg{}, trf);
    hipLaunchKernelGGL((mlp_head_kernel<false, true, 0, KS2>), dim3(B), dim3(64), 0, stream, p_new,
                       p_new, 0.f, nullptr, labels, w, B, trh, MlpXg{}, nullptr);
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

// nslab: the K slabs the first launch wrote -- 0: the single-GPU step's (mlp_single_ks());
// the fused2 / fused2x first launch writes KS3 = 28, the factor engine's KS2 = 14.
void mlp_head2_launch(const float* p, const int* labels, float* ws, int B, hipStream_t stream,
                      int nslab) {
  using namespace mlp;
  check_b(B);
  if (nslab == 0) nslab = mlp_single_ks();
  if (nslab != KS2 && nslab != KS3) throw std::runtime_error("mlp_head2: nslab must be 0, 14 or 28");
  const Bufs w = make_bufs(ws, B);
  if (nslab == KS3)
    hipLaunchKernelGGL((mlp_head_kernel<false, false, 0, KS3>), dim3(B), dim3(64), 0, stream, p, p,
                       0.f, nullptr, labels, w, B, nullptr, MlpXg{}, nullptr);
  else
    hipLaunchKernelGGL((mlp_head_kernel<false, false, 0, KS2>), dim3(B), dim3(64), 0, stream, p, p,
                       0.f, nullptr, labels, w, B, nullptr, MlpXg{}, nullptr);
  DTFX_HIP_CHECK(hipGetLastError());
}

// n pipelined single-GPU steps issued from ONE host call (no Python, no hipGraph): step i
// trains on batch (pos + i) % nbatches of the device-resident dataset and ping-pongs the
// parameter buffers exactly like n calls of mlp_fwdapply_launch + mlp_head2_launch.  A graph
// replay pays ~15 us of submission before its first kernel runs; these launches reach the GPU
// one by one while the host keeps queueing ahead (host ~2 us per launch < ~4 us of GPU time
// per launch), so a short run starts at once.  Returns nothing: the caller advances its host
// mirrors (batch position, parity, pending) by n.
// flush != 0: the pending update of the last step is applied by one more launch
// (mlp_apply_launch, into the other buffer: the parity then moves by n + 1).
// DTFX_MLP_FLUSH_FUSED=1: the last step's head and the flush in ONE launch
// (mlp_head_flush_kernel).  Opt-in: correct (bit-identical to the separate flush, tests/
// test_kernels_gpu.py) but measured SLOWER in the driver-sized region -- 10.97-11.05 M vs
// 11.37-11.46 M samples/s, six interleaved pairs on one box (profiles/r6/k20/flush_fused_ab/):
// the in-kernel hand-off (release adds of 100 row waves, the apply blocks' acquire poll, their
// cold operand loads after it) costs ~7 us more than the kernel boundary it replaces, as the
// persistent engine's hand-offs did (mlp_persistent.hip).
static int g_flush_fused = -1;  // -1: read DTFX_MLP_FLUSH_FUSED on first use
static bool mlp_flush_fused() {
  if (g_flush_fused < 0) {
    const char* e = std::getenv("DTFX_MLP_FLUSH_FUSED");
    g_flush_fused = e && std::atoi(e) == 1 ? 1 : 0;
  }
  return g_flush_fused == 1;
}
// tests: select the terminal form in-process (returns the previous setting)
int mlp_set_flush_fused(int on) {
  const int old = mlp_flush_fused() ? 1 : 0;
  g_flush_fused = on ? 1 : 0;
  return old;
}

void mlp_run_pipelined_launch(float* p0, float* p1, int cur, int pending, float lr,
                              const float* x, const int* labels, int nbatches, int pos, int n,
                              float* ws, int* ctr, float* stats, int stats_ring, int B,
                              hipStream_t stream, int flush) {
  using namespace mlp;
  check_b(B);
  if (!p0 || !p1 || p0 == p1 || !x || !labels || !ctr || nbatches < 1 || pos < 0 ||
      pos >= nbatches || n < 0)
    throw std::runtime_error("mlp_run_pipelined: bad buffers / position / count");
  if (stats && stats_ring < 1) throw std::runtime_error("mlp_run_pipelined: stats_ring < 1");
  const Bufs w = make_bufs(ws, B);
  float* bufs[2] = {p0, p1};
  const size_t xb = (size_t)B * D;
  const bool rt7 = (B + 15) / 16 == 7;
  const bool ks3 = mlp_single_ks() == KS3;
  const bool fused_flush = flush && n > 0 && mlp_flush_fused();
  for (int i = 0; i < n; ++i) {
    const int prev = (pos + nbatches - 1) % nbatches;
    const float* xcur = x + (size_t)pos * xb;
    const float* xprev = pending ? x + (size_t)prev * xb : xcur;
    const float* po = bufs[cur];
    float* pn = bufs[cur ^ 1];
    const float l = pending ? lr : 0.f;  // (pending doubles as the kernel's "apply / record
                                         //  the previous step" flag, as in step_pipelined)
    if (fused_flush && i == n - 1) {
      // the last step: its first launch as usual, then ONE launch for its head and the apply
      // of its update (pn -> po: the flush's destination, the other buffer)
      const int nhb = (B + 3) / 4;
      const long long ticks = 200000000LL;  // 2 s of s_memrealtime (100 MHz)
#define DTFX_HF(NGT, KSV)                                                                        \
  do {                                                                                           \
    hipLaunchKernelGGL((mlp_fwdapply_kernel<NGT, 0, false, false, KSV>), dim3(HT * KSV + HT),      \
                       dim3(256), 0, stream, po, pn, l, xprev, xcur, w, ctr, stats, stats_ring, B, \
                       pending, MlpXg{}, nullptr);                                               \
    hipLaunchKernelGGL((mlp_head_flush_kernel<NGT, KSV>), dim3(nhb + HT * KSV + HT), dim3(256), 0, \
                       stream, pn, bufs[cur], lr, xcur, labels + (size_t)pos * B, w, ctr, stats,  \
                       stats_ring, B, ticks);                                                    \
  } while (0)
      if (ks3) {
        if (rt7) DTFX_HF(7, KS3);
        else DTFX_HF(0, KS3);
      } else {
        if (rt7) DTFX_HF(7, KS2);
        else DTFX_HF(0, KS2);
      }
#undef DTFX_HF
      cur ^= 1;  // (the step: po -> pn; the flush below moves it back -- net parity n + 1)
      pending = 0;
      pos = (pos + 1) % nbatches;
      break;
    }
    if (ks3) {
      if (rt7)
        hipLaunchKernelGGL((mlp_fwdapply_kernel<7, 0, false, false, KS3>), dim3(HT * KS3 + HT),
                           dim3(256), 0, stream, po, pn, l, xprev, xcur, w, ctr, stats, stats_ring,
                           B, pending, MlpXg{}, nullptr);
      else
        hipLaunchKernelGGL((mlp_fwdapply_kernel<0, 0, false, false, KS3>), dim3(HT * KS3 + HT),
                           dim3(256), 0, stream, po, pn, l, xprev, xcur, w, ctr, stats, stats_ring,
                           B, pending, MlpXg{}, nullptr);
      hipLaunchKernelGGL((mlp_head_kernel<false, false, 0, KS3>), dim3(B), dim3(64), 0, stream, pn,
                         pn, 0.f, nullptr, labels + (size_t)pos * B, w, B, nullptr, MlpXg{},
                         nullptr);
    } else {
      if (rt7)
        hipLaunchKernelGGL((mlp_fwdapply_kernel<7>), dim3(HT * KS2 + HT), dim3(256), 0, stream, po,
                           pn, l, xprev, xcur, w, ctr, stats, stats_ring, B, pending, MlpXg{});
      else
        hipLaunchKernelGGL((mlp_fwdapply_kernel<0>), dim3(HT * KS2 + HT), dim3(256), 0, stream, po,
                           pn, l, xprev, xcur, w, ctr, stats, stats_ring, B, pending, MlpXg{});
      hipLaunchKernelGGL((mlp_head_kernel<false, false, 0, KS2>), dim3(B), dim3(64), 0, stream, pn,
                         pn, 0.f, nullptr, labels + (size_t)pos * B, w, B, nullptr, MlpXg{},
                         nullptr);
    }
    cur ^= 1;
    pending = 1;
    pos = (pos + 1) % nbatches;
  }
  if (flush && pending) {  // the last step's pending update: bufs[cur] -> bufs[cur ^ 1]
    const int prev = (pos + nbatches - 1) % nbatches;
    mlp_apply_launch(bufs[cur], bufs[cur ^ 1], lr, x + (size_t)prev * xb, ws, ctr, stats,
                     stats_ring, B, stream);
  }
  DTFX_HIP_CHECK(hipGetLastError());
}

// Pipelined factor engine, first launch (see mlp_fwdapply_factor_kernel).
void mlp_fwdapply_factor_launch(const float* p_old, float* p_new, float lr, const float* x_prev,
                                const float* x, long long xstride, const float* dz1A, float* ws,
                                int* ctr, float* stats, int stats_ring, int B, int stats_on,
                                hipStream_t stream, const MlpXg& xg, int world) {
  using namespace mlp;
  check_b(B);
  if ((B + 15) / 16 > 8) throw std::runtime_error("mlp_fwdapply_factor: batch must be <= 128");
  if (!p_old || !p_new || p_old == p_new || !x_prev || !x || !ctr || !dz1A)
    throw std::runtime_error("mlp_fwdapply_factor: needs ping-pong buffers, batches, ctr, dz1A");
  if (xg.S < NPARAM) throw std::runtime_error("mlp_fwdapply_factor: exchange slots too small");
  const Bufs w = make_bufs(ws, B);
  dim3 grid(8 * FX_SLOTS + HT);
#define DTFX_FF(WW, NGT)                                                                       \
  hipLaunchKernelGGL((mlp_fwdapply_factor_kernel<WW, NGT>), grid, dim3(128 * fx_kspl<NGT>()), 0, \
                     stream, p_old,                                                            \
                     p_new, lr, x_prev, x, xstride, dz1A, w, ctr, stats, stats_ring, B,        \
                     stats_on, xg)
#define DTFX_FFW(WW)                                 \
  case WW:                                           \
    if ((B + 15) / 16 == 7) DTFX_FF(WW, 7);          \
    else DTFX_FF(WW, 0);                             \
    break;
  switch (world) {
    DTFX_FFW(2) DTFX_FFW(3) DTFX_FFW(4) DTFX_FFW(5) DTFX_FFW(6) DTFX_FFW(7) DTFX_FFW(8)
    default:
      throw std::runtime_error("mlp_fwdapply_factor: world must be 2..8");
  }
#undef DTFX_FFW
#undef DTFX_FF
  DTFX_HIP_CHECK(hipGetLastError());
}
// Async-PS worker step (train/worker.py, the reference's hot loop worker.py:131-137) in ONE
// host call: the staged batch (pinned host -> device), the parameters pulled by the last
// push/step/pull exchange (pinned host, TF layout -> device flat layout; skipped when
// pulled_host is null), forward + backward writing the flat gradient, the gradient in TF
// layout with the step's loss / accuracy record appended (-> pinned host), and a wait for the
// stream.  Replaces ~10 Python-issued copies / launches / syncs per step; the caller releases
// the GIL for the call.  Host buffers must be pinned (hipHostMalloc'd); *_dev are device staging
// buffers of NPARAM + 2 floats.
// Device address of a pinned host buffer when the runtime maps it into the GPU's address
// space (hipHostMalloc'd memory: the kernels then read / write it over the host link
// directly), else null and the caller moves it with a DMA copy.  Looked up per buffer once.
static const void* mapped_device_ptr(const void* host) {
  static std::mutex mu;
  static std::map<const void*, const void*> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(host);
  if (it != cache.end()) return it->second;
  hipPointerAttribute_t a{};
  const void* d = nullptr;
  if (hipPointerGetAttributes(&a, host) == hipSuccess) {
    if (a.type == hipMemoryTypeHost && a.devicePointer) d = a.devicePointer;
  } else {
    (void)hipGetLastError();  // not a HIP allocation: clear the sticky error
  }
  if (getenv("DTFX_PS_NO_ZERO_COPY")) d = nullptr;
  cache[host] = d;
  return d;
}

void mlp_ps_worker_step(float* p, const float* pulled_host, float* pull_dev, const float* x_host,
                        const int* y_host, float* x_dev, int* y_dev, float* grad, float* ws,
                        int* ctr, float* stats, int stats_ring, const float* record, int B,
                        float* grad_dev, float* grad_host, hipStream_t s) {
  using namespace mlp;
  check_b(B);
  if (!p || (x_host && !y_host) || !x_dev || !y_dev || !grad || !ws || !ctr || !grad_dev ||
      !grad_host || (pulled_host && !pull_dev) || (record && !stats))
    throw std::runtime_error("mlp_ps_worker_step: missing buffer");
  if (x_host) {  // (null: already staged by mlp_ps_stage while the last exchange was in flight)
    DTFX_HIP_CHECK(hipMemcpyAsync(x_dev, x_host, sizeof(float) * (size_t)B * D,
                                  hipMemcpyHostToDevice, s));
    DTFX_HIP_CHECK(hipMemcpyAsync(y_dev, y_host, sizeof(int) * (size_t)B, hipMemcpyHostToDevice, s));
  }
  // zero copy where the pinned buffers are device-mapped: the layout kernels read the pulled
  // parameters from / write the gradient to host memory themselves -- no DMA copy (each has
  // a setup latency of several us on top of the transfer) and two fewer queue entries
  const float* pulled_map = pulled_host ? (const float*)mapped_device_ptr(pulled_host) : nullptr;
  float* grad_map = (float*)mapped_device_ptr(grad_host);
  if (pulled_host) {
    if (pulled_map) {
      hipLaunchKernelGGL(mlp_from_tf_src_major_kernel, dim3((NPARAM + 255) / 256), dim3(256), 0,
                         s, pulled_map, p);
      DTFX_HIP_CHECK(hipGetLastError());
    } else {
      DTFX_HIP_CHECK(hipMemcpyAsync(pull_dev, pulled_host, sizeof(float) * NPARAM,
                                    hipMemcpyHostToDevice, s));
      mlp_tf_layout_launch(pull_dev, p, 0, nullptr, 0, s);
    }
  }
  mlp_fwd_launch(p, nullptr, 0.f, nullptr, x_dev, ws, B, s, nullptr);
  mlp_head_launch(p, nullptr, 0.f, nullptr, y_dev, ws, B, s, nullptr);
  mlp_wgrad_launch(nullptr, 0.f, grad, x_dev, ws, ctr, stats, stats_ring, B, s, nullptr);
  if (grad_map) {
    mlp_tf_layout_launch(grad, grad_map, 1, record, record ? 2 : 0, s);
  } else {
    mlp_tf_layout_launch(grad, grad_dev, 1, record, record ? 2 : 0, s);
    DTFX_HIP_CHECK(hipMemcpyAsync(grad_host, grad_dev, sizeof(float) * (NPARAM + (record ? 2 : 0)),
                                  hipMemcpyDeviceToHost, s));
  }
  DTFX_HIP_CHECK(hipStreamSynchronize(s));
}


// The next batch's H2D copies (pinned host -> device), issued while the previous step's
// push/step/pull exchange is on the wire; mlp_ps_worker_step then runs with x_host = null.
void mlp_ps_stage(const float* x_host, const int* y_host, float* x_dev, int* y_dev, int B,
                  hipStream_t s) {
  check_b(B);
  DTFX_HIP_CHECK(hipMemcpyAsync(x_dev, x_host, sizeof(float) * (size_t)B * mlp::D,
                                hipMemcpyHostToDevice, s));
  DTFX_HIP_CHECK(hipMemcpyAsync(y_dev, y_host, sizeof(int) * (size_t)B, hipMemcpyHostToDevice, s));
}
}  // namespace dtfx
