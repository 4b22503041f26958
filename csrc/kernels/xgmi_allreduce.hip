// One-shot all-reduce over xGMI peer memory for SMALL gradient buffers (the
// MNIST MLP's 318 KB), one kernel launch per call.
//
// Why: a ring all-reduce moves data through world-1 dependent hops per phase,
// each a link latency, so a few-hundred-KB bucket is latency bound.  On MI355X
// every GPU has a direct xGMI link to every other GPU of the node, so one
// "publish, flag, read-all" round suffices: each rank copies its buffer into an
// uncached (fine-grained, MTYPE UC) IPC-shared slot, raises a per-block flag in
// every peer's flag array (remote stores), waits for all peers' flags for the
// same block, then sums the world slices in rank order (so every replica
// computes bit-identical results) straight from peer memory.  UC accesses
// bypass all GPU caches, so ordering needs only vmcnt waits -- no system-scope
// fence (which would write back / invalidate the whole L2).
//
// Safety: the flag of block b is an epoch counter owned by block b (device
// resident, so hipGraph replays advance it); slots alternate by epoch parity,
// and a rank can only overwrite a parity after every peer has finished the
// previous round of that block (argument in docs/COMM.md).  Every spin is
// bounded (s_memrealtime, default 2 s): on timeout the kernel raises an error
// word and returns, the host raises instead of hanging.
//
// Reference counterpart: the reference's PS pull/push per step (worker.py:131,
// 135-137) -- here replaced by sync all-reduce; RCCL stays the default path.
#include "common.h"

#include "xgmi.h"
#include "xgmi_ll.h"

#include <cstdlib>
#include <stdexcept>

namespace dtfx {

__global__ __launch_bounds__(256) void xgmi_allreduce_kernel(float* __restrict__ g, long long n,
                                                             int rank, int world, long long S,
                                                             XgPeers peers,
                                                             unsigned* __restrict__ epochs,
                                                             int* __restrict__ err,
                                                             long long timeout_ticks) {
  __shared__ unsigned s_epoch;
  __shared__ int s_fail;
  const int b = blockIdx.x, t = threadIdx.x;
  if (t == 0) {
    s_epoch = epochs[b] + 1;  // block-private counter: no cross-block race
    s_fail = 0;
  }
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long long par = (long long)(epoch & 1u) * S;
  const long long n4 = n >> 2;
  const long long per = (n4 + gridDim.x - 1) / gridDim.x;
  const long long lo = b * per, hi = min(n4, lo + per);

  // 1) publish this block's slice into my uncached slot
  f32x4* mine = (f32x4*)(peers.data[rank] + par);
  for (long long i = lo + t; i < hi; i += blockDim.x) mine[i] = ((const f32x4*)g)[i];
  if (b == 0 && t < (int)(n & 3)) peers.data[rank][par + 4 * n4 + t] = g[4 * n4 + t];
  // the slice's UC stores are acknowledged (globally visible) before any flag goes out
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 2) raise my flag for this block at every rank (remote stores over xGMI).  RELEASE at
  // system scope: an acknowledged store (vmcnt) is not yet ordered before a store to
  // another channel, and a reader that saw the flag read the previous epoch's slice
  // (measured: 3 ranks on one GPU, a few stale elements per 40 steps).  The LL protocols
  // below carry the epoch inside every data word and need no such fence; this one is
  // only used beyond 8 ranks.
  if (t < world)
    __hip_atomic_store(peers.flags[t] + rank * XG_BLOCKS + b, epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  // 3) wait until every rank published this block for this epoch (bounded spin)
  if (t < world) {
    const unsigned* f = peers.flags[rank] + t * XG_BLOCKS + b;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        s_fail = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
  if (s_fail) {
    if (t == 0) atomicExch(err, 1);
    return;  // g keeps the local gradient; the host sees err and raises
  }
  // acquire: no load of peer data above this point, none served by a stale cache line.
  // ONE lane per block (buffer_inv sc1 invalidates the CU's whole L1), the block held by a
  // barrier until it completed
  if (t == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // 4) sum the world slices in rank order (identical on every rank) into g
  for (long long i = lo + t; i < hi; i += blockDim.x) {
    f32x4 acc = ((const f32x4*)(peers.data[0] + par))[i];
    for (int j = 1; j < world; ++j) {
      const f32x4 v = ((const f32x4*)(peers.data[j] + par))[i];
      acc += v;
    }
    ((f32x4*)g)[i] = acc;
  }
  if (b == 0 && t < (int)(n & 3)) {
    float a = 0.f;
    for (int j = 0; j < world; ++j) a += peers.data[j][par + 4 * n4 + t];
    g[4 * n4 + t] = a;
  }
  if (t == 0) epochs[b] = epoch;
}

// ---------------------------------------------------------------------------
// LL ("low-latency") protocols: every element travels as ONE 8-byte word {f32 value,
// u32 epoch}, so the data carries its own ready flag -- no store-acknowledge wait and no
// separate flag round trip.  Receivers re-poll only the words whose epoch is not yet
// current (bounded by s_memrealtime).  All slot regions alternate by epoch parity, with
// the same "a rank can only reach epoch e+2 after every peer finished epoch e" argument
// as the flag protocol (docs/COMM.md).  Three data-flow variants:
//   LL_PULL  one-shot, each rank publishes into its OWN slot [2][S]; readers load the
//            peers' words over xGMI (remote polling).
//   LL_PUSH  one-shot, each rank stores its words into slot[me] of EVERY peer
//            ([2][W][S] per rank); receivers poll LOCAL memory only.  Per link: n words.
//   LL_PUSH2 two-shot (reduce-scatter + all-gather): element i is owned by rank
//            i / ceil(n/W); senders push only the owner's share, the owner sums it in
//            rank order and pushes the result into every peer's result region [2][S].
//            Per link: 2n/W words -- the choice for larger worlds / buffers.
// Every rank sums in rank order, so the replicas stay bit-identical.
// ---------------------------------------------------------------------------
using xgll::u64;

template <int W, int MODE>
__global__ __launch_bounds__(256) void xgmi_ll_kernel(float* __restrict__ g, long long n, int rank,
                                                      long long S, XgPeers peers,
                                                      unsigned* __restrict__ epochs,
                                                      int* __restrict__ err, long long ticks) {
  __shared__ unsigned s_epoch;
  const int b = blockIdx.x, t = threadIdx.x, nb = gridDim.x;
  if (t == 0) s_epoch = epochs[b] + 1;  // block-private counter; all blocks advance in step
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long long par = epoch & 1u;
  const long long per = (n + nb - 1) / nb;
  const long long lo = b * per, hi = min(n, lo + per);
  bool fail = false;
  if constexpr (MODE == XG_LL_PULL) {
    // slot: rank j's [2][S] words
    u64* mine = (u64*)peers.data[rank] + par * S;
    for (long long i = lo + t; i < hi; i += blockDim.x) xgll::store(mine + i, xgll::word(g[i], epoch));
    auto base = [&](int j) { return (const u64*)peers.data[j] + par * S; };
    for (long long i = lo + t; i < hi && !fail; i += blockDim.x) {
      const float acc = xgll::gather_sum<W>(base, i, rank, epoch, g[i], ticks, fail);
      if (!fail) g[i] = acc;
    }
  } else {
    // slot(dst, src) = rank dst's words from sender src: [2][W][S]; result region [2][S] after
    auto slot = [&](int dst, int src) { return (u64*)peers.data[dst] + (par * W + src) * S; };
    auto local = [&](int j) { return (const u64*)slot(rank, j); };
    if constexpr (MODE == XG_LL_PUSH) {
      for (long long i = lo + t; i < hi; i += blockDim.x) {
        const u64 w = xgll::word(g[i], epoch);
#pragma unroll
        for (int j = 0; j < W; ++j)
          if (j != rank) xgll::store(slot(j, rank) + i, w);
      }
      for (long long i = lo + t; i < hi && !fail; i += blockDim.x) {
        const float acc = xgll::gather_sum<W>(local, i, rank, epoch, g[i], ticks, fail);
        if (!fail) g[i] = acc;
      }
    } else {  // XG_LL_PUSH2
      auto result = [&](int dst) { return (u64*)peers.data[dst] + (2 * W + par) * S; };
      const long long shard = (n + W - 1) / W;
      // 1) reduce-scatter sends: element i goes to its owner only
      for (long long i = lo + t; i < hi; i += blockDim.x) {
        const int o = (int)(i / shard);
        if (o != rank) xgll::store(slot(o, rank) + i, xgll::word(g[i], epoch));
      }
      // 2) owner: sum my shard (split over the blocks), push the result to every peer
      const long long s0 = rank * shard, s1 = min(n, s0 + shard);
      const long long sper = (s1 - s0 + nb - 1) / nb;
      const long long slo = s0 + b * sper, shi = min(s1, slo + sper);
      for (long long i = slo + t; i < shi && !fail; i += blockDim.x) {
        const float acc = xgll::gather_sum<W>(local, i, rank, epoch, g[i], ticks, fail);
        if (fail) break;
        g[i] = acc;
        const u64 w = xgll::word(acc, epoch);
#pragma unroll
        for (int j = 0; j < W; ++j)
          if (j != rank) xgll::store(result(j) + i, w);
      }
      // 3) all-gather receives: every element owned by a peer
      const u64* res = result(rank);
      for (long long i = lo + t; i < hi && !fail; i += blockDim.x) {
        if ((int)(i / shard) == rank) continue;
        const float v = xgll::wait_one(res + i, epoch, ticks, fail);
        if (!fail) g[i] = v;
      }
    }
  }
  if (fail) atomicExch(err, 1);
  __syncthreads();
  if (t == 0) epochs[b] = epoch;
}

// ---------------------------------------------------------------------------
// BW: bandwidth-mode two-shot all-reduce for LARGE buckets (BERT / ResNet gradients),
// f32 payload (no epoch inside the data: every byte on the links is gradient) and
// per-(phase, source, block) release flags.  Each rank owns chunk r = [r*cs, (r+1)*cs) of
// the buffer (cs = ceil(n / W), float4-aligned):
//   1) reduce-scatter: rank r stores its share of EVERY peer's chunk straight into that
//      peer's receive slot rs(q, par, r) -- remote writes over the W-1 xGMI links in
//      parallel -- then raises flag (0, r, b) at every peer;
//   2) once the W-1 flags of its chunk are up, the owner sums the W contributions in rank
//      order (bit-identical on every rank), keeps the result and stores it into every
//      peer's gather region ag(q, par) (remote writes again), then raises flag (1, r, b);
//   3) once the W-1 gather flags are up, every rank copies the other owners' chunks from
//      its local gather region into g.
// Per link and direction: 2 (W-1)/W * n * 4 bytes -- a ring's volume, but moved over all
// W-1 links at once instead of one.  Block b handles sub-range b of every chunk; flags are
// epoch counters owned by block b (device-resident epochs: graph replays advance them),
// slots alternate by epoch parity (the flag protocol's argument: a rank reaches epoch e+2
// only after every peer finished epoch e).  Every wait is bounded (s_memrealtime).
// Region of one rank (floats): rs [2][W][CS] | ag [2][S]; flags [2 phases][W][XG_BLOCKS].
// OP 0 is that all-reduce; the owner-sharded optimizer (ZeRO-1, train/bert_trainer.py) uses
// its halves alone: OP 1 = reduce-scatter (step 1 and the owner sum, kept in g's chunk r,
// nothing pushed), OP 2 = all-gather (g's chunk r is already final: step 2's push of it, then
// step 3).  The epoch / parity argument holds for any sequence of the three: every call waits
// on all peers' flags after its own writes and before its reads of the slots.
// ---------------------------------------------------------------------------
__host__ __device__ inline long long xg_bw_cs(long long S, int W) {
  return ((S + W - 1) / W + 3) / 4 * 4;
}

template <int W, int OP>
__global__ __launch_bounds__(512) void xgmi_bw_kernel(float* __restrict__ g, long long n, int rank,
                                                      long long S, XgPeers peers,
                                                      unsigned* __restrict__ epochs,
                                                      int* __restrict__ err, long long ticks,
                                                      const int* __restrict__ abort_word) {
  __shared__ unsigned s_epoch;
  __shared__ int s_fail;
  const int b = blockIdx.x, t = threadIdx.x, nt = blockDim.x, nb = gridDim.x;
  if (t == 0) {
    s_epoch = epochs[b] + 1;
    // a communicator that already timed out (a peer is gone) or was aborted by the host is
    // broken for good: calls queued behind the failed one leave at once instead of each waiting
    // `ticks` again, so the stream drains within one timeout
    s_fail = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
             __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  if (s_fail) return;
  const unsigned epoch = s_epoch;
  const long long par = epoch & 1u;
  const long long CS = xg_bw_cs(S, W);             // slot capacity of one chunk
  const long long cs = ((n + W - 1) / W + 3) / 4 * 4;  // this call's chunk length
  const long long per = ((cs + nb - 1) / nb + 3) / 4 * 4;
  const long long lo = b * per;                    // sub-range [lo, hi) of every chunk
  // elements of chunk c in this block's sub-range (<= 0: none)
  auto chunk_hi = [&](int c) { return min(min(per, cs - lo), n - c * cs - lo); };
  auto rs = [&](int q, int src) { return peers.data[q] + (par * W + src) * CS; };
  auto ag = [&](int q) { return peers.data[q] + 2 * W * CS + par * S; };
  auto flag = [&](int q, int phase, int src) {
    return peers.flags[q] + (phase * W + src) * XG_BLOCKS + b;
  };
  // consumer: the W-1 polls, then ONE agent-scope acquire per block -- buffer_inv sc1
  // invalidates the whole CU's L1, so one lane suffices (every thread of the 256 512-thread
  // blocks fencing cost ~28 us per call, docs/COMM.md) -- and a barrier that holds the
  // block until it has completed
  auto wait_flags = [&](int phase) {
    if (t < W && t != rank) {
      const unsigned* f = flag(rank, phase, t);
      const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
      long long t_ab = t0;
      while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
        const long long now = (long long)__builtin_amdgcn_s_memrealtime();
        if (now - t0 > ticks) {
          s_fail = 1;
          break;
        }
        // the host's abort word (pinned host memory, set by the peer watchdog's abort hook:
        // XgmiComm.abort) is read once per ~1 ms of waiting -- a PCIe round trip per spin
        // would slow the flag poll -- so an aborted job's waves leave the GPU within ~1 ms
        // instead of at the end of a long training timeout
        if (now - t_ab > 100000) {
          t_ab = now;
          if (__hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) {
            s_fail = 1;
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
  };
  // producer: every thread's stores acknowledged, then ONE system-scope release per block
  // (with the explicit vmcnt wait the compiler may otherwise drop, MI355X_MICROARCH.md
  // "Compiler hazard") and relaxed flag stores to the W-1 peers
  auto raise_flags = [&](int phase) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int q = 0; q < W; ++q)
        if (q != rank)
          __hip_atomic_store(flag(q, phase, rank), epoch, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    }
  };
  // 1) reduce-scatter sends: my share of chunk q -> rs(q, par, me), all peers interleaved
  //    so every link carries traffic at once
  if constexpr (OP != 2) {
  for (int k = 1; k < W; ++k) {
    const int q = (rank + k) % W;
    const long long m = chunk_hi(q);
    if (m <= 0) continue;
    const f32x4* src = (const f32x4*)(g + q * cs + lo);
    f32x4* dst = (f32x4*)(rs(q, rank) + lo);
    const long long m4 = m >> 2;
    for (long long i = t; i < m4; i += nt) dst[i] = src[i];
    for (long long i = 4 * m4 + t; i < m; i += nt) rs(q, rank)[lo + i] = g[q * cs + lo + i];
  }
  raise_flags(0);
  wait_flags(0);
  if (s_fail) {
    if (t == 0) atomicExch(err, 1);
    return;
  }
  }  // OP != 2
  // 2) owner: rank-ordered sum of my chunk's sub-range, kept in g and pushed to every peer
  //    (OP 1: kept only; OP 2: my chunk is final already -- pushed only)
  {
    const long long m = chunk_hi(rank);
    if (m > 0) {
      float* mine = g + rank * cs + lo;
      const long long m4 = m >> 2;
      for (long long i = t; i < m4; i += nt) {
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
        if constexpr (OP == 2) {
          acc = ((const f32x4*)mine)[i];
        } else {
#pragma unroll
          for (int j = 0; j < W; ++j) {
            const f32x4 v = j == rank ? ((const f32x4*)mine)[i] : ((const f32x4*)(rs(rank, j) + lo))[i];
            acc += v;
          }
          ((f32x4*)mine)[i] = acc;
        }
        if constexpr (OP != 1) {
#pragma unroll
          for (int k = 1; k < W; ++k) ((f32x4*)(ag((rank + k) % W) + rank * cs + lo))[i] = acc;
        }
      }
      for (long long i = 4 * m4 + t; i < m; i += nt) {
        float acc = 0.f;
        if constexpr (OP == 2) {
          acc = mine[i];
        } else {
#pragma unroll
          for (int j = 0; j < W; ++j) acc += j == rank ? mine[i] : rs(rank, j)[lo + i];
          mine[i] = acc;
        }
        if constexpr (OP != 1) {
#pragma unroll
          for (int k = 1; k < W; ++k) ag((rank + k) % W)[rank * cs + lo + i] = acc;
        }
      }
    }
  }
  if constexpr (OP == 1) {
    __syncthreads();
    if (t == 0) epochs[b] = epoch;
    return;
  }
  raise_flags(1);
  wait_flags(1);
  if (s_fail) {
    if (t == 0) atomicExch(err, 1);
    return;
  }
  // 3) all-gather receives: the other owners' chunks from my gather region
  for (int k = 1; k < W; ++k) {
    const int c = (rank + k) % W;
    const long long m = chunk_hi(c);
    if (m <= 0) continue;
    const f32x4* src = (const f32x4*)(ag(rank) + c * cs + lo);
    f32x4* dst = (f32x4*)(g + c * cs + lo);
    const long long m4 = m >> 2;
    for (long long i = t; i < m4; i += nt) dst[i] = src[i];
    for (long long i = 4 * m4 + t; i < m; i += nt) g[c * cs + lo + i] = ag(rank)[c * cs + lo + i];
  }
  __syncthreads();
  if (t == 0) epochs[b] = epoch;
}

long long xgmi_ll_bytes(int mode, int world, long long S) {
  if (mode == XG_LL_PULL) return 8LL * 2 * S;
  if (mode == XG_BW) return 4LL * (2LL * world * xg_bw_cs(S, world) + 2 * S);
  return 8LL * (2LL * world * S + 2 * S);
}

void xgmi_bw_launch(float* g, long long n, int rank, int world, long long S, const XgPeers& peers,
                    unsigned* epochs, int* err, long long ticks, hipStream_t stream, int blocks,
                    const int* abort_word, int op) {
  if (!abort_word) throw std::runtime_error("xgmi bw protocol: needs the host abort word");
  if (op < 0 || op > 2) throw std::runtime_error("xgmi bw protocol: op must be 0 (all-reduce), "
                                                 "1 (reduce-scatter) or 2 (all-gather)");
  const dim3 grid(blocks), block(512);
#define DTFX_BW(WW)                                                                          \
  case WW:                                                                                   \
    if (op == 0)                                                                             \
      hipLaunchKernelGGL((xgmi_bw_kernel<WW, 0>), grid, block, 0, stream, g, n, rank, S,     \
                         peers, epochs, err, ticks, abort_word);                             \
    else if (op == 1)                                                                        \
      hipLaunchKernelGGL((xgmi_bw_kernel<WW, 1>), grid, block, 0, stream, g, n, rank, S,     \
                         peers, epochs, err, ticks, abort_word);                             \
    else                                                                                     \
      hipLaunchKernelGGL((xgmi_bw_kernel<WW, 2>), grid, block, 0, stream, g, n, rank, S,     \
                         peers, epochs, err, ticks, abort_word);                             \
    break;
  switch (world) {
    DTFX_BW(1) DTFX_BW(2) DTFX_BW(3) DTFX_BW(4) DTFX_BW(5) DTFX_BW(6) DTFX_BW(7) DTFX_BW(8)
    default:
      throw std::runtime_error("xgmi bw protocol: world must be <= 8");
  }
#undef DTFX_BW
  DTFX_HIP_CHECK(hipGetLastError());
}

void xgmi_ll_launch(int mode, float* g, long long n, int rank, int world, long long S,
                    const XgPeers& peers, unsigned* epochs, int* err, long long ticks,
                    hipStream_t stream) {
  const dim3 grid(XG_BLOCKS), block(256);
#define DTFX_LL(WW, MM)                                                                       \
  hipLaunchKernelGGL((xgmi_ll_kernel<WW, MM>), grid, block, 0, stream, g, n, rank, S, peers, \
                     epochs, err, ticks)
#define DTFX_LLW(WW)                   \
  case WW:                             \
    if (mode == XG_LL_PULL)            \
      DTFX_LL(WW, XG_LL_PULL);         \
    else if (mode == XG_LL_PUSH)       \
      DTFX_LL(WW, XG_LL_PUSH);         \
    else                               \
      DTFX_LL(WW, XG_LL_PUSH2);        \
    break;
  switch (world) {
    DTFX_LLW(1) DTFX_LLW(2) DTFX_LLW(3) DTFX_LLW(4) DTFX_LLW(5) DTFX_LLW(6) DTFX_LLW(7)
    DTFX_LLW(8)
    default:
      throw std::runtime_error("xgmi LL protocols: world must be <= 8");
  }
#undef DTFX_LLW
#undef DTFX_LL
  DTFX_HIP_CHECK(hipGetLastError());
}

void xgmi_allreduce_launch(float* g, long long n, int rank, int world, long long S,
                           const XgPeers& peers, unsigned* epochs, int* err, long long ticks,
                           hipStream_t stream) {
  hipLaunchKernelGGL(xgmi_allreduce_kernel, dim3(XG_BLOCKS), dim3(256), 0, stream, g, n, rank, world,
                     S, peers, epochs, err, ticks);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
