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
  // 2) raise my flag for this block at every rank (remote stores over xGMI)
  if (t < world)
    __hip_atomic_store(peers.flags[t] + rank * XG_BLOCKS + b, epoch, __ATOMIC_RELAXED,
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
  asm volatile("" ::: "memory");  // no load of peer data above this point
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
// LL ("low-latency") variant: every element travels as ONE 8-byte word {f32 value,
// u32 epoch}, so the data carries its own ready flag -- no store-acknowledge wait,
// no separate flag round trip.  Readers load the W peers' words of an element
// together and re-poll only the ones whose epoch is not yet current.  Slots are
// u64 [2][S], parity by epoch as in the flag protocol (same overwrite argument).
// ---------------------------------------------------------------------------
template <int W>
__global__ __launch_bounds__(256) void xgmi_ll_kernel(float* __restrict__ g, long long n, int rank,
                                                      long long S, XgPeers peers,
                                                      unsigned* __restrict__ epochs,
                                                      int* __restrict__ err, long long timeout_ticks) {
  __shared__ unsigned s_epoch;
  const int b = blockIdx.x, t = threadIdx.x;
  if (t == 0) s_epoch = epochs[b] + 1;
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long long par = (long long)(epoch & 1u) * S;
  const long long per = (n + gridDim.x - 1) / gridDim.x;
  const long long lo = b * per, hi = min(n, lo + per);
  unsigned long long* mine = (unsigned long long*)peers.data[rank] + par;
  for (long long i = lo + t; i < hi; i += blockDim.x)
    __hip_atomic_store(mine + i, ((unsigned long long)epoch << 32) | __float_as_uint(g[i]),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  bool fail = false;
  for (long long i = lo + t; i < hi; i += blockDim.x) {
    unsigned long long w[W];
#pragma unroll
    for (int j = 0; j < W; ++j)
      w[j] = j == rank ? 0ull
                       : __hip_atomic_load((unsigned long long*)peers.data[j] + par + i,
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    for (;;) {
      bool ready = true;
#pragma unroll
      for (int j = 0; j < W; ++j)
        if (j != rank && (unsigned)(w[j] >> 32) != epoch) {
          ready = false;
          w[j] = __hip_atomic_load((unsigned long long*)peers.data[j] + par + i, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
        }
      if (ready) break;
      if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        fail = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (fail) break;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < W; ++j) acc += j == rank ? g[i] : __uint_as_float((unsigned)w[j]);
    g[i] = acc;
  }
  if (fail) atomicExch(err, 1);
  __syncthreads();
  if (t == 0) epochs[b] = epoch;
}

void xgmi_ll_launch(float* g, long long n, int rank, int world, long long S, const XgPeers& peers,
                    unsigned* epochs, int* err, long long ticks, hipStream_t stream) {
  const dim3 grid(XG_BLOCKS), block(256);
  switch (world) {
#define DTFX_LL(WW)                                                                            \
  case WW:                                                                                     \
    hipLaunchKernelGGL(xgmi_ll_kernel<WW>, grid, block, 0, stream, g, n, rank, S, peers, epochs, \
                       err, ticks);                                                            \
    break;
    DTFX_LL(1) DTFX_LL(2) DTFX_LL(3) DTFX_LL(4) DTFX_LL(5) DTFX_LL(6) DTFX_LL(7) DTFX_LL(8)
#undef DTFX_LL
    default:
      throw std::runtime_error("xgmi LL protocol: world must be <= 8");
  }
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
