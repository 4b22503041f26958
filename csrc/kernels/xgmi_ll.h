// Device helpers of the xGMI LL ("low-latency") protocols: one 8-byte word per
// element = {f32 value, u32 epoch}, stored / loaded with single relaxed
// system-scope 64-bit accesses into uncached IPC memory, so a word with the
// current epoch always carries the value written with it.  Shared by the
// stand-alone all-reduce (xgmi_allreduce.hip) and the MLP step kernel that
// exchanges its gradient in the epilogue (mlp_step.hip).
#pragma once

#include "common.h"
#include "xgmi.h"

namespace dtfx {
namespace xgll {

using u64 = unsigned long long;

__device__ __forceinline__ u64 word(float v, unsigned e) {
  return ((u64)e << 32) | __float_as_uint(v);
}
// Every LL word lives in device / IPC global memory, so the accesses are issued through the
// global address space (`global_*` instructions, vmcnt only) rather than as FLAT ones (which
// also count in lgkmcnt, so each wait on them waited for the wave's LDS traffic too).
typedef __attribute__((address_space(1))) u64 gu64;
__device__ __forceinline__ void store(u64* p, u64 w) {
  __hip_atomic_store((gu64*)p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ u64 load(const u64* p) {
  return __hip_atomic_load((const gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A 16-byte LL word pair {v0, epoch, v1, epoch} read as TWO relaxed system-scope 8-byte loads
// (each half carries its own epoch).  Not a `volatile` 16-byte load: LLVM completes every
// volatile access before the next one (an `s_waitcnt vmcnt(0)` after each, and a FLAT load
// here), which turned a wave's W - 1 polls into W - 1 serial memory round trips.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 load_pair(const u64* p) {
  const u64 a = load(p), b = load(p + 1);
  return u32x4{(unsigned)a, (unsigned)(a >> 32), (unsigned)b, (unsigned)(b >> 32)};
}

// Polls of a rank's OWN slot region as raw buffer loads (round 6): one 16-byte
// `buffer_load_dwordx4 ... sc0 sc1` per pair instead of two FLAT 8-byte atomic loads.  The
// aux bits are the system-scope coherence bits the relaxed system atomics set (sc0 | sc1), each
// aligned 8-byte half of the access is one {value, epoch} word as before (the half is what
// carries its epoch, so a reader never trusts more than 8 bytes), and unlike a `volatile`
// 16-byte load the compiler tracks the buffer intrinsic like any load: the W - 1 polls stay in
// flight together.  Buffer (and global) instructions count in vmcnt only; a FLAT access counts
// in vmcnt AND lgkmcnt, so every wait on one also waited for the wave's LDS traffic.
struct OwnPoll {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit OwnPoll(const u64* base)
      : r(__builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, 0x7fffffff, 0x00020000)) {}
  // word offsets: `region` (wave-uniform, -> soffset) + `lane_off` (per lane, -> voffset)
  __device__ __forceinline__ u32x4 pair(long long region, long long lane_off) const {
    return __builtin_amdgcn_raw_buffer_load_b128(r, (int)(lane_off * 8), (int)(region * 8), 17);
  }
};
// A 16-byte pair stored to a peer (or own) slot as a GLOBAL store (not FLAT: vmcnt only).
__device__ __forceinline__ void store_pair_g(u64* p, const u32x4& w) {
  *(__attribute__((address_space(1))) u32x4*)p = w;
}

// A wave-uniform value made provably uniform (scalar registers): the peer pointer table and
// the rank come from a kernel-argument struct passed by reference into device helpers, where
// the compiler otherwise may index it with a vector register (a per-lane load of the pointer
// and an s_waitcnt vmcnt(0) before every peer access).
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const u64 v = (u64)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)v);
  const unsigned hi = __builtin_amdgcn_readfirstlane((unsigned)(v >> 32));
  return (T*)(((u64)hi << 32) | lo);
}

// Loads word i of every peer j != rank from base(j) and re-polls the stale ones; returns
// the rank-ordered sum with `own` at position `rank` (identical on every rank), or sets
// fail after `ticks` of s_memrealtime (100 MHz).
template <int W, class Base>
__device__ __forceinline__ float gather_sum(Base base, long long i, int rank, unsigned epoch,
                                            float own, long long ticks, bool& fail) {
  u64 w[W];
#pragma unroll
  for (int j = 0; j < W; ++j) w[j] = j == rank ? 0ull : load(base(j) + i);
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int j = 0; j < W; ++j)
      if (j != rank && (unsigned)(w[j] >> 32) != epoch) {
        ready = false;
        w[j] = load(base(j) + i);
      }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      return 0.f;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  float acc = 0.f;
#pragma unroll
  for (int j = 0; j < W; ++j) acc += j == rank ? own : __uint_as_float((unsigned)w[j]);
  return acc;
}

// Like gather_sum, but returns every peer's value (out[rank] = own): the all-gather form used
// by the MLP factor exchange.
template <int W, class Base>
__device__ __forceinline__ void gather_all(Base base, long long i, int rank, unsigned epoch,
                                           float own, long long ticks, float (&out)[W],
                                           bool& fail) {
  u64 w[W];
#pragma unroll
  for (int j = 0; j < W; ++j) w[j] = j == rank ? 0ull : load(base(j) + i);
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int j = 0; j < W; ++j)
      if (j != rank && (unsigned)(w[j] >> 32) != epoch) {
        ready = false;
        w[j] = load(base(j) + i);
      }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int j = 0; j < W; ++j) out[j] = j == rank ? own : __uint_as_float((unsigned)w[j]);
}

// gather_sum over N elements of a lane at once: every first load of the N x (W-1) words is
// issued before the first wait, so the N round trips overlap instead of serialising (the MLP
// exchange epilogues hold 4 elements per lane).  v[n] holds the own value on entry and the
// rank-ordered sum on return for act[n]; inactive elements are left as they are.
//
// Split form (first_loads + finish_sum_n): the exchanges issue their first polls BEFORE their
// own pushes.  CDNA counts a wave's stores and loads in ONE in-order vmcnt, so a load issued
// after a store cannot be consumed until that store is acknowledged -- for a push into a
// peer's memory a full round trip, paid on top of the peer data's own one-way arrival.
template <int W, int N, class Base>
__device__ __forceinline__ void first_loads(Base base, const size_t (&off)[N], const bool (&act)[N],
                                            int rank, unsigned epoch, u64 (&w)[N][W]) {
  const u64 done = (u64)epoch << 32;
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int j = 0; j < W; ++j) w[n][j] = (act[n] && j != rank) ? load(base(j) + off[n]) : done;
}
template <int W, int N, class Base>
__device__ __forceinline__ void finish_sum_n(Base base, const size_t (&off)[N],
                                             const bool (&act)[N], int rank, unsigned epoch,
                                             u64 (&w)[N][W], float (&v)[N], long long ticks,
                                             bool& fail) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
      for (int j = 0; j < W; ++j)
        if ((unsigned)(w[n][j] >> 32) != epoch) {
          ready = false;
          w[n][j] = load(base(j) + off[n]);
        }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    if (!act[n]) continue;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < W; ++j) acc += j == rank ? v[n] : __uint_as_float((unsigned)w[n][j]);
    v[n] = acc;
  }
}
// All-gather counterpart of finish_sum_n: out[n][j] = peer j's value (out[n][rank] = own[n]).
template <int W, int N, class Base>
__device__ __forceinline__ void finish_all_n(Base base, const size_t (&off)[N],
                                             const bool (&act)[N], int rank, unsigned epoch,
                                             u64 (&w)[N][W], const float (&own)[N],
                                             float (&out)[N][W], long long ticks, bool& fail) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
      for (int j = 0; j < W; ++j)
        if ((unsigned)(w[n][j] >> 32) != epoch) {
          ready = false;
          w[n][j] = load(base(j) + off[n]);
        }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int j = 0; j < W; ++j) out[n][j] = j == rank ? own[n] : __uint_as_float((unsigned)w[n][j]);
}
template <int W, int N, class Base>
__device__ __forceinline__ void gather_sum_n(Base base, const size_t (&off)[N], const bool (&act)[N],
                                             int rank, unsigned epoch, float (&v)[N],
                                             long long ticks, bool& fail) {
  const u64 done = (u64)epoch << 32;
  u64 w[N][W];
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int j = 0; j < W; ++j) w[n][j] = (act[n] && j != rank) ? load(base(j) + off[n]) : done;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
      for (int j = 0; j < W; ++j)
        if ((unsigned)(w[n][j] >> 32) != epoch) {
          ready = false;
          w[n][j] = load(base(j) + off[n]);
        }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int n = 0; n < N; ++n) {
    if (!act[n]) continue;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < W; ++j) acc += j == rank ? v[n] : __uint_as_float((unsigned)w[n][j]);
    v[n] = acc;
  }
}

// wait_n in split form (first polls issued before the caller's pushes, see first_loads).
template <int N>
__device__ __forceinline__ void first_loads1(const u64* p, const size_t (&off)[N], const bool (&act)[N],
                                             unsigned epoch, u64 (&w)[N]) {
  const u64 done = (u64)epoch << 32;
#pragma unroll
  for (int n = 0; n < N; ++n) w[n] = act[n] ? load(p + off[n]) : done;
}
template <int N>
__device__ __forceinline__ void finish_wait_n(const u64* p, const size_t (&off)[N],
                                              const bool (&act)[N], unsigned epoch, u64 (&w)[N],
                                              float (&v)[N], long long ticks, bool& fail) {
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int n = 0; n < N; ++n)
      if ((unsigned)(w[n] >> 32) != epoch) {
        ready = false;
        w[n] = load(p + off[n]);
      }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int n = 0; n < N; ++n)
    if (act[n]) v[n] = __uint_as_float((unsigned)w[n]);
}

// wait_one over N words at once (first loads issued together); v[n] = the word's value.
template <int N>
__device__ __forceinline__ void wait_n(const u64* p, const size_t (&off)[N], const bool (&act)[N],
                                       unsigned epoch, float (&v)[N], long long ticks, bool& fail) {
  const u64 done = (u64)epoch << 32;
  u64 w[N];
#pragma unroll
  for (int n = 0; n < N; ++n) w[n] = act[n] ? load(p + off[n]) : done;
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  for (;;) {
    bool ready = true;
#pragma unroll
    for (int n = 0; n < N; ++n)
      if ((unsigned)(w[n] >> 32) != epoch) {
        ready = false;
        w[n] = load(p + off[n]);
      }
    if (ready) break;
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
#pragma unroll
  for (int n = 0; n < N; ++n)
    if (act[n]) v[n] = __uint_as_float((unsigned)w[n]);
}

__device__ __forceinline__ float wait_one(const u64* p, unsigned epoch, long long ticks,
                                          bool& fail) {
  u64 w = load(p);
  const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
  while ((unsigned)(w >> 32) != epoch) {
    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      fail = true;
      return 0.f;
    }
    __builtin_amdgcn_s_sleep(1);
    w = load(p);
  }
  return __uint_as_float((unsigned)w);
}

}  // namespace xgll
}  // namespace dtfx
