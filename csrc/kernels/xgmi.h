// Shared declarations of the xGMI one-shot all-reduce (kernel in xgmi_allreduce.hip,
// host communicator + bindings in xgmi_comm.cpp).
#pragma once
#include <hip/hip_runtime.h>

namespace dtfx {

constexpr int XG_MAX_WORLD = 16;
constexpr int XG_BLOCKS = 256;

struct XgPeers {
  float* data[XG_MAX_WORLD];      // each rank's slot base ([2][S] floats)
  unsigned* flags[XG_MAX_WORLD];  // each rank's flag array ([world][XG_BLOCKS])
};

void xgmi_allreduce_launch(float* g, long long n, int rank, int world, long long S,
                           const XgPeers& peers, unsigned* epochs, int* err, long long ticks,
                           hipStream_t stream);

enum { XG_LL_PULL = 0, XG_LL_PUSH = 1, XG_LL_PUSH2 = 2 };

// bytes of one rank's LL data region (the flag array follows it)
long long xgmi_ll_bytes(int mode, int world, long long S);

void xgmi_ll_launch(int mode, float* g, long long n, int rank, int world, long long S,
                    const XgPeers& peers, unsigned* epochs, int* err, long long ticks,
                    hipStream_t stream);

}  // namespace dtfx
