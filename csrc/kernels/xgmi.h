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

// Gradient exchange fused into the MNIST-MLP weight-gradient kernel (mlp_step.hip): every
// lane pushes its gradient elements as LL words into slot[me] of every peer (push layout
// [2][W][S] words per rank), gathers the peers' words for the same elements from local
// memory, sums in rank order and applies SGD -- the all-reduce costs no extra launch.
struct MlpXg {
  XgPeers peers;
  long long S;          // slot stride (elements)
  int rank;
  unsigned* epochs;     // one counter per (block, wave) of the kernel, device resident
  int* err;             // set on a timed-out wait
  long long ticks;      // wait bound in s_memrealtime ticks (100 MHz)
};
constexpr int MLP_XG_EPOCHS = 1024;

void mlp_wgrad_xg_launch(float* p, float lr, const float* x, float* ws, int* ctr, float* stats,
                         int stats_ring, int B, hipStream_t stream, const MlpXg& xg, int world);

}  // namespace dtfx
