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

enum { XG_LL_PULL = 0, XG_LL_PUSH = 1, XG_LL_PUSH2 = 2, XG_BW = 3 };

// bytes of one rank's LL / BW data region (the flag array follows it)
long long xgmi_ll_bytes(int mode, int world, long long S);

// bandwidth-mode two-shot all-reduce for large buckets (f32 payload + release flags)
void xgmi_bw_launch(float* g, long long n, int rank, int world, long long S, const XgPeers& peers,
                    unsigned* epochs, int* err, long long ticks, hipStream_t stream,
                    int blocks, const int* abort_word, int op = 0);

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
  // exchange work split (DTFX_XG_SPLIT, default 51): bit 0 -- mlp_fwdapply_kernel's W1 slices
  // over both K-split waves; bit 1 -- the small parameters' dW2 over two waves (A/B probes);
  // bit 4 -- the pair exchanges' polls as 16-byte buffer loads, pushes as global stores;
  // bit 5 -- the factor first launch's global W1 gradient in row-quad form (fx_phase_a_quads)
  int split;
};
constexpr int MLP_XG_EPOCHS = 1024;
// epoch slots of the factor engine (mlp_head_kernel<.., XW> rows / mlp_wgrad_factor_kernel's
// small-parameter waves; also the pipelined fused engine's); mlp_wgrad_kernel<.., XW> and
// mlp_fwdapply_kernel<.., XW> use [0, 392) (never on the same communicator)
constexpr int MLP_XG_SMALL_EPOCH = 400;
constexpr int MLP_XG_HEAD_EPOCH = 512;

// Factor engine (sufficient-factor exchange): head launch that all-gathers the backprop
// factors dz1 of every rank into dz1A [world][112][BP], then the weight-gradient launch that
// forms the global dW1 from them and every rank's (resident) batch x, applying directly.
void mlp_head_xg_launch(const float* p, const int* labels, float* ws, float* dz1A, int B,
                        hipStream_t stream, const MlpXg& xg, int world, int nslab = 7);
// Pipelined factor engine: step t-1's global W1 update (from dz1A and every rank's x_prev)
// fused with step t's forward (head of step t: mlp_head_xg_launch with nslab = 14).
void mlp_fwdapply_factor_launch(const float* p_old, float* p_new, float lr, const float* x_prev,
                                const float* x, long long xstride, const float* dz1A, float* ws,
                                int* ctr, float* stats, int stats_ring, int B, int stats_on,
                                hipStream_t stream, const MlpXg& xg, int world);
void mlp_wgrad_factor_launch(float* p, float lr, const float* x, long long xstride,
                             const float* dz1A, float* ws, int* ctr, float* stats, int stats_ring,
                             int B, hipStream_t stream, const MlpXg& xg, int world);

// Pipelined fused engine: step t-1's local W1/W2/b gradient tiles exchanged and applied
// (p_old -> p_new) in the launch that runs step t's forward; the head is the plain one.
// two_shot: the W1 tiles' exchange as reduce-scatter + all-gather (xg_exchange2): 2 (W-1)/W
// words per element per rank instead of W-1 (needs the push layout's result region)
void mlp_fwdapply_xg_launch(const float* p_old, float* p_new, float lr, const float* x_prev,
                            const float* x, float* ws, int* ctr, float* stats, int stats_ring,
                            int B, int stats_on, hipStream_t stream, const MlpXg& xg, int world,
                            int two_shot = 0, unsigned long long* trace = nullptr);

void mlp_wgrad_xg_launch(float* p, float lr, const float* x, float* ws, int* ctr, float* stats,
                         int stats_ring, int B, hipStream_t stream, const MlpXg& xg, int world);
// plain head of the pipelined step (mlp_step.hip); nslab = 28 after the fused engines' launch
void mlp_head2_launch(const float* p, const int* labels, float* ws, int B, hipStream_t stream,
                      int nslab);

}  // namespace dtfx
