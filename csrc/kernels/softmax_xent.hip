// Fused softmax cross-entropy, forward + backward + accuracy, one wave per row.
//
// TF semantics of tf.nn.softmax_cross_entropy_with_logits (worker.py:63-64):
// per-row loss = -sum_c y_c log softmax(l)_c and the op's backprop output
// (softmax - y), here pre-scaled by `scale` (1/B folds in the reduce_mean of
// worker.py:66).  Labels are either dense [N][C] (TF's one-hot/soft labels) or
// int class indices (ignore_index < 0 disables a row: MLM masking).  The
// accuracy of worker.py:89-90 (argmax(softmax) == argmax(y), first max wins)
// is fused in: argmax(softmax(l)) = argmax(l).
#include "common.h"

#include <stdexcept>

namespace dtfx {

__global__ __launch_bounds__(256) void softmax_xent_kernel(
    int N, int C, const float* __restrict__ logits, int ldl, const int* __restrict__ lab_idx,
    const float* __restrict__ lab_dense, int ldy, int ignore_index, float scale,
    float* __restrict__ loss, float* __restrict__ dlogits, int ldd, float* __restrict__ correct,
    float* __restrict__ probs) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const float* l = logits + (size_t)row * ldl;

  // max + argmax of the logits (lowest index on ties)
  float m = -INFINITY;
  int am = 0x7fffffff;
  for (int c = lane; c < C; c += 64) {
    const float v = l[c];
    if (v > m) { m = v; am = c; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64);
    const int oa = __shfl_xor(am, o, 64);
    if (om > m || (om == m && oa < am)) { m = om; am = oa; }
  }
  float se = 0.f;
  for (int c = lane; c < C; c += 64) se += __expf(l[c] - m);
  se = wave_sum(se);
  const float lse = m + __logf(se);

  int yi = -1;
  bool valid = true;
  float ysum = 1.f;
  float lossv = 0.f;
  if (lab_idx) {
    yi = lab_idx[row];
    valid = !(ignore_index < 0 ? false : yi == ignore_index) && yi >= 0 && yi < C;
    lossv = valid ? (lse - l[yi]) : 0.f;
  } else {
    const float* y = lab_dense + (size_t)row * ldy;
    float s = 0.f, ys = 0.f, ym = -INFINITY;
    int ya = 0x7fffffff;
    for (int c = lane; c < C; c += 64) {
      const float yc = y[c];
      s += yc * (lse - l[c]);
      ys += yc;
      if (yc > ym) { ym = yc; ya = c; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float om = __shfl_xor(ym, o, 64);
      const int oa = __shfl_xor(ya, o, 64);
      if (om > ym || (om == ym && oa < ya)) { ym = om; ya = oa; }
    }
    lossv = wave_sum(s);
    ysum = wave_sum(ys);
    yi = ya;
  }
  if (lane == 0) {
    if (loss) loss[row] = lossv;
    if (correct) correct[row] = valid ? ((am == yi) ? 1.f : 0.f) : 0.f;
  }
  const float inv = 1.f / se;
  for (int c = lane; c < C; c += 64) {
    const float p = __expf(l[c] - m) * inv;
    if (probs) probs[(size_t)row * C + c] = p;
    if (dlogits) {
      float g;
      if (lab_idx) g = valid ? (p - (c == yi ? 1.f : 0.f)) : 0.f;
      else g = p * ysum - lab_dense[(size_t)row * ldy + c];
      dlogits[(size_t)row * ldd + c] = g * scale;
    }
  }
}

void softmax_xent_launch(int N, int C, const float* logits, int ldl, const int* lab_idx,
                         const float* lab_dense, int ldy, int ignore_index, float scale,
                         float* loss, float* dlogits, int ldd, float* correct, float* probs,
                         hipStream_t stream) {
  if (N <= 0) return;
  if ((lab_idx == nullptr) == (lab_dense == nullptr))
    throw std::runtime_error("softmax_xent: exactly one of int / dense labels");
  hipLaunchKernelGGL(softmax_xent_kernel, dim3((N + 3) / 4), dim3(256), 0, stream, N, C, logits,
                     ldl, lab_idx, lab_dense, ldy, ignore_index, scale, loss, dlogits, ldd,
                     correct, probs);
  DTFX_HIP_CHECK(hipGetLastError());
}

}  // namespace dtfx
