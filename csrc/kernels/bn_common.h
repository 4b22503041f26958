// Training-mode BatchNorm coefficient math shared by the elementwise BatchNorm kernels
// (cnn.hip) and the 1x1 convolutions with a BatchNorm prologue (conv1x1.hip).
#pragma once

#include "common.h"

namespace dtfx {

// Statistics of one BatchNorm from its producer's column sums (see cnn.hip bn_apply_kernel):
// mean = ssum / M, var = ssq / M - mean^2 (biased, for the normalisation), the running
// statistics updated with the unbiased variance (momentum form of tf / keras).
struct BnStats {
  const float* ssum;
  const float* ssq;
  float inv_m, eps, unbias, momentum;
  float* mean_out;
  float* rstd_out;
  float* run_mean;
  float* run_var;
  const float* gamma2;  // st2 only: the residual BN's affine
  const float* beta2;
};
__device__ __forceinline__ void bn_store_stats(const BnStats& st, int c, float mu, float rs) {
  st.mean_out[c] = mu;
  st.rstd_out[c] = rs;
  if (st.run_mean) {
    const float var = fmaxf(st.ssq[c] * st.inv_m - mu * mu, 0.f);
    st.run_mean[c] = st.momentum * st.run_mean[c] + (1.f - st.momentum) * mu;
    st.run_var[c] = st.momentum * st.run_var[c] + (1.f - st.momentum) * var * st.unbias;
  }
}
template <bool STATS>
__device__ __forceinline__ void bn_coef(const BnStats& st, const float* mean, const float* rstd, int c,
                                        float& mu, float& rs) {
  if (STATS) {
    mu = st.ssum[c] * st.inv_m;
    rs = rsqrtf(fmaxf(st.ssq[c] * st.inv_m - mu * mu, 0.f) + st.eps);
  } else {
    mu = mean[c];
    rs = rstd[c];
  }
}

// Per-channel coefficients of a BatchNorm prologue, op = (s0 a + c) + (s1 b + d):
//   rows != null: read from the [4][K] rows bn_fwd_coef / bn_bwd_coef wrote (one launch each);
//   else formed by the consuming block itself (no coefficient launch):
//     forward  a = rstd gamma, c = beta - mean a; residual b = 1, d = 0, or its own BN
//              b = rstd2 gamma2, d = beta2 - mean2 b (st2.ssum set) -- bn_fwd_coef_kernel's
//              arithmetic, so both paths give the same bits;
//     backward bn_bwd_apply's affine form, a = gamma rstd, b = -a rstd s2, c = 0,
//              d = -a s1 + a rstd s2 mean (s1 / s2 = sum_dy / sum_dyxh over M) --
//              bn_bwd_coef_kernel's arithmetic.
// The forward's side duties (mean / rstd for the backward, running statistics) then fall to
// block 0 of the consumer (bn_coef_duty).
struct BnCoefSrc {
  const float* rows;
  int bwd;
  BnStats st, st2;
  const float* gamma;
  const float* beta;
  const float* mean;
  const float* rstd;
  const float* sum_dy;
  const float* sum_dyxh;
  float inv_m;
};
__device__ __forceinline__ void bn_coef_at(const BnCoefSrc& s, int K, int c, float& a, float& b,
                                           float& cc, float& d) {
  if (s.rows) {
    a = s.rows[c];
    b = s.rows[K + c];
    cc = s.rows[2 * K + c];
    d = s.rows[3 * K + c];
    return;
  }
  if (s.bwd) {
    const float A = s.gamma[c] * s.rstd[c], s1 = s.sum_dy[c] * s.inv_m,
                s2 = s.sum_dyxh[c] * s.inv_m;
    a = A;
    b = -A * s.rstd[c] * s2;
    cc = 0.f;
    d = -A * s1 + A * s.rstd[c] * s2 * s.mean[c];
    return;
  }
  float mu, rs;
  bn_coef<true>(s.st, nullptr, nullptr, c, mu, rs);
  a = rs * s.gamma[c];
  cc = s.beta[c] - mu * a;
  b = 1.f;
  d = 0.f;
  if (s.st2.ssum) {
    float mu2, rs2;
    bn_coef<true>(s.st2, nullptr, nullptr, c, mu2, rs2);
    b = rs2 * s.st2.gamma2[c];
    d = s.st2.beta2[c] - mu2 * b;
  }
}
// forward with formed coefficients: mean / rstd (and the residual BN's) stored, running
// statistics updated -- by ONE block (call with blockIdx.x == 0's threads t of n)
__device__ __forceinline__ void bn_coef_duty(const BnCoefSrc& s, int K, int t, int n) {
  if (s.rows || s.bwd) return;
  for (int c = t; c < K; c += n) {
    float mu, rs;
    bn_coef<true>(s.st, nullptr, nullptr, c, mu, rs);
    bn_store_stats(s.st, c, mu, rs);
    if (s.st2.ssum) {
      bn_coef<true>(s.st2, nullptr, nullptr, c, mu, rs);
      bn_store_stats(s.st2, c, mu, rs);
    }
  }
}

}  // namespace dtfx
