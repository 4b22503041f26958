// Python bindings of the bf16 north-star kernels (BERT-base / ResNet-50 path):
// registered into module `_hip` by bindings.cpp.  Same conventions: raw device
// addresses + a hipStream_t handle; validation in distributedtensorflowexample_amd/ops/.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

namespace py = pybind11;

namespace dtfx {
void gemm_bf16_set_cfg(int);
int gemm_bf16_set_pers(int);
void attn_bwd_set_variant(int);
void attn_bwd_set_pf(int);
void ln_bwd_set_slots(int);
void xent_set_regs(int);
void ln_bwd_set_h768(int);
void attn_set_swizzle(int);
void attn_fwd_set_variant(int);
void transpose_bf16_batch_launch(const long long*, int, int, hipStream_t);
void gemm_bf16_launch(bool, bool, bool, int, int, int, const void*, int, const void*, int, void*,
                      int, float, float, const float*, int, const void*, void*, int, const void*,
                      int, int, int, int, long long, long long, long long,
                      float*, hipStream_t, float*, long long, bool);
void colsum_bf16_launch(const void*, int, int, int, float*, float, hipStream_t);
void colsum_set_rows_in_flight(int);
long long gemm_bf16_ws_floats(bool, bool, int, int, int, int, float);
long long conv_wgrad_ws_floats(int, int, int, int, int, int, int, int, int);
long long conv_splitk_ws_floats(int, int, int, int, int, int, int, int, int, int);
void conv_bf16_launch(int, int, int, int, int, int, int, int, int, int, const void*, const void*, int,
                      void*, float, const void*, float*, float*, int, hipStream_t, const void*,
                      const void*, const float*, const float*, float*, long long, int);
void bn_bwd_apply_launch(long long, int, const void*, const void*, const float*, const float*,
                         const float*, const float*, const float*, void*, hipStream_t);
void bn_finalize_launch(int, long long, const float*, const float*, float, float*, float*, float*,
                        float*, float, hipStream_t);
void bn_apply_launch(long long, int, const void*, const float*, const float*, const float*,
                     const float*, const void*, int, void*, hipStream_t);
void bn_apply_stats_launch(long long, int, const void*, const float*, const float*, float, float*,
                           float*, float*, float*, float, const float*, const float*, const void*,
                           int, void*, const float*, const float*, const float*, const float*,
                           float*, float*, float*, float*, hipStream_t);
void bn_bwd_launch(long long, int, const void*, const void*, const void*, const float*, const float*,
                   const float*, int, float*, float*, float*, void*, void*, hipStream_t);
long long bn_bwd_scratch_rows(long long, int);
void colpart_reduce_launch(int, int, const float*, const float*, float*, float*, hipStream_t);
bool stem_conv_applies(int, int, int, int, int, int, int, int);
int stem_conv_fwd_rows(int, int, int);
void stem_conv_fwd_launch(int, int, int, const void*, const void*, int, void*, float*, float*,
                          hipStream_t);
void stem_conv_wgrad_launch(int, int, int, const void*, const void*, float*, int, float,
                            hipStream_t, const void*, const float*);
bool conv3x3_c64_applies(int, int, int, int, int, int, int, int);
void conv3x3_c64_fwd_launch(int, int, int, const void*, const void*, int, void*, float*, float*,
                            hipStream_t, const float* = nullptr, void* = nullptr);
void conv3x3_c64_wgrad_launch(int, int, int, const void*, const void*, float*, int, float,
                              hipStream_t);
void conv3x3_c64_dgrad_launch(int, int, int, const void*, const void*, int, void*, const void*,
                              const void*, const float*, const float*, float*, float*, void*, hipStream_t);
bool conv3x3_c128_applies(int, int, int, int, int, int, int, int);
bool conv1x1_applies(int, int, int);
int conv1x1_rows(int, int, int, int);
void conv1x1_launch(int, int, int, int, const void*, const void*, int, void*, const void*,
                    const void*, const void*, const float*, const float*, float*, float*, void*,
                    hipStream_t);
bool conv1x1_pro_applies(int, int, int, int);
void conv1x1_pro_launch(int, int, int, int, const void*, const void*, const float*, void*,
                        const void*, int, void*, const void*, const void*, const void*,
                        const float*, const float*, float*, float*, void*, hipStream_t,
                        int = 0, int = 0);
void conv1x1_pro_fwdbn_launch(int, int, int, int, const void*, const void*, long long,
                              const float*, const float*, float, float*, float*, float*, float*,
                              float, const float*, const float*, const float*, const float*,
                              const float*, const float*, float*, float*, float*, float*, void*,
                              const void*, int, void*, float*, float*, hipStream_t);
void conv1x1_pro_bwdbn_launch(int, int, int, const void*, const void*, long long, const float*,
                              const float*, const float*, const float*, const float*, void*,
                              const void*, int, void*, const void*, const void*, const void*,
                              const float*, const float*, float*, float*, void*, hipStream_t, int,
                              int);
void bn_fwd_coef_launch(long long, int, const float*, const float*, float, float*, float*, float*,
                        float*, float, const float*, const float*, const float*, const float*,
                        const float*, const float*, float*, float*, float*, float*, float*,
                        hipStream_t);
void bn_bwd_coef_launch(long long, int, const float*, const float*, const float*, const float*,
                        const float*, float*, hipStream_t);
void conv3x3_c128_launch(int, int, int, int, const void*, const void*, int, void*, void*,
                         const void*, const void*, const float*, const float*, float*, float*,
                         hipStream_t);
void maxpool_fwd_launch(int, int, int, int, const void*, void*, void*, hipStream_t);
void maxpool_bn_fwd_launch(int, int, int, int, const void*, const float*, void*, void*, hipStream_t);
int maxpool_bn_bwd_rows(int, int, int, int);
void maxpool_bn_bwd_launch(int, int, int, int, const void*, const void*, const void*, const float*,
                           const float*, const float*, const float*, float*, float*, float*,
                           void*, void*, float*, hipStream_t);
void maxpool_bwd_launch(int, int, int, int, const void*, const void*, void*, hipStream_t);
void avgpool_fwd_launch(int, int, int, const void*, void*, hipStream_t);
void avgpool_bwd_launch(int, int, int, const void*, void*, hipStream_t);
void sgd_momentum_mixed_launch(long long, float*, const float*, float*, void*, float, float, float,
                               float, hipStream_t, const long long*, int);
void layernorm_fwd_launch(int, int, const void*, const float*, const float*, float, void*, float*,
                          float*, hipStream_t);
void layernorm_bwd_launch(int, int, const void*, const void*, const float*, const float*,
                          const float*, const void*, void*, float*, float*, float*, hipStream_t);
void embed_ln_fwd_launch(int, int, int, const int*, const int*, const void*, const void*,
                         const void*, const float*, const float*, float, void*, void*, float*,
                         float*, hipStream_t);
void embed_bwd_launch(int, int, int, const int*, const int*, const void*, float*, float*, float*,
                      hipStream_t);
void attn_fwd_launch(int, int, int, const void*, void*, float*, const float*, float, hipStream_t);
void attn_bwd_launch(int, int, int, const void*, const void*, const void*, const float*,
                     const float*, float, void*, float*, hipStream_t);
void adam_mixed_launch(long long, float*, const float*, float*, float*, void*, float, float, float,
                       float, float, float, const int*, int, hipStream_t, const long long*, int,
                       long long);
void cast_f32_bf16_launch(long long, const float*, void*, hipStream_t);
void zero_ranges_launch(const long long*, int, long long, hipStream_t);
void act_grad_bf16_launch(long long, int, const void*, const void*, void*, hipStream_t);
void flash_fwd_launch(int, int, int, const void*, void*, float*, int, const float*, float,
                      hipStream_t);
void flash_bwd_launch(int, int, int, const void*, const void*, const void*, const float*, int,
                      const float*, float, void*, float*, float*, hipStream_t);
void mlm_xent_launch(int, int, const void*, bool, int, const int*, float, float*, float*, void*, int,
                     hipStream_t);
}  // namespace dtfx

template <typename T>
static inline T* P(uintptr_t a) { return reinterpret_cast<T*>(a); }
static inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

void register_nn(py::module_& m) {
  m.def("attn_set_swizzle", &dtfx::attn_set_swizzle,
        "attention LDS images: -1 = environment (DTFX_ATTN_SWZ), 0 = padded rows, 1 = swizzled");
  m.def("attn_bwd_set_variant", &dtfx::attn_bwd_set_variant,
        "force the attention-backward kernel (-1 = environment; 0: 8 waves, 1: 4 waves, "
        "2: two query halves, two blocks per CU)");
  m.def("colsum_set_rows_in_flight", &dtfx::colsum_set_rows_in_flight,
        "bf16 column sums: rows in flight per thread, 4 or 8 (0 = from DTFX_COLSUM_U)");
  m.def("xent_set_regs", &dtfx::xent_set_regs,
        "bf16 MLM cross-entropy: 1 = the row held in registers (one read of the logits), "
        "0 = the two-pass kernel, -1 = from DTFX_XENT_REGS");
  m.def("ln_bwd_set_h768", &dtfx::ln_bwd_set_h768,
        "LayerNorm backward at H = 768: 1 = the 12-columns-per-lane kernel (two blocks per CU), "
        "0 = the generic one, -1 = from DTFX_LN_H768");
  m.def("ln_bwd_set_slots", &dtfx::ln_bwd_set_slots,
        "LayerNorm backward row slots per wave: 2 (default) or 3 (one more row in flight), "
        "-1 = from DTFX_LN_SLOTS");
  m.def("attn_bwd_set_pf", &dtfx::attn_bwd_set_pf,
        "two-halves attention backward: 1 = V rows requested at block start (L2 warm-up, "
        "opt-in, measured slower), 0 = not (default), -1 = from DTFX_ATTN_BWD_PF");
  m.def("attn_fwd_set_variant", &dtfx::attn_fwd_set_variant,
        "attention forward: 1 = P in registers (attn_fwd_rp_kernel, default), 0 = P through "
        "LDS (attn_fwd_kernel), -1 = from DTFX_ATTN_FWD");
  m.def("gemm_bf16_set_pers", &dtfx::gemm_bf16_set_pers,
        "1: plain 8-phase GEMMs with more 256x256 tiles than CUs run the persistent tile loop "
        "(opt-in, measured slower), 0: one block per tile (default); returns the previous "
        "setting");
  m.def("gemm_bf16_set_cfg", &dtfx::gemm_bf16_set_cfg,
        "force the bf16 GEMM tile configuration (-1 = auto; 0: 128x128, 3: 256x256 2-stage, "
        "5: 256x256 8-phase)");
  m.def("gemm_bf16", [](bool ta, bool tb, bool out_f32, int M, int N, int K, uintptr_t A, int lda,
                        uintptr_t B, int ldb, uintptr_t C, int ldc, float alpha, float beta,
                        uintptr_t bias, int act, uintptr_t aux_in, uintptr_t aux_out, int ld_aux,
                        uintptr_t residual, int ld_res, int act_grad, int splitk, int batch, long long sA,
                        long long sB, long long sC, uintptr_t colsum, uintptr_t s, uintptr_t ws,
                        long long ws_floats, bool defer_reduce) {
    dtfx::gemm_bf16_launch(ta, tb, out_f32, M, N, K, P<const void>(A), lda, P<const void>(B), ldb,
                           P<void>(C), ldc, alpha, beta, P<const float>(bias), act,
                           P<const void>(aux_in), P<void>(aux_out), ld_aux, P<const void>(residual),
                           ld_res, act_grad, splitk, batch, sA, sB, sC,
                           P<float>(colsum), S(s), P<float>(ws), ws_floats, defer_reduce);
  }, py::arg("ta"), py::arg("tb"), py::arg("out_f32"), py::arg("M"), py::arg("N"), py::arg("K"),
     py::arg("A"), py::arg("lda"), py::arg("B"), py::arg("ldb"), py::arg("C"), py::arg("ldc"),
     py::arg("alpha") = 1.f, py::arg("beta") = 0.f, py::arg("bias") = 0, py::arg("act") = 0,
     py::arg("aux_in") = 0, py::arg("aux_out") = 0, py::arg("ld_aux") = 0,
     py::arg("residual") = 0, py::arg("ld_res") = 0, py::arg("act_grad") = 0,
     py::arg("splitk") = 0, py::arg("batch") = 1, py::arg("sA") = 0, py::arg("sB") = 0,
     py::arg("sC") = 0, py::arg("colsum") = 0, py::arg("stream") = 0, py::arg("ws") = 0,
     py::arg("ws_floats") = 0, py::arg("defer_reduce") = false);
  m.def("gemm_bf16_ws_floats", &dtfx::gemm_bf16_ws_floats,
        "f32 elements of split-K workspace gemm_bf16 would use (0: no split-K)");
  m.def("conv_splitk_ws_floats", &dtfx::conv_splitk_ws_floats,
        "f32 elements of split-K workspace a forward (mode 1) / stride-1 data-gradient (mode 2) "
        "conv_bf16 would use (0: no split-K)");
  m.def("conv_wgrad_ws_floats", &dtfx::conv_wgrad_ws_floats,
        "f32 elements of split-K workspace a conv weight gradient would use (0: no split-K)");
  m.def("colsum_bf16", [](uintptr_t G, int M, int N, int ldg, uintptr_t out, float beta,
                          uintptr_t s) {
    dtfx::colsum_bf16_launch(P<const void>(G), M, N, ldg, P<float>(out), beta, S(s));
  });
  m.def("layernorm_fwd", [](int T, int H, uintptr_t x, uintptr_t g, uintptr_t b, float eps,
                            uintptr_t y, uintptr_t mean, uintptr_t rstd, uintptr_t s) {
    dtfx::layernorm_fwd_launch(T, H, P<const void>(x), P<const float>(g), P<const float>(b), eps,
                               P<void>(y), P<float>(mean), P<float>(rstd), S(s));
  });
  m.def("layernorm_bwd", [](int T, int H, uintptr_t dy, uintptr_t x, uintptr_t mean,
                            uintptr_t rstd, uintptr_t g, uintptr_t dres, uintptr_t dx,
                            uintptr_t dg, uintptr_t db, uintptr_t dxsum, uintptr_t s) {
    dtfx::layernorm_bwd_launch(T, H, P<const void>(dy), P<const void>(x), P<const float>(mean),
                               P<const float>(rstd), P<const float>(g), P<const void>(dres),
                               P<void>(dx), P<float>(dg), P<float>(db), P<float>(dxsum), S(s));
  });
  m.def("embed_ln_fwd", [](int T, int Sq, int H, uintptr_t ids, uintptr_t tt, uintptr_t word,
                           uintptr_t pos, uintptr_t type, uintptr_t g, uintptr_t b, float eps,
                           uintptr_t xsum, uintptr_t y, uintptr_t mean, uintptr_t rstd,
                           uintptr_t s) {
    dtfx::embed_ln_fwd_launch(T, Sq, H, P<const int>(ids), P<const int>(tt), P<const void>(word),
                              P<const void>(pos), P<const void>(type), P<const float>(g),
                              P<const float>(b), eps, P<void>(xsum), P<void>(y), P<float>(mean),
                              P<float>(rstd), S(s));
  });
  m.def("embed_bwd", [](int Bn, int Sq, int H, uintptr_t ids, uintptr_t tt, uintptr_t dx,
                        uintptr_t dword, uintptr_t dpos, uintptr_t dtype_, uintptr_t s) {
    dtfx::embed_bwd_launch(Bn, Sq, H, P<const int>(ids), P<const int>(tt), P<const void>(dx),
                           P<float>(dword), P<float>(dpos), P<float>(dtype_), S(s));
  });
  m.def("attn_fwd", [](int Bn, int Sq, int nh, uintptr_t qkv, uintptr_t out, uintptr_t lse,
                       uintptr_t kmask, float scale, uintptr_t s) {
    dtfx::attn_fwd_launch(Bn, Sq, nh, P<const void>(qkv), P<void>(out), P<float>(lse),
                          P<const float>(kmask), scale, S(s));
  });
  m.def("attn_bwd", [](int Bn, int Sq, int nh, uintptr_t qkv, uintptr_t o, uintptr_t dout,
                       uintptr_t lse, uintptr_t kmask, float scale, uintptr_t dqkv,
                       uintptr_t dbias, uintptr_t s) {
    dtfx::attn_bwd_launch(Bn, Sq, nh, P<const void>(qkv), P<const void>(o), P<const void>(dout),
                          P<const float>(lse), P<const float>(kmask), scale, P<void>(dqkv),
                          P<float>(dbias), S(s));
  });
  m.def("adam_mixed", [](long long n, uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v,
                         uintptr_t pb, float lr, float b1, float b2, float eps, float wd,
                         float gscale, uintptr_t step_ptr, int step, uintptr_t s, uintptr_t segs,
                         int nseg, long long base4) {
    dtfx::adam_mixed_launch(n, P<float>(p), P<const float>(g), P<float>(mm), P<float>(v),
                            P<void>(pb), lr, b1, b2, eps, wd, gscale, P<const int>(step_ptr), step,
                            S(s), P<const long long>(segs), nseg, base4);
  }, py::arg("n"), py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("pb"),
     py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"),
     py::arg("gscale"), py::arg("step_ptr"), py::arg("step"), py::arg("stream"),
     py::arg("segs") = 0, py::arg("nseg") = 0, py::arg("base4") = 0);
  m.def("zero_ranges", [](uintptr_t tab, int n, long long total, uintptr_t s) {
    dtfx::zero_ranges_launch(P<const long long>(tab), n, total, S(s));
  }, "zero n f32 ranges in one launch: int64 table [n][3] {pointer, length, prefix}");
  m.def("cast_f32_bf16", [](long long n, uintptr_t x, uintptr_t y, uintptr_t s) {
    dtfx::cast_f32_bf16_launch(n, P<const float>(x), P<void>(y), S(s));
  });
  m.def("act_grad_bf16", [](long long n, int act, uintptr_t dy, uintptr_t u, uintptr_t dx,
                            uintptr_t s) {
    dtfx::act_grad_bf16_launch(n, act, P<const void>(dy), P<const void>(u), P<void>(dx), S(s));
  });
  m.def("mlm_xent", [](int N, int C, uintptr_t logits, int ldl, uintptr_t labels, float scale,
                       uintptr_t loss, uintptr_t correct, uintptr_t dl, int ldd, uintptr_t s,
                       bool logits_bf16) {
    dtfx::mlm_xent_launch(N, C, P<const void>(logits), logits_bf16, ldl, P<const int>(labels), scale,
                          P<float>(loss), P<float>(correct), P<void>(dl), ldd, S(s));
  }, py::arg("N"), py::arg("C"), py::arg("logits"), py::arg("ldl"), py::arg("labels"),
     py::arg("scale"), py::arg("loss"), py::arg("correct"), py::arg("dl"), py::arg("ldd"),
     py::arg("s"), py::arg("logits_bf16") = false);
  m.def("conv_bf16", [](int mode, int N, int H, int W, int C, int Cout, int KH, int KW, int stride,
                        int pad, uintptr_t a, uintptr_t b, int ldw, uintptr_t out, float beta,
                        uintptr_t residual, uintptr_t colsum, uintptr_t colsq, int splitk,
                        uintptr_t s, uintptr_t relu_y, uintptr_t bn_x, uintptr_t bn_mean,
                        uintptr_t bn_rstd, uintptr_t ws, long long ws_floats, bool defer) {
    dtfx::conv_bf16_launch(mode, N, H, W, C, Cout, KH, KW, stride, pad, P<const void>(a),
                           P<const void>(b), ldw, P<void>(out), beta, P<const void>(residual),
                           P<float>(colsum), P<float>(colsq), splitk, S(s),
                           P<const void>(relu_y), P<const void>(bn_x), P<const float>(bn_mean),
                           P<const float>(bn_rstd), P<float>(ws), ws_floats, defer ? 1 : 0);
  }, py::arg("mode"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("Cout"),
     py::arg("KH"), py::arg("KW"), py::arg("stride"), py::arg("pad"), py::arg("a"), py::arg("b"),
     py::arg("ldw"), py::arg("out"), py::arg("beta"), py::arg("residual"), py::arg("colsum"),
     py::arg("colsq"), py::arg("splitk"), py::arg("stream"), py::arg("relu_y") = 0,
     py::arg("bn_x") = 0, py::arg("bn_mean") = 0, py::arg("bn_rstd") = 0, py::arg("ws") = 0,
     py::arg("ws_floats") = 0, py::arg("defer_reduce") = false);
  m.def("bn_bwd_apply", [](long long M, int C, uintptr_t de, uintptr_t x, uintptr_t mean,
                           uintptr_t rstd, uintptr_t g, uintptr_t sdy, uintptr_t sdyxh,
                           uintptr_t dx, uintptr_t s) {
    dtfx::bn_bwd_apply_launch(M, C, P<const void>(de), P<const void>(x), P<const float>(mean),
                              P<const float>(rstd), P<const float>(g), P<const float>(sdy),
                              P<const float>(sdyxh), P<void>(dx), S(s));
  });
  m.def("bn_finalize", [](int C, long long M, uintptr_t s_, uintptr_t q, float eps, uintptr_t mean,
                          uintptr_t rstd, uintptr_t rm, uintptr_t rv, float momentum, uintptr_t s) {
    dtfx::bn_finalize_launch(C, M, P<const float>(s_), P<const float>(q), eps, P<float>(mean),
                             P<float>(rstd), P<float>(rm), P<float>(rv), momentum, S(s));
  });
  m.def("bn_apply", [](long long M, int C, uintptr_t x, uintptr_t mean, uintptr_t rstd,
                       uintptr_t g, uintptr_t b, uintptr_t res, int relu, uintptr_t y, uintptr_t s) {
    dtfx::bn_apply_launch(M, C, P<const void>(x), P<const float>(mean), P<const float>(rstd),
                          P<const float>(g), P<const float>(b), P<const void>(res), relu, P<void>(y),
                          S(s));
  });
  m.def("bn_apply_stats", [](long long M, int C, uintptr_t x, uintptr_t sum, uintptr_t sq, float eps,
                             uintptr_t mean, uintptr_t rstd, uintptr_t run_mean, uintptr_t run_var,
                             float momentum, uintptr_t g, uintptr_t b, uintptr_t res, int relu,
                             uintptr_t y, uintptr_t sum2, uintptr_t sq2, uintptr_t g2, uintptr_t b2,
                             uintptr_t mean2, uintptr_t rstd2, uintptr_t run_mean2,
                             uintptr_t run_var2, uintptr_t s) {
    dtfx::bn_apply_stats_launch(M, C, P<const void>(x), P<const float>(sum), P<const float>(sq), eps,
                                P<float>(mean), P<float>(rstd), P<float>(run_mean), P<float>(run_var),
                                momentum, P<const float>(g), P<const float>(b), P<const void>(res),
                                relu, P<void>(y), P<const float>(sum2), P<const float>(sq2),
                                P<const float>(g2), P<const float>(b2), P<float>(mean2),
                                P<float>(rstd2), P<float>(run_mean2), P<float>(run_var2), S(s));
  });
  m.def("bn_bwd", [](long long M, int C, uintptr_t dy, uintptr_t yout, uintptr_t x, uintptr_t mean,
                     uintptr_t rstd, uintptr_t g, int relu, uintptr_t sdy, uintptr_t sdyxh,
                     uintptr_t scratch, uintptr_t dx, uintptr_t dres, uintptr_t s) {
    dtfx::bn_bwd_launch(M, C, P<const void>(dy), P<const void>(yout), P<const void>(x),
                        P<const float>(mean), P<const float>(rstd), P<const float>(g), relu,
                        P<float>(sdy), P<float>(sdyxh), P<float>(scratch), P<void>(dx),
                        P<void>(dres), S(s));
  });
  m.def("bn_bwd_scratch_rows", &dtfx::bn_bwd_scratch_rows);
  m.def("stem_conv_fwd_rows", &dtfx::stem_conv_fwd_rows,
        "(N, OH, OW): partial statistics rows stem_conv_fwd writes ([rows][64] each)");
  m.def("stem_conv_applies", &dtfx::stem_conv_applies,
        "the ResNet stem kernel handles this conv (7x7/2, pad 3, 8 -> 64 channels, OH % 8, OW % 16)");
  m.def("stem_conv_fwd", [](int N, int H, int W, uintptr_t x, uintptr_t w, int ldw, uintptr_t y,
                            uintptr_t ps, uintptr_t pq, uintptr_t s) {
    dtfx::stem_conv_fwd_launch(N, H, W, P<const void>(x), P<const void>(w), ldw, P<void>(y),
                               P<float>(ps), P<float>(pq), S(s));
  });
  m.def("stem_conv_wgrad", [](int N, int H, int W, uintptr_t x, uintptr_t dy, uintptr_t dw, int ldw,
                              float beta, uintptr_t s, uintptr_t bnx, uintptr_t coef) {
    dtfx::stem_conv_wgrad_launch(N, H, W, P<const void>(x), P<const void>(dy), P<float>(dw), ldw,
                                 beta, S(s), P<const void>(bnx), P<const float>(coef));
  }, py::arg("N"), py::arg("H"), py::arg("W"), py::arg("x"), py::arg("dy"), py::arg("dw"),
     py::arg("ldw"), py::arg("beta"), py::arg("stream"), py::arg("bnx") = 0, py::arg("coef") = 0);
  m.def("conv3x3_c64_applies", &dtfx::conv3x3_c64_applies,
        "the 64-channel 3x3 kernel handles this conv (stride 1, pad 1, H % 4, W % 28)");
  m.def("conv3x3_c64_fwd", [](int N, int H, int W, uintptr_t x, uintptr_t w, int ldw, uintptr_t y,
                              uintptr_t ps, uintptr_t pq, uintptr_t s, uintptr_t coef, uintptr_t xo) {
    dtfx::conv3x3_c64_fwd_launch(N, H, W, P<const void>(x), P<const void>(w), ldw, P<void>(y),
                                 P<float>(ps), P<float>(pq), S(s), P<const float>(coef), P<void>(xo));
  }, py::arg("N"), py::arg("H"), py::arg("W"), py::arg("x"), py::arg("w"), py::arg("ldw"),
     py::arg("y"), py::arg("ps"), py::arg("pq"), py::arg("s"), py::arg("coef") = 0,
     py::arg("xo") = 0, "coef / xo: relu(bn(x)) formed in the patch staging and written to xo");
  m.def("conv3x3_c64_wgrad", [](int N, int H, int W, uintptr_t x, uintptr_t dy, uintptr_t dw,
                                int ldw, float beta, uintptr_t s) {
    dtfx::conv3x3_c64_wgrad_launch(N, H, W, P<const void>(x), P<const void>(dy), P<float>(dw), ldw,
                                   beta, S(s));
  });
  m.def("conv3x3_c64_dgrad", [](int N, int H, int W, uintptr_t dy, uintptr_t w, int ldw,
                                uintptr_t dx, uintptr_t relu_y, uintptr_t bn_x, uintptr_t mean,
                                uintptr_t rstd, uintptr_t ps, uintptr_t pq, uintptr_t wf, uintptr_t s) {
    dtfx::conv3x3_c64_dgrad_launch(N, H, W, P<const void>(dy), P<const void>(w), ldw, P<void>(dx),
                                   P<const void>(relu_y), P<const void>(bn_x), P<const float>(mean),
                                   P<const float>(rstd), P<float>(ps), P<float>(pq), P<void>(wf),
                                   S(s));
  }, "wf: [64][576] bf16 workspace for the flipped weights");
  m.def("conv1x1_applies", &dtfx::conv1x1_applies,
        "(M, K, N): the streaming 1x1 kernel takes this product (K 64 / 128, N = 256 * 2^i)");
  m.def("conv1x1_rows", &dtfx::conv1x1_rows, "(mode, M, K, N): partial statistics rows a launch writes");
  m.def("conv1x1", [](int mode, int M, int K, int N, uintptr_t x, uintptr_t w, int ldw,
                      uintptr_t y, uintptr_t res, uintptr_t relu_y, uintptr_t bn_x, uintptr_t mean,
                      uintptr_t rstd, uintptr_t ps, uintptr_t pq, uintptr_t wt, uintptr_t s) {
    dtfx::conv1x1_launch(mode, M, K, N, P<const void>(x), P<const void>(w), ldw, P<void>(y),
                         P<const void>(res), P<const void>(relu_y), P<const void>(bn_x),
                         P<const float>(mean), P<const float>(rstd), P<float>(ps), P<float>(pq),
                         P<void>(wt), S(s));
  });
  m.def("transpose_bf16_batch", [](uintptr_t tab, int n, int tiles, uintptr_t s) {
    dtfx::transpose_bf16_batch_launch(P<const long long>(tab), n, tiles, S(s));
  }, "n bf16 transposes in one launch: int64 table [n][6] {src, dst, rows, cols, ld_src, first "
     "32x32 tile}; a 1x1 dgrad given w = 0 reads such a copy from wt");
  m.def("conv1x1_pro_applies", &dtfx::conv1x1_pro_applies,
        "(mode, M, K, N): a 1x1 kernel with the BatchNorm prologue takes this product");
  m.def("conv1x1_pro", [](int mode, int M, int K, int N, uintptr_t s0, uintptr_t s1, uintptr_t coef,
                          uintptr_t xo, uintptr_t w, int ldw, uintptr_t y, uintptr_t res,
                          uintptr_t relu_y, uintptr_t bn_x, uintptr_t mean, uintptr_t rstd,
                          uintptr_t ps, uintptr_t pq, uintptr_t wt, uintptr_t s, int res_h,
                          int res_w) {
    dtfx::conv1x1_pro_launch(mode, M, K, N, P<const void>(s0), P<const void>(s1),
                             P<const float>(coef), P<void>(xo), P<const void>(w), ldw, P<void>(y),
                             P<const void>(res), P<const void>(relu_y), P<const void>(bn_x),
                             P<const float>(mean), P<const float>(rstd), P<float>(ps), P<float>(pq),
                             P<void>(wt), S(s), res_h, res_w);
  }, py::arg("mode"), py::arg("M"), py::arg("K"), py::arg("N"), py::arg("s0"), py::arg("s1"),
     py::arg("coef"), py::arg("xo"), py::arg("w"), py::arg("ldw"), py::arg("y"), py::arg("res"),
     py::arg("relu_y"), py::arg("bn_x"), py::arg("mean"), py::arg("rstd"), py::arg("ps"),
     py::arg("pq"), py::arg("wt"), py::arg("s"), py::arg("res_h") = 0, py::arg("res_w") = 0,
     "res_h / res_w (mode 2, wide): the residual is a stride-2 conv's data gradient stored "
     "compact [pixels / 4][N] for an res_h x res_w grid (zero at odd rows / columns)");
  m.def("conv1x1_pro_fwdbn", [](int mode, int M, int K, int N, uintptr_t s0, uintptr_t s1,
                                long long Mst, uintptr_t sum, uintptr_t sq, float eps,
                                uintptr_t mean, uintptr_t rstd, uintptr_t run_mean,
                                uintptr_t run_var, float momentum, uintptr_t g, uintptr_t b,
                                uintptr_t sum2, uintptr_t sq2, uintptr_t g2, uintptr_t b2,
                                uintptr_t mean2, uintptr_t rstd2, uintptr_t run_mean2,
                                uintptr_t run_var2, uintptr_t xo, uintptr_t w, int ldw,
                                uintptr_t y, uintptr_t ps, uintptr_t pq, uintptr_t s) {
    dtfx::conv1x1_pro_fwdbn_launch(
        mode, M, K, N, P<const void>(s0), P<const void>(s1), Mst, P<const float>(sum),
        P<const float>(sq), eps, P<float>(mean), P<float>(rstd), P<float>(run_mean),
        P<float>(run_var), momentum, P<const float>(g), P<const float>(b), P<const float>(sum2),
        P<const float>(sq2), P<const float>(g2), P<const float>(b2), P<float>(mean2),
        P<float>(rstd2), P<float>(run_mean2), P<float>(run_var2), P<void>(xo), P<const void>(w),
        ldw, P<void>(y), P<float>(ps), P<float>(pq), S(s));
  }, "conv1x1_pro mode 1 / 3 with the BatchNorm coefficients formed in the kernel from the "
     "BN's column sums and affine (bn_fwd_coef's outputs written by block 0): no coefficient "
     "launch");
  m.def("conv1x1_pro_bwdbn", [](int M, int K, int N, uintptr_t s0, uintptr_t s1, long long Mst,
                                uintptr_t bmean, uintptr_t brstd, uintptr_t g, uintptr_t sum_dy,
                                uintptr_t sum_dyxh, uintptr_t xo, uintptr_t w, int ldw,
                                uintptr_t y, uintptr_t res, uintptr_t relu_y, uintptr_t bn_x,
                                uintptr_t mean, uintptr_t rstd, uintptr_t ps, uintptr_t pq,
                                uintptr_t wt, uintptr_t s, int res_h, int res_w) {
    dtfx::conv1x1_pro_bwdbn_launch(
        M, K, N, P<const void>(s0), P<const void>(s1), Mst, P<const float>(bmean),
        P<const float>(brstd), P<const float>(g), P<const float>(sum_dy),
        P<const float>(sum_dyxh), P<void>(xo), P<const void>(w), ldw, P<void>(y),
        P<const void>(res), P<const void>(relu_y), P<const void>(bn_x), P<const float>(mean),
        P<const float>(rstd), P<float>(ps), P<float>(pq), P<void>(wt), S(s), res_h, res_w);
  }, py::arg("M"), py::arg("K"), py::arg("N"), py::arg("s0"), py::arg("s1"), py::arg("Mst"),
     py::arg("bmean"), py::arg("brstd"), py::arg("gamma"), py::arg("sum_dy"),
     py::arg("sum_dyxh"), py::arg("xo"), py::arg("w"), py::arg("ldw"), py::arg("y"),
     py::arg("res"), py::arg("relu_y"), py::arg("bn_x"), py::arg("mean"), py::arg("rstd"),
     py::arg("ps"), py::arg("pq"), py::arg("wt"), py::arg("s"), py::arg("res_h") = 0,
     py::arg("res_w") = 0,
     "conv1x1_pro mode 2 with BatchNorm backward's coefficients formed in the kernel from "
     "mean / rstd / gamma and the final reductions: no coefficient launch");
  m.def("bn_fwd_coef", [](long long M, int C, uintptr_t sum, uintptr_t sq, float eps, uintptr_t mean,
                          uintptr_t rstd, uintptr_t run_mean, uintptr_t run_var, float momentum,
                          uintptr_t g, uintptr_t b, uintptr_t sum2, uintptr_t sq2, uintptr_t g2,
                          uintptr_t b2, uintptr_t mean2, uintptr_t rstd2, uintptr_t run_mean2,
                          uintptr_t run_var2, uintptr_t coef, uintptr_t s) {
    dtfx::bn_fwd_coef_launch(M, C, P<const float>(sum), P<const float>(sq), eps, P<float>(mean),
                             P<float>(rstd), P<float>(run_mean), P<float>(run_var), momentum,
                             P<const float>(g), P<const float>(b), P<const float>(sum2),
                             P<const float>(sq2), P<const float>(g2), P<const float>(b2),
                             P<float>(mean2), P<float>(rstd2), P<float>(run_mean2),
                             P<float>(run_var2), P<float>(coef), S(s));
  });
  m.def("bn_bwd_coef", [](long long M, int C, uintptr_t mean, uintptr_t rstd, uintptr_t g,
                          uintptr_t sdy, uintptr_t sdyxh, uintptr_t coef, uintptr_t s) {
    dtfx::bn_bwd_coef_launch(M, C, P<const float>(mean), P<const float>(rstd), P<const float>(g),
                             P<const float>(sdy), P<const float>(sdyxh), P<float>(coef), S(s));
  });
  m.def("maxpool_bn_fwd", [](int N, int H, int W, int C, uintptr_t x, uintptr_t fcoef, uintptr_t y,
                             uintptr_t idx, uintptr_t s) {
    dtfx::maxpool_bn_fwd_launch(N, H, W, C, P<const void>(x), P<const float>(fcoef), P<void>(y),
                                P<void>(idx), S(s));
  });
  m.def("maxpool_bn_bwd_rows", &dtfx::maxpool_bn_bwd_rows);
  m.def("maxpool_bn_bwd", [](int N, int H, int W, int C, uintptr_t dy, uintptr_t idx, uintptr_t x,
                             uintptr_t fcoef, uintptr_t mean, uintptr_t rstd, uintptr_t g,
                             uintptr_t sdy, uintptr_t sdyxh, uintptr_t scratch, uintptr_t de,
                             uintptr_t dx, uintptr_t bcoef, uintptr_t s) {
    dtfx::maxpool_bn_bwd_launch(N, H, W, C, P<const void>(dy), P<const void>(idx), P<const void>(x),
                                P<const float>(fcoef), P<const float>(mean), P<const float>(rstd),
                                P<const float>(g), P<float>(sdy), P<float>(sdyxh),
                                P<float>(scratch), P<void>(de), P<void>(dx), P<float>(bcoef), S(s));
  });
  m.def("conv3x3_c128_applies", &dtfx::conv3x3_c128_applies,
        "the 128-channel 3x3 kernel handles this conv (stride 1, pad 1, H % 4, W % 28)");
  m.def("conv3x3_c128", [](int mode, int N, int H, int W, uintptr_t x, uintptr_t w, int ldw,
                           uintptr_t y, uintptr_t wf, uintptr_t relu_y, uintptr_t bn_x,
                           uintptr_t mean, uintptr_t rstd, uintptr_t ps, uintptr_t pq, uintptr_t s) {
    dtfx::conv3x3_c128_launch(mode, N, H, W, P<const void>(x), P<const void>(w), ldw, P<void>(y),
                              P<void>(wf), P<const void>(relu_y), P<const void>(bn_x),
                              P<const float>(mean), P<const float>(rstd), P<float>(ps),
                              P<float>(pq), S(s));
  });
  m.def("colpart_reduce", [](int R, int C, uintptr_t ps, uintptr_t pq, uintptr_t os, uintptr_t oq,
                             uintptr_t s) {
    dtfx::colpart_reduce_launch(R, C, P<const float>(ps), P<const float>(pq), P<float>(os),
                                P<float>(oq), S(s));
  });
  m.def("maxpool_fwd", [](int N, int H, int W, int C, uintptr_t x, uintptr_t y, uintptr_t idx,
                          uintptr_t s) {
    dtfx::maxpool_fwd_launch(N, H, W, C, P<const void>(x), P<void>(y), P<void>(idx), S(s));
  });
  m.def("maxpool_bwd", [](int N, int H, int W, int C, uintptr_t dy, uintptr_t idx, uintptr_t dx,
                          uintptr_t s) {
    dtfx::maxpool_bwd_launch(N, H, W, C, P<const void>(dy), P<const void>(idx), P<void>(dx), S(s));
  });
  m.def("avgpool_fwd", [](int N, int HW, int C, uintptr_t x, uintptr_t y, uintptr_t s) {
    dtfx::avgpool_fwd_launch(N, HW, C, P<const void>(x), P<void>(y), S(s));
  });
  m.def("avgpool_bwd", [](int N, int HW, int C, uintptr_t dy, uintptr_t dx, uintptr_t s) {
    dtfx::avgpool_bwd_launch(N, HW, C, P<const void>(dy), P<void>(dx), S(s));
  });
  m.def("sgd_momentum_mixed", [](long long n, uintptr_t p, uintptr_t g, uintptr_t v, uintptr_t pb,
                                 float lr, float mu, float wd, float gscale, uintptr_t s,
                                 uintptr_t segs, int nseg) {
    dtfx::sgd_momentum_mixed_launch(n, P<float>(p), P<const float>(g), P<float>(v), P<void>(pb), lr,
                                    mu, wd, gscale, S(s), P<const long long>(segs), nseg);
  }, py::arg("n"), py::arg("p"), py::arg("g"), py::arg("v"), py::arg("pb"), py::arg("lr"),
     py::arg("mu"), py::arg("wd"), py::arg("gscale"), py::arg("s"), py::arg("segs") = 0,
     py::arg("nseg") = 0,
     "segs (int64 [nseg][5]: lo4, hi4, planes, plane stride in float4s, S): ranges whose "
     "gradient is the sum of S split-K planes (conv_bf16 defer_reduce), summed here");
  m.def("flash_fwd", [](int Bn, int Sq, int nh, uintptr_t qkv, uintptr_t out, uintptr_t lse,
                        int ld_lse, uintptr_t kmask, float scale, uintptr_t s) {
    dtfx::flash_fwd_launch(Bn, Sq, nh, P<const void>(qkv), P<void>(out), P<float>(lse), ld_lse,
                           P<const float>(kmask), scale, S(s));
  });
  m.def("flash_bwd", [](int Bn, int Sq, int nh, uintptr_t qkv, uintptr_t o, uintptr_t dout,
                        uintptr_t lse, int ld_lse, uintptr_t kmask, float scale, uintptr_t dqkv,
                        uintptr_t dbias, uintptr_t scratch, uintptr_t s) {
    dtfx::flash_bwd_launch(Bn, Sq, nh, P<const void>(qkv), P<const void>(o), P<const void>(dout),
                           P<const float>(lse), ld_lse, P<const float>(kmask), scale, P<void>(dqkv),
                           P<float>(dbias), P<float>(scratch), S(s));
  });
}
