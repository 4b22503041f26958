// Python bindings of the gfx950 kernel launchers (module `_hip`).
//
// The binding deliberately takes raw device addresses and a hipStream_t handle
// (Python passes tensor.data_ptr() and torch.cuda.current_stream().cuda_stream)
// instead of including torch headers: the module then builds in seconds, has
// no C++ ABI coupling to the torch build, and every launch lands on whatever
// stream the caller is on, including a stream under hipGraph capture.
// Shape/dtype/device validation lives in the Python wrappers
// (distributedtensorflowexample_amd/ops/).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace dtfx {
void mlp_fwd_launch(const float*, const float*, float, float*, const float*, float*, int,
                    hipStream_t, unsigned long long*);
void mlp_head_launch(const float*, const float*, float, float*, const int*, float*, int,
                     hipStream_t, unsigned long long*);
void mlp_wgrad_launch(float*, float, float*, const float*, float*, int*, float*, int, int,
                      hipStream_t, unsigned long long*);
long long mlp_workspace_floats(int);
void mlp_ps_stage(const float*, const int*, float*, int*, int, hipStream_t);
void mlp_ps_worker_step(float*, const float*, float*, const float*, const int*, float*, int*,
                        float*, float*, int*, float*, int, const float*, int, float*, float*,
                        hipStream_t);
void mlp_tf_layout_launch(const float*, float*, int, const float*, int, hipStream_t);
void mlp_fwdapply_launch(const float*, float*, float, const float*, const float*, float*, int*,
                         float*, int, int, int, hipStream_t, int);
void mlp_head2_launch(const float*, const int*, float*, int, hipStream_t, int);
int mlp_single_ks_query();
int mlp_set_flush_fused(int on);
void mlp_pipelined_trace_launch(const float*, float*, float, const float*, const float*,
                                const int*, float*, int*, float*, int, int, hipStream_t,
                                unsigned long long*, unsigned long long*);
void mlp_run_pipelined_launch(float*, float*, int, int, float, const float*, const int*, int, int,
                              int, float*, int*, float*, int, int, hipStream_t, int);
void mlp_apply_launch(const float*, float*, float, const float*, float*, int*, float*, int, int,
                      hipStream_t);
long long mlp_persistent_ll_words();
int mlp_persistent_blocks();
int mlp_persistent_trace_steps();
void mlp_persistent_launch(float*, const float*, const int*, int, int, int, float, unsigned,
                           unsigned long long*, int*, float*, int, int, long long,
                           unsigned long long*, hipStream_t);
void calib_launch(int, int, int, const int*, const float*, float*, hipStream_t);
void clock_probe_launch(int, int, unsigned long long*, float*, hipStream_t);
void gemm_f32_launch(bool, bool, int, int, int, float, const float*, int, const float*, int,
                     float, float*, int, const float*, int, const float*, int, bool, hipStream_t);
void colsum_launch(int, int, const float*, int, float, float*, hipStream_t);
void softmax_xent_launch(int, int, const float*, int, const int*, const float*, int, int, float,
                         float*, float*, int, float*, float*, hipStream_t);
void sgd_launch(long long, float*, const float*, float, const float*, float, hipStream_t);
void momentum_launch(long long, float*, const float*, float*, float, const float*, float, float,
                     bool, hipStream_t);
void adam_launch(long long, float*, const float*, float*, float*, float, const float*, float,
                 float, float, float, bool, int, const int*, hipStream_t);
void scale_launch(long long, float*, float, hipStream_t);
void counter_add_launch(int*, int, hipStream_t);
void philox_init_launch(long long, float*, unsigned long long, unsigned long long, int, float,
                        float, hipStream_t);
void act_bwd_launch(long long, int, const float*, const float*, float*, hipStream_t);
void act_fwd_launch(long long, int, const float*, float*, hipStream_t);
}  // namespace dtfx

void register_rccl(py::module_& m);
void register_nn(py::module_& m);
void register_xgmi(py::module_& m);
void register_gpu_ps(py::module_& m);

template <typename T>
static inline T* P(uintptr_t a) { return reinterpret_cast<T*>(a); }
static inline hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

PYBIND11_MODULE(_hip, m) {
  m.doc() = "gfx950 HIP kernels of distributedtensorflowexample_amd";
  m.attr("ARCH") = "gfx950";

  m.def("mlp_workspace_floats", &dtfx::mlp_workspace_floats);
  m.def("mlp_tf_layout", [](uintptr_t src, uintptr_t dst, int to_tf, uintptr_t xsrc, int extra,
                            uintptr_t s) {
    dtfx::mlp_tf_layout_launch(P<const float>(src), P<float>(dst), to_tf, P<const float>(xsrc),
                               extra, S(s));
  });
  m.def("mlp_ps_worker_step", [](uintptr_t p, uintptr_t pulled_host, uintptr_t pull_dev,
                                 uintptr_t x_host, uintptr_t y_host, uintptr_t x_dev,
                                 uintptr_t y_dev, uintptr_t grad, uintptr_t ws, uintptr_t ctr,
                                 uintptr_t stats, int ring, uintptr_t record, int B,
                                 uintptr_t grad_dev, uintptr_t grad_host, uintptr_t s) {
    dtfx::mlp_ps_worker_step(P<float>(p), P<const float>(pulled_host), P<float>(pull_dev),
                             P<const float>(x_host), P<const int>(y_host), P<float>(x_dev),
                             P<int>(y_dev), P<float>(grad), P<float>(ws), P<int>(ctr),
                             P<float>(stats), ring, P<const float>(record), B, P<float>(grad_dev),
                             P<float>(grad_host), S(s));
  }, py::call_guard<py::gil_scoped_release>(),
     "async-PS worker step: staged batch + pulled params (TF layout) in, TF-layout gradient "
     "+ loss/accuracy record out, one call (train/worker.py)");
  m.def("mlp_ps_stage", [](uintptr_t x_host, uintptr_t y_host, uintptr_t x_dev, uintptr_t y_dev,
                           int B, uintptr_t s) {
    dtfx::mlp_ps_stage(P<const float>(x_host), P<const int>(y_host), P<float>(x_dev),
                       P<int>(y_dev), B, S(s));
  });
  m.def("mlp_fwd", [](uintptr_t p_old, uintptr_t grad, float lr, uintptr_t p_new, uintptr_t x,
                      uintptr_t ws, int B, uintptr_t s, uintptr_t tr) {
    dtfx::mlp_fwd_launch(P<const float>(p_old), P<const float>(grad), lr, P<float>(p_new),
                         P<const float>(x), P<float>(ws), B, S(s), P<unsigned long long>(tr));
  }, py::arg("p_old"), py::arg("grad"), py::arg("lr"), py::arg("p_new"), py::arg("x"),
     py::arg("ws"), py::arg("B"), py::arg("stream"), py::arg("trace") = 0);
  m.def("mlp_head", [](uintptr_t p_old, uintptr_t grad, float lr, uintptr_t p_new, uintptr_t lab,
                       uintptr_t ws, int B, uintptr_t s, uintptr_t tr) {
    dtfx::mlp_head_launch(P<const float>(p_old), P<const float>(grad), lr, P<float>(p_new),
                          P<const int>(lab), P<float>(ws), B, S(s), P<unsigned long long>(tr));
  }, py::arg("p_old"), py::arg("grad"), py::arg("lr"), py::arg("p_new"), py::arg("labels"),
     py::arg("ws"), py::arg("B"), py::arg("stream"), py::arg("trace") = 0);
  m.def("mlp_wgrad", [](uintptr_t p, float lr, uintptr_t grad, uintptr_t x, uintptr_t ws,
                        uintptr_t ctr, uintptr_t stats, int ring, int B, uintptr_t s,
                        uintptr_t tr) {
    dtfx::mlp_wgrad_launch(P<float>(p), lr, P<float>(grad), P<const float>(x), P<float>(ws),
                           P<int>(ctr), P<float>(stats), ring, B, S(s), P<unsigned long long>(tr));
  }, py::arg("p"), py::arg("lr"), py::arg("grad"), py::arg("x"), py::arg("ws"), py::arg("ctr"),
     py::arg("stats"), py::arg("ring"), py::arg("B"), py::arg("stream"), py::arg("trace") = 0);
  m.def("mlp_fwdapply", [](uintptr_t p_old, uintptr_t p_new, float lr, uintptr_t x_prev,
                           uintptr_t x, uintptr_t ws, uintptr_t ctr, uintptr_t stats, int ring,
                           int B, int stats_on, uintptr_t s, int ks) {
    dtfx::mlp_fwdapply_launch(P<const float>(p_old), P<float>(p_new), lr, P<const float>(x_prev),
                              P<const float>(x), P<float>(ws), P<int>(ctr), P<float>(stats), ring,
                              B, stats_on, S(s), ks);
  }, py::arg("p_old"), py::arg("p_new"), py::arg("lr"), py::arg("x_prev"), py::arg("x"),
     py::arg("ws"), py::arg("ctr"), py::arg("stats"), py::arg("ring"), py::arg("B"),
     py::arg("stats_on"), py::arg("stream"), py::arg("ks") = 0,
     "first launch of the 2-launch step; ks: K slices (0: the single-GPU setting, 14, 28)");
  m.def("mlp_single_ks", &dtfx::mlp_single_ks_query,
        "K slices of the single-GPU pipelined MLP step (28, or 14 with DTFX_MLP_KS=14)");
  m.def("mlp_pipelined_trace", [](uintptr_t p_old, uintptr_t p_new, float lr, uintptr_t x_prev,
                                   uintptr_t x, uintptr_t lab, uintptr_t ws, uintptr_t ctr,
                                   uintptr_t stats, int ring, int B, uintptr_t s, uintptr_t trf,
                                   uintptr_t trh) {
    dtfx::mlp_pipelined_trace_launch(P<const float>(p_old), P<float>(p_new), lr,
                                     P<const float>(x_prev), P<const float>(x), P<const int>(lab),
                                     P<float>(ws), P<int>(ctr), P<float>(stats), ring, B, S(s),
                                     reinterpret_cast<unsigned long long*>(trf),
                                     reinterpret_cast<unsigned long long*>(trh));
  });
  m.def("mlp_head2", [](uintptr_t p, uintptr_t lab, uintptr_t ws, int B, uintptr_t s, int nslab) {
    dtfx::mlp_head2_launch(P<const float>(p), P<const int>(lab), P<float>(ws), B, S(s), nslab);
  }, py::arg("p"), py::arg("labels"), py::arg("ws"), py::arg("B"), py::arg("stream"),
     py::arg("nslab") = 0,
     "head of the 2-launch step; nslab: slabs the first launch wrote (0: the single-GPU "
     "step's, 14: every data-parallel engine's)");
  m.def("mlp_run_pipelined", [](uintptr_t p0, uintptr_t p1, int cur, int pending, float lr,
                                uintptr_t x, uintptr_t lab, int nbatches, int pos, int n,
                                uintptr_t ws, uintptr_t ctr, uintptr_t stats, int ring, int B,
                                uintptr_t s, int flush) {
    py::gil_scoped_release nogil;
    dtfx::mlp_run_pipelined_launch(P<float>(p0), P<float>(p1), cur, pending, lr, P<const float>(x),
                                   P<const int>(lab), nbatches, pos, n, P<float>(ws), P<int>(ctr),
                                   P<float>(stats), ring, B, S(s), flush);
  }, py::arg("p0"), py::arg("p1"), py::arg("cur"), py::arg("pending"), py::arg("lr"), py::arg("x"),
     py::arg("labels"), py::arg("nbatches"), py::arg("pos"), py::arg("n"), py::arg("ws"),
     py::arg("ctr"), py::arg("stats"), py::arg("ring"), py::arg("B"), py::arg("stream"),
     py::arg("flush") = 0);
  m.def("mlp_set_flush_fused", &dtfx::mlp_set_flush_fused,
        "run_launched(.., flush=True): 1 = the last step's head and the flush in one launch "
        "(mlp_head_flush_kernel; opt-in, measured slower), 0 = the flush as its own launch; "
        "returns the previous setting");
  // The C++ host loop with its fixed arguments bound once (FusedMLPTrainer.run_launched): a
  // driver-sized timed region starts on the host, so the per-call Python -> C++ argument
  // conversion of the 17-argument form sits in front of the region's first kernel.
  struct MlpRunPlan {
    float *p0, *p1;
    const float* x;
    const int* labels;
    int nbatches;
    float* ws;
    int* ctr;
    float* stats;
    int ring, B;
  };
  py::class_<MlpRunPlan>(m, "MlpRunPlan")
      .def(py::init([](uintptr_t p0, uintptr_t p1, uintptr_t x, uintptr_t lab, int nbatches,
                       uintptr_t ws, uintptr_t ctr, uintptr_t stats, int ring, int B) {
        return MlpRunPlan{P<float>(p0), P<float>(p1), P<const float>(x), P<const int>(lab),
                          nbatches, P<float>(ws), P<int>(ctr), P<float>(stats), ring, B};
      }))
      .def("run", [](const MlpRunPlan& p, int cur, int pending, float lr, int pos, int n,
                     int flush, uintptr_t s) {
        py::gil_scoped_release nogil;
        dtfx::mlp_run_pipelined_launch(p.p0, p.p1, cur, pending, lr, p.x, p.labels, p.nbatches,
                                       pos, n, p.ws, p.ctr, p.stats, p.ring, p.B, S(s), flush);
      }, "(cur, pending, lr, pos, n, flush, stream): mlp_run_pipelined with the bound buffers");
  m.def("mlp_apply", [](uintptr_t p_old, uintptr_t p_new, float lr, uintptr_t x_prev, uintptr_t ws,
                        uintptr_t ctr, uintptr_t stats, int ring, int B, uintptr_t s) {
    dtfx::mlp_apply_launch(P<const float>(p_old), P<float>(p_new), lr, P<const float>(x_prev),
                           P<float>(ws), P<int>(ctr), P<float>(stats), ring, B, S(s));
  });
  m.def("mlp_persistent_ll_words", &dtfx::mlp_persistent_ll_words);
  m.def("mlp_persistent_blocks", &dtfx::mlp_persistent_blocks);
  m.def("mlp_persistent_trace_steps", &dtfx::mlp_persistent_trace_steps);
  m.def("mlp_persistent", [](uintptr_t p, uintptr_t x, uintptr_t lab, int nbatches, int pos,
                             int steps, float lr, unsigned ebase, uintptr_t ll, uintptr_t ctr,
                             uintptr_t stats, int ring, int B, long long ticks, uintptr_t s,
                             uintptr_t trace) {
    py::gil_scoped_release nogil;
    dtfx::mlp_persistent_launch(P<float>(p), P<const float>(x), P<const int>(lab), nbatches, pos,
                                steps, lr, ebase, P<unsigned long long>(ll), P<int>(ctr),
                                P<float>(stats), ring, B, ticks, P<unsigned long long>(trace),
                                S(s));
  }, py::arg("p"), py::arg("x"), py::arg("labels"), py::arg("nbatches"), py::arg("pos"),
     py::arg("steps"), py::arg("lr"), py::arg("ebase"), py::arg("ll"), py::arg("ctr"),
     py::arg("stats"), py::arg("ring"), py::arg("B"), py::arg("ticks"), py::arg("stream"),
     py::arg("trace") = 0);
  m.def("gemm_f32", [](bool ta, bool tb, int M, int N, int K, float alpha, uintptr_t A, int lda,
                       uintptr_t B, int ldb, float beta, uintptr_t C, int ldc, uintptr_t bias,
                       int act, uintptr_t aux, int ldaux, bool act_grad, uintptr_t s) {
    dtfx::gemm_f32_launch(ta, tb, M, N, K, alpha, P<const float>(A), lda, P<const float>(B), ldb,
                          beta, P<float>(C), ldc, P<const float>(bias), act, P<const float>(aux),
                          ldaux, act_grad, S(s));
  });
  m.def("colsum", [](int M, int N, uintptr_t G, int ldg, float beta, uintptr_t out, uintptr_t s) {
    dtfx::colsum_launch(M, N, P<const float>(G), ldg, beta, P<float>(out), S(s));
  });
  m.def("softmax_xent", [](int N, int C, uintptr_t logits, int ldl, uintptr_t lab_idx,
                           uintptr_t lab_dense, int ldy, int ignore, float scale, uintptr_t loss,
                           uintptr_t dlogits, int ldd, uintptr_t correct, uintptr_t probs,
                           uintptr_t s) {
    dtfx::softmax_xent_launch(N, C, P<const float>(logits), ldl, P<const int>(lab_idx),
                              P<const float>(lab_dense), ldy, ignore, scale, P<float>(loss),
                              P<float>(dlogits), ldd, P<float>(correct), P<float>(probs), S(s));
  });
  m.def("sgd", [](long long n, uintptr_t p, uintptr_t g, float lr, uintptr_t lr_ptr, float wd,
                  uintptr_t s) {
    dtfx::sgd_launch(n, P<float>(p), P<const float>(g), lr, P<const float>(lr_ptr), wd, S(s));
  });
  m.def("momentum", [](long long n, uintptr_t p, uintptr_t g, uintptr_t v, float lr,
                       uintptr_t lr_ptr, float mu, float wd, bool nesterov, uintptr_t s) {
    dtfx::momentum_launch(n, P<float>(p), P<const float>(g), P<float>(v), lr,
                          P<const float>(lr_ptr), mu, wd, nesterov, S(s));
  });
  m.def("adam", [](long long n, uintptr_t p, uintptr_t g, uintptr_t mm, uintptr_t v, float lr,
                   uintptr_t lr_ptr, float b1, float b2, float eps, float wd, bool adamw, int step,
                   uintptr_t step_ptr, uintptr_t s) {
    dtfx::adam_launch(n, P<float>(p), P<const float>(g), P<float>(mm), P<float>(v), lr,
                      P<const float>(lr_ptr), b1, b2, eps, wd, adamw, step, P<const int>(step_ptr),
                      S(s));
  });
  m.def("scale", [](long long n, uintptr_t x, float a, uintptr_t s) {
    dtfx::scale_launch(n, P<float>(x), a, S(s));
  });
  m.def("counter_add", [](uintptr_t c, int d, uintptr_t s) {
    dtfx::counter_add_launch(P<int>(c), d, S(s));
  });
  m.def("philox_init", [](long long n, uintptr_t out, unsigned long long seed,
                          unsigned long long offset, int mode, float a, float b, uintptr_t s) {
    dtfx::philox_init_launch(n, P<float>(out), seed, offset, mode, a, b, S(s));
  });
  m.def("act_bwd", [](long long n, int act, uintptr_t dy, uintptr_t sv, uintptr_t dz,
                      uintptr_t s) {
    dtfx::act_bwd_launch(n, act, P<const float>(dy), P<const float>(sv), P<float>(dz), S(s));
  });
  m.def("act_fwd", [](long long n, int act, uintptr_t x, uintptr_t y, uintptr_t s) {
    dtfx::act_fwd_launch(n, act, P<const float>(x), P<float>(y), S(s));
  });
  m.def("calib", [](int mode, int grid, int block, uintptr_t ctr, uintptr_t data, uintptr_t out,
                    uintptr_t s) {
    dtfx::calib_launch(mode, grid, block, P<const int>(ctr), P<const float>(data), P<float>(out),
                       S(s));
  });
  m.def("clock_probe", [](int iters, int grid, uintptr_t out2, uintptr_t sink, uintptr_t s) {
    dtfx::clock_probe_launch(iters, grid, P<unsigned long long>(out2), P<float>(sink), S(s));
  });
  register_rccl(m);
  register_nn(m);
  register_xgmi(m);
  register_gpu_ps(m);
  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
  });
}
