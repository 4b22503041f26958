// Host side of the xGMI one-shot all-reduce: IPC-shared uncached slots, peer
// mapping, launch, error word.  Kernel and protocol: xgmi_allreduce.hip.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "xgmi.h"

namespace py = pybind11;

#define XG_CHECK(expr)                                                                 \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +     \
                               " in " #expr);                                          \
  } while (0)

namespace dtfx {

class XgmiAllReduce {
 public:
  // own_slots = false: the slot regions are supplied by open_local() (test harness).
  XgmiAllReduce(int rank, int world, int device, long long max_numel, const std::string& protocol,
                bool own_slots = true)
      : rank_(rank), world_(world), device_(device), S_((max_numel + 63) / 64 * 64) {
    if (protocol == "flag") mode_ = -1;
    else if (protocol == "ll") mode_ = XG_LL_PULL;
    else if (protocol == "push") mode_ = XG_LL_PUSH;
    else if (protocol == "push2") mode_ = XG_LL_PUSH2;
    else if (protocol == "bw") mode_ = XG_BW;
    else throw std::runtime_error("xgmi: protocol must be flag|ll|push|push2|bw");
    if (mode_ >= 0 && world > 8) throw std::runtime_error("xgmi: LL / bw protocols support world <= 8");
    if (world < 1 || world > XG_MAX_WORLD) throw std::runtime_error("xgmi: world must be 1..16");
    XG_CHECK(hipSetDevice(device));
    // ONE fine-grained uncached (MTYPE UC) allocation: data slots [2][S] f32 followed by the
    // flag array (LL protocols: their word regions, see xgmi_allreduce.hip).  UC accesses bypass every GPU cache, so neither side needs L2 writeback /
    // invalidation (a system-scope fence would write back or invalidate the whole L2):
    // ordering alone (vmcnt waits) makes the protocol correct.  Rounded to 2 MiB.
    data_bytes_ = mode_ < 0 ? (long long)sizeof(float) * 2 * S_ : xgmi_ll_bytes(mode_, world, S_);
    bytes_ = data_bytes_ + sizeof(unsigned) * XG_MAX_WORLD * XG_BLOCKS;
    bytes_ = (bytes_ + (2u << 20) - 1) / (2u << 20) * (2u << 20);
    if (own_slots) {
      XG_CHECK(hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocUncached));
      XG_CHECK(hipMemset(base_, 0, bytes_));
    }
    XG_CHECK(hipMalloc(&epochs_, sizeof(unsigned) * XG_BLOCKS + sizeof(int)));
    XG_CHECK(hipMemset(epochs_, 0, sizeof(unsigned) * XG_BLOCKS + sizeof(int)));
    err_ = (int*)(epochs_ + XG_BLOCKS);
    // host-visible abort word (pinned, mapped): abort() sets it with a plain host store -- no
    // HIP call, so the peer watchdog's thread can run it while the stream is blocked -- and
    // the bandwidth kernel's peer waits read it (xgmi_bw_kernel)
    XG_CHECK(hipHostMalloc((void**)&abort_host_, sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    *abort_host_ = 0;
    XG_CHECK(hipHostGetDevicePointer((void**)&abort_dev_, abort_host_, 0));
    XG_CHECK(hipMalloc(&mlp_epochs_, sizeof(unsigned) * MLP_XG_EPOCHS));
    XG_CHECK(hipMemset(mlp_epochs_, 0, sizeof(unsigned) * MLP_XG_EPOCHS));
    for (int i = 0; i < XG_MAX_WORLD; ++i) {
      peers_.data[i] = nullptr;
      peers_.flags[i] = nullptr;
    }
  }
  ~XgmiAllReduce() { close(); }

  size_t region_bytes() const { return bytes_; }
  // bandwidth protocol: workgroups per call (<= XG_BLOCKS).  Fewer leave more CUs to the
  // backward kernels an overlapped all-reduce runs beside; every rank must use the same.
  void set_bw_blocks(int nb) {
    if (nb < 1 || nb > XG_BLOCKS) throw std::runtime_error("xgmi: bw blocks must be 1..256");
    bw_blocks_ = nb;
  }
  long long slot_stride() const { return S_; }

  // Test harness ("peer buffers that are local allocations"): every rank's slot
  // region is a caller-owned allocation of region_bytes() on THIS device, so one process can
  // run any rank's kernels of any world size with the other ranks' words pre-staged.  The
  // kernels and the layout are exactly those of open(); only the pointers' origin differs.
  void open_local(const std::vector<uintptr_t>& regions) {
    if ((int)regions.size() != world_) throw std::runtime_error("xgmi: need one region per rank");
    if (base_) throw std::runtime_error("xgmi: open_local() is for communicators without slots");
    for (int j = 0; j < world_; ++j) {
      if (!regions[j] || (regions[j] & 255)) throw std::runtime_error("xgmi: region must be 256-B aligned");
      peers_.data[j] = (float*)regions[j];
      peers_.flags[j] = (unsigned*)((char*)regions[j] + data_bytes_);
    }
    ready_ = true;
  }

  py::bytes handle() {
    hipIpcMemHandle_t h;
    XG_CHECK(hipIpcGetMemHandle(&h, base_));
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  void open(const std::vector<std::string>& handles) {
    if ((int)handles.size() != world_) throw std::runtime_error("xgmi: need one handle per rank");
    XG_CHECK(hipSetDevice(device_));
    for (int j = 0; j < world_; ++j) {
      char* p;
      if (j == rank_) {
        p = (char*)base_;
      } else {
        hipIpcMemHandle_t h;
        if (handles[j].size() != sizeof(h)) throw std::runtime_error("xgmi: bad handle size");
        memcpy(&h, handles[j].data(), sizeof(h));
        void* q = nullptr;
        XG_CHECK(hipIpcOpenMemHandle(&q, h, hipIpcMemLazyEnablePeerAccess));
        opened_.push_back(q);
        p = (char*)q;
      }
      peers_.data[j] = (float*)p;
      peers_.flags[j] = (unsigned*)(p + data_bytes_);
    }
    ready_ = true;
  }

  void all_reduce(uintptr_t g, long long n, uintptr_t stream, double timeout_s) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (n > S_) throw std::runtime_error("xgmi: buffer larger than max_numel");
    if (g & 15) throw std::runtime_error("xgmi: buffer must be 16-byte aligned");
    const long long ticks = (long long)(timeout_s * 1e8);  // s_memrealtime: 100 MHz
    if (mode_ == XG_BW)
      xgmi_bw_launch((float*)g, n, rank_, world_, S_, peers_, epochs_, err_, ticks,
                     (hipStream_t)stream, bw_blocks_, abort_dev_, 0);
    else if (mode_ >= 0)
      xgmi_ll_launch(mode_, (float*)g, n, rank_, world_, S_, peers_, epochs_, err_, ticks,
                     (hipStream_t)stream);
    else
      xgmi_allreduce_launch((float*)g, n, rank_, world_, S_, peers_, epochs_, err_, ticks,
                            (hipStream_t)stream);
  }

  // In-place halves of the bandwidth two-shot over g[0, n) (n a multiple of 4 x world, so
  // rank r's chunk is exactly [r n / W, (r + 1) n / W)): op 1 reduce-scatter -- chunk r of g
  // becomes the sum over ranks; op 2 all-gather -- every rank's chunk r lands in every g.
  void shard_op(int op, uintptr_t g, long long n, uintptr_t stream, double timeout_s) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (mode_ != XG_BW) throw std::runtime_error("xgmi: reduce-scatter / all-gather need protocol bw");
    if (op != 1 && op != 2) throw std::runtime_error("xgmi: shard op must be 1 or 2");
    if (n > S_) throw std::runtime_error("xgmi: buffer larger than max_numel");
    if (n % (4LL * world_)) throw std::runtime_error("xgmi: shard ops need n % (4 x world) == 0");
    if (g & 15) throw std::runtime_error("xgmi: buffer must be 16-byte aligned");
    xgmi_bw_launch((float*)g, n, rank_, world_, S_, peers_, epochs_, err_,
                   (long long)(timeout_s * 1e8), (hipStream_t)stream, bw_blocks_, abort_dev_, op);
  }

  // MNIST-MLP weight-gradient kernel with the gradient exchange fused into its epilogue
  // (push layout only): p -= lr * sum_over_ranks(grad), one launch.
  void mlp_wgrad(uintptr_t p, float lr, uintptr_t x, uintptr_t ws, uintptr_t ctr, uintptr_t stats,
                 int ring, int B, uintptr_t stream, double timeout_s) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (mode_ != XG_LL_PUSH) throw std::runtime_error("xgmi: the fused MLP exchange needs protocol push");
    MlpXg xg;
    xg.peers = peers_;
    xg.S = S_;
    xg.rank = rank_;
    xg.epochs = mlp_epochs_;
    xg.err = err_;
    xg.ticks = (long long)(timeout_s * 1e8);
    mlp_wgrad_xg_launch((float*)p, lr, (const float*)x, (float*)ws, (int*)ctr, (float*)stats, ring, B,
                        (hipStream_t)stream, xg, world_);
  }

  MlpXg mlp_xg(double timeout_s) const {
    MlpXg xg;
    xg.peers = peers_;
    xg.S = S_;
    xg.rank = rank_;
    xg.epochs = mlp_epochs_;
    xg.err = err_;
    xg.ticks = (long long)(timeout_s * 1e8);
    const char* sp = getenv("DTFX_XG_SPLIT");
    xg.split = sp ? atoi(sp) : 51;
    return xg;
  }

  // Factor engine: head launch with the dz1 all-gather, then the global-dW1 launch.
  void mlp_head(uintptr_t p, uintptr_t labels, uintptr_t ws, uintptr_t dz1A, int B,
                uintptr_t stream, double timeout_s, int nslab) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (mode_ != XG_LL_PUSH) throw std::runtime_error("xgmi: the factor exchange needs protocol push");
    mlp_head_xg_launch((const float*)p, (const int*)labels, (float*)ws, (float*)dz1A, B,
                       (hipStream_t)stream, mlp_xg(timeout_s), world_, nslab);
  }

  void mlp_fwdapply_factor(uintptr_t p_old, uintptr_t p_new, float lr, uintptr_t x_prev,
                           uintptr_t x, long long xstride, uintptr_t dz1A, uintptr_t ws,
                           uintptr_t ctr, uintptr_t stats, int ring, int B, int stats_on,
                           uintptr_t stream, double timeout_s) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (mode_ != XG_LL_PUSH) throw std::runtime_error("xgmi: the factor exchange needs protocol push");
    mlp_fwdapply_factor_launch((const float*)p_old, (float*)p_new, lr, (const float*)x_prev,
                               (const float*)x, xstride, (const float*)dz1A, (float*)ws,
                               (int*)ctr, (float*)stats, ring, B, stats_on, (hipStream_t)stream,
                               mlp_xg(timeout_s), world_);
  }

  // Pipelined fused engine: exchange + apply of step t-1 fused with step t's forward.
  void mlp_fwdapply(uintptr_t p_old, uintptr_t p_new, float lr, uintptr_t x_prev, uintptr_t x,
                    uintptr_t ws, uintptr_t ctr, uintptr_t stats, int ring, int B, int stats_on,
                    uintptr_t stream, double timeout_s, int two_shot, uintptr_t trace) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (mode_ != XG_LL_PUSH) throw std::runtime_error("xgmi: the fused MLP exchange needs protocol push");
    mlp_fwdapply_xg_launch((const float*)p_old, (float*)p_new, lr, (const float*)x_prev,
                           (const float*)x, (float*)ws, (int*)ctr, (float*)stats, ring, B,
                           stats_on, (hipStream_t)stream, mlp_xg(timeout_s), world_, two_shot,
                           (unsigned long long*)trace);
  }

  // Host loop of the pipelined exchange engines (FusedMLPTrainer.run_launched, data-parallel
  // form of mlp_run_pipelined_launch): n two-launch steps of kind 0 fused2 / 1 fused2x /
  // 2 factor2 over the device-resident batches, issued by ONE call -- no graph submission
  // (the ~17 us fixed cost of a replay that a driver-sized K = 20 run feels) and no Python per
  // step.  Same launches, arguments and order as step_xgmi_pipelined / step_factor_pipelined;
  // flush: the last step's pending update too (flush_xgmi / flush_factor).  x: this rank's
  // batches (factor2: its slice of x_all, the peers' at +- xstride).
  void mlp_run_engine(int kind, uintptr_t p0, uintptr_t p1, int cur, int pending, float lr,
                      uintptr_t x, long long xstride, uintptr_t labels, int nbatches, int pos,
                      int n, uintptr_t ws, uintptr_t ctr, uintptr_t stats, int ring, int B,
                      uintptr_t dz1A, uintptr_t stream, double timeout_s, int flush) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (mode_ != XG_LL_PUSH) throw std::runtime_error("xgmi: the MLP engines need protocol push");
    if (kind < 0 || kind > 2 || !p0 || !p1 || p0 == p1 || !x || !labels || !ctr || nbatches < 1 ||
        pos < 0 || pos >= nbatches || n < 0 || (kind == 2 && !dz1A))
      throw std::runtime_error("mlp_run_engine: bad kind / buffers / position / count");
    const MlpXg xg = mlp_xg(timeout_s);
    hipStream_t s = (hipStream_t)stream;
    float* bufs[2] = {(float*)p0, (float*)p1};
    const float* xs = (const float*)x;
    const int* lab = (const int*)labels;
    const size_t xb = (size_t)B * 784;
    for (int i = 0; i < n; ++i) {
      const int prev = (pos + nbatches - 1) % nbatches;
      const float* xcur = xs + (size_t)pos * xb;
      const float* xprev = pending ? xs + (size_t)prev * xb : xcur;
      const float l = pending ? lr : 0.f;
      float* po = bufs[cur];
      float* pn = bufs[cur ^ 1];
      if (kind == 2) {
        mlp_fwdapply_factor_launch(po, pn, l, xprev, xcur, xstride, (const float*)dz1A,
                                   (float*)ws, (int*)ctr, (float*)stats, ring, B, pending, s, xg,
                                   world_);
        mlp_head_xg_launch(pn, lab + (size_t)pos * B, (float*)ws, (float*)dz1A, B, s, xg,
                           world_, 28);
      } else {
        mlp_fwdapply_xg_launch(po, pn, l, xprev, xcur, (float*)ws, (int*)ctr, (float*)stats,
                               ring, B, pending, s, xg, world_, kind);
        mlp_head2_launch(pn, lab + (size_t)pos * B, (float*)ws, B, s, 28);
      }
      cur ^= 1;
      pending = 1;
      pos = (pos + 1) % nbatches;
    }
    if (flush && pending) {
      const float* xp = xs + (size_t)((pos + nbatches - 1) % nbatches) * xb;
      if (kind == 2)  // in place
        mlp_wgrad_factor_launch(bufs[cur], lr, xp, xstride, (const float*)dz1A, (float*)ws,
                                (int*)ctr, (float*)stats, ring, B, s, xg, world_);
      else            // bufs[cur] -> bufs[cur ^ 1]
        mlp_fwdapply_xg_launch(bufs[cur], bufs[cur ^ 1], lr, xp, xp, (float*)ws, (int*)ctr,
                               (float*)stats, ring, B, 1, s, xg, world_, kind);
    }
  }

  void mlp_wgrad_factor(uintptr_t p, float lr, uintptr_t x, long long xstride, uintptr_t dz1A,
                        uintptr_t ws, uintptr_t ctr, uintptr_t stats, int ring, int B,
                        uintptr_t stream, double timeout_s) {
    if (!ready_) throw std::runtime_error("xgmi: open() the peer handles first");
    if (mode_ != XG_LL_PUSH) throw std::runtime_error("xgmi: the factor exchange needs protocol push");
    mlp_wgrad_factor_launch((float*)p, lr, (const float*)x, xstride, (const float*)dz1A,
                            (float*)ws, (int*)ctr, (float*)stats, ring, B, (hipStream_t)stream,
                            mlp_xg(timeout_s), world_);
  }

  // Probe / test hook: every exchange-epoch counter back to 0 on `stream` (the next call of
  // any kernel of this communicator uses epoch 1 again).  Only meaningful with simulated peers
  // (open_local), whose words the caller stages for that epoch.
  void reset_epochs(uintptr_t stream) {
    XG_CHECK(hipMemsetAsync(epochs_, 0, sizeof(unsigned) * XG_BLOCKS, (hipStream_t)stream));
    XG_CHECK(hipMemsetAsync(mlp_epochs_, 0, sizeof(unsigned) * MLP_XG_EPOCHS, (hipStream_t)stream));
  }

  int error() {
    int e = 0;
    XG_CHECK(hipMemcpy(&e, err_, sizeof(int), hipMemcpyDeviceToHost));
    return e | (abort_host_ && __atomic_load_n(abort_host_, __ATOMIC_RELAXED));
  }

  // Peer-watchdog hook: release every bandwidth-mode wait of this communicator (running or
  // queued) within ~1 ms.  A plain store to pinned host memory, safe from any thread.
  void abort() {
    if (abort_host_) __atomic_store_n(abort_host_, 1, __ATOMIC_RELEASE);
  }

  void close() {
    for (void* q : opened_) hipIpcCloseMemHandle(q);
    opened_.clear();
    if (base_) hipFree(base_);
    if (epochs_) hipFree(epochs_);
    if (mlp_epochs_) hipFree(mlp_epochs_);
    if (abort_host_) hipHostFree(abort_host_);
    abort_host_ = abort_dev_ = nullptr;
    base_ = nullptr;
    epochs_ = nullptr;
    mlp_epochs_ = nullptr;
    ready_ = false;
  }

 private:
  int rank_, world_, device_;
  long long S_;
  int mode_ = -1;  // -1: flag protocol, else XG_LL_* / XG_BW
  int bw_blocks_ = XG_BLOCKS;
  long long data_bytes_ = 0;
  size_t bytes_ = 0;
  void* base_ = nullptr;
  unsigned* epochs_ = nullptr;
  unsigned* mlp_epochs_ = nullptr;
  int* err_ = nullptr;
  int* abort_host_ = nullptr;  // pinned host abort word and its device mapping
  int* abort_dev_ = nullptr;
  XgPeers peers_;
  std::vector<void*> opened_;
  bool ready_ = false;
};

}  // namespace dtfx

void register_xgmi(py::module_& m) {
  py::class_<dtfx::XgmiAllReduce>(m, "XgmiAllReduce")
      .def(py::init<int, int, int, long long, const std::string&>(), py::arg("rank"),
           py::arg("world"), py::arg("device"), py::arg("max_numel"),
           py::arg("protocol") = "ll")
      .def(py::init<int, int, int, long long, const std::string&, bool>(), py::arg("rank"),
           py::arg("world"), py::arg("device"), py::arg("max_numel"), py::arg("protocol"),
           py::arg("own_slots"))
      .def("region_bytes", &dtfx::XgmiAllReduce::region_bytes)
      .def("set_bw_blocks", &dtfx::XgmiAllReduce::set_bw_blocks)
      .def("slot_stride", &dtfx::XgmiAllReduce::slot_stride)
      .def("open_local", &dtfx::XgmiAllReduce::open_local)
      .def("handle", &dtfx::XgmiAllReduce::handle)
      .def("open", &dtfx::XgmiAllReduce::open)
      .def("all_reduce", &dtfx::XgmiAllReduce::all_reduce, py::arg("g"), py::arg("n"),
           py::arg("stream"), py::arg("timeout_s") = 2.0)
      .def("mlp_wgrad", &dtfx::XgmiAllReduce::mlp_wgrad, py::arg("p"), py::arg("lr"), py::arg("x"),
           py::arg("ws"), py::arg("ctr"), py::arg("stats"), py::arg("ring"), py::arg("B"),
           py::arg("stream"), py::arg("timeout_s") = 2.0)
      .def("mlp_head", &dtfx::XgmiAllReduce::mlp_head, py::arg("p"), py::arg("labels"),
           py::arg("ws"), py::arg("dz1A"), py::arg("B"), py::arg("stream"),
           py::arg("timeout_s") = 2.0, py::arg("nslab") = 7)
      .def("mlp_fwdapply_factor", &dtfx::XgmiAllReduce::mlp_fwdapply_factor, py::arg("p_old"),
           py::arg("p_new"), py::arg("lr"), py::arg("x_prev"), py::arg("x"), py::arg("xstride"),
           py::arg("dz1A"), py::arg("ws"), py::arg("ctr"), py::arg("stats"), py::arg("ring"),
           py::arg("B"), py::arg("stats_on"), py::arg("stream"), py::arg("timeout_s") = 2.0)
      .def("mlp_fwdapply", &dtfx::XgmiAllReduce::mlp_fwdapply, py::arg("p_old"),
           py::arg("p_new"), py::arg("lr"), py::arg("x_prev"), py::arg("x"), py::arg("ws"),
           py::arg("ctr"), py::arg("stats"), py::arg("ring"), py::arg("B"), py::arg("stats_on"),
           py::arg("stream"), py::arg("timeout_s") = 2.0, py::arg("two_shot") = 0,
           py::arg("trace") = 0)
      .def("mlp_wgrad_factor", &dtfx::XgmiAllReduce::mlp_wgrad_factor, py::arg("p"),
           py::arg("lr"), py::arg("x"), py::arg("xstride"), py::arg("dz1A"), py::arg("ws"),
           py::arg("ctr"), py::arg("stats"), py::arg("ring"), py::arg("B"), py::arg("stream"),
           py::arg("timeout_s") = 2.0)
      .def("mlp_run_engine", &dtfx::XgmiAllReduce::mlp_run_engine, py::arg("kind"),
           py::arg("p0"), py::arg("p1"), py::arg("cur"), py::arg("pending"), py::arg("lr"),
           py::arg("x"), py::arg("xstride"), py::arg("labels"), py::arg("nbatches"),
           py::arg("pos"), py::arg("n"), py::arg("ws"), py::arg("ctr"), py::arg("stats"),
           py::arg("ring"), py::arg("B"), py::arg("dz1A"), py::arg("stream"),
           py::arg("timeout_s"), py::arg("flush"))
      .def("shard_op", &dtfx::XgmiAllReduce::shard_op, py::arg("op"), py::arg("g"), py::arg("n"),
           py::arg("stream"), py::arg("timeout_s") = 2.0)
      .def("error", &dtfx::XgmiAllReduce::error)
      .def("abort", &dtfx::XgmiAllReduce::abort, py::call_guard<py::gil_scoped_release>())
      .def("reset_epochs", &dtfx::XgmiAllReduce::reset_epochs)
      .def("close", &dtfx::XgmiAllReduce::close);
}
