// Native RCCL communicator (the sync-DP transport of the framework).
//
// Replaces the reference's gRPC parameter-server fabric (main.py:67-75,
// worker.py:123) for synchronous data parallelism: one process per GPU, one
// RCCL communicator, collectives enqueued on the caller's HIP stream (so a
// hipGraph capture of a training step records them as graph nodes and no
// Python runs per step).  RCCL rides xGMI between the MI355X of a node.
//
// The unique id is exchanged by the Python layer through the
// torch.distributed TCP store (parallel/comm.py), so the control plane can be
// gloo/TCP while all tensor traffic is RCCL.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstring>
#include <memory>
#include <thread>
#include <stdexcept>
#include <string>

namespace py = pybind11;

namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

ncclDataType_t dtype_of(const std::string& d) {
  if (d == "float32") return ncclFloat32;
  if (d == "float16") return ncclFloat16;
  if (d == "bfloat16") return ncclBfloat16;
  if (d == "float64") return ncclFloat64;
  if (d == "int32") return ncclInt32;
  if (d == "int64") return ncclInt64;
  if (d == "uint8") return ncclUint8;
  throw std::runtime_error("rccl: unsupported dtype " + d);
}

ncclRedOp_t op_of(const std::string& o) {
  if (o == "sum") return ncclSum;
  if (o == "max") return ncclMax;
  if (o == "min") return ncclMin;
  if (o == "prod") return ncclProd;
  if (o == "avg") return ncclAvg;
  throw std::runtime_error("rccl: unsupported op " + o);
}

class RcclComm {
 public:
  RcclComm(py::bytes uid, int nranks, int rank, int device) : nranks_(nranks), rank_(rank) {
    std::string s = uid;
    if (s.size() != sizeof(ncclUniqueId)) throw std::runtime_error("rccl: bad unique id size");
    ncclUniqueId id;
    std::memcpy(&id, s.data(), sizeof(id));
    if (hipSetDevice(device) != hipSuccess) throw std::runtime_error("rccl: hipSetDevice failed");
    ncclComm_t c = nullptr;
    check(ncclCommInitRank(&c, nranks, id, rank), "ncclCommInitRank");
    comm_.store(c, std::memory_order_release);
  }
  ~RcclComm() { destroy(); }

  void destroy() {
    ncclComm_t c = comm_.exchange(nullptr);
    if (c) ncclCommDestroy(c);
  }
  // Fail-fast teardown (parallel/watchdog.py): called from a watchdog thread while the
  // training thread may be blocked on a stream whose RCCL kernels wait for a dead peer.
  // ncclCommAbort makes those kernels return and frees the communicator; every later
  // collective on this object raises.  The pointer is swapped out atomically (no new call
  // can pick it up) and the abort waits, bounded, for calls already inside RCCL on another
  // thread (`Use` guards) to leave, so it does not free a communicator under an enqueue.
  void abort() {
    ncclComm_t c = comm_.exchange(nullptr);
    if (!c) return;
    const auto until = std::chrono::steady_clock::now() + std::chrono::seconds(2);
    while (inflight_.load(std::memory_order_acquire) > 0 && std::chrono::steady_clock::now() < until)
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    ncclCommAbort(c);
  }
  // ncclSuccess (0) while healthy; an RCCL error code once a remote failure / abort was seen.
  int async_error() {
    Use u(this);
    if (!u.c) return static_cast<int>(ncclInvalidUsage);
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(u.c, &r) != ncclSuccess) return static_cast<int>(ncclInternalError);
    return static_cast<int>(r);
  }
  // A call's hold on the communicator: counted in inflight_ for abort() to wait on.
  struct Use {
    RcclComm* o;
    ncclComm_t c;
    explicit Use(RcclComm* o_) : o(o_) {
      o->inflight_.fetch_add(1, std::memory_order_acq_rel);
      c = o->comm_.load(std::memory_order_acquire);
    }
    ~Use() { o->inflight_.fetch_sub(1, std::memory_order_acq_rel); }
    ncclComm_t get() const {
      if (!c) throw std::runtime_error("rccl: communicator destroyed");
      return c;
    }
  };

  void all_reduce(uintptr_t send, uintptr_t recv, size_t count, const std::string& dt,
                  const std::string& op, uintptr_t stream) {
    Use u(this);
    check(ncclAllReduce(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                        dtype_of(dt), op_of(op), u.get(), reinterpret_cast<hipStream_t>(stream)),
          "ncclAllReduce");
  }
  void reduce_scatter(uintptr_t send, uintptr_t recv, size_t recv_count, const std::string& dt,
                      const std::string& op, uintptr_t stream) {
    Use u(this);
    check(ncclReduceScatter(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                            recv_count, dtype_of(dt), op_of(op), u.get(),
                            reinterpret_cast<hipStream_t>(stream)),
          "ncclReduceScatter");
  }
  void all_gather(uintptr_t send, uintptr_t recv, size_t send_count, const std::string& dt,
                  uintptr_t stream) {
    Use u(this);
    check(ncclAllGather(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv),
                        send_count, dtype_of(dt), u.get(), reinterpret_cast<hipStream_t>(stream)),
          "ncclAllGather");
  }
  void broadcast(uintptr_t send, uintptr_t recv, size_t count, const std::string& dt, int root,
                 uintptr_t stream) {
    Use u(this);
    check(ncclBroadcast(reinterpret_cast<const void*>(send), reinterpret_cast<void*>(recv), count,
                        dtype_of(dt), root, u.get(), reinterpret_cast<hipStream_t>(stream)),
          "ncclBroadcast");
  }
  void all_to_all(uintptr_t send, uintptr_t recv, size_t count_per_rank, const std::string& dt,
                  size_t elem_size, uintptr_t stream) {
    // grouped send/recv: rank r's slice i goes to rank i
    const ncclDataType_t t = dtype_of(dt);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    Use u(this);
    ncclComm_t c = u.get();
    check(ncclGroupStart(), "ncclGroupStart");
    // the group is ALWAYS closed: an error inside it is recorded and raised after
    // ncclGroupEnd, so the next collective is never merged into an unfinished group
    ncclResult_t first = ncclSuccess;
    const char* what = "";
    for (int peer = 0; peer < nranks_ && first == ncclSuccess; ++peer) {
      const char* sp = reinterpret_cast<const char*>(send) + peer * count_per_rank * elem_size;
      char* rp = reinterpret_cast<char*>(recv) + peer * count_per_rank * elem_size;
      ncclResult_t r = ncclSend(sp, count_per_rank, t, peer, c, s);
      if (r != ncclSuccess) {
        first = r;
        what = "ncclSend";
        break;
      }
      r = ncclRecv(rp, count_per_rank, t, peer, c, s);
      if (r != ncclSuccess) {
        first = r;
        what = "ncclRecv";
      }
    }
    const ncclResult_t end = ncclGroupEnd();
    check(first, what);
    check(end, "ncclGroupEnd");
  }
  int nranks() const { return nranks_; }
  int rank() const { return rank_; }

 private:
  std::atomic<ncclComm_t> comm_{nullptr};
  std::atomic<int> inflight_{0};
  int nranks_, rank_;
};

}  // namespace

void register_rccl(py::module_& m) {
  m.def("rccl_unique_id", []() {
    ncclUniqueId id;
    check(ncclGetUniqueId(&id), "ncclGetUniqueId");
    return py::bytes(reinterpret_cast<const char*>(&id), sizeof(id));
  });
  m.def("rccl_version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<py::bytes, int, int, int>(), py::arg("unique_id"), py::arg("nranks"),
           py::arg("rank"), py::arg("device"))
      // the collectives touch no Python object: they run without the GIL, so a collective
      // blocked inside RCCL (e.g. connecting to a dead peer) cannot keep the peer watchdog's
      // thread from entering abort() -- whose Use/inflight guard then really waits for it
      .def("all_reduce", &RcclComm::all_reduce, py::arg("send"), py::arg("recv"), py::arg("count"),
           py::arg("dtype") = "float32", py::arg("op") = "sum", py::arg("stream") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &RcclComm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("all_gather", &RcclComm::all_gather, py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &RcclComm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("all_to_all", &RcclComm::all_to_all, py::call_guard<py::gil_scoped_release>())
      .def("destroy", &RcclComm::destroy)
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def("async_error", &RcclComm::async_error)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("rank", &RcclComm::rank);
}
