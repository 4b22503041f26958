// Host side of the GPU-resident parameter store (kernels and rationale: gpu_ps.hip): one
// uncached allocation [params f32 | control words u64] on the owner's GPU, exported as an IPC
// handle; other processes open it (over xGMI when they run on another GPU).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>

namespace py = pybind11;

#define GPS_CHECK(expr)                                                                \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) +     \
                               " in " #expr);                                          \
  } while (0)

namespace dtfx {

void gps_pull_launch(float*, const float*, long long, hipStream_t);
void gps_apply_launch(float*, const float*, float, long long, bool, hipStream_t);
void gps_fetch_add_launch(unsigned long long*, long long, unsigned long long*, const float*, int,
                          hipStream_t);

class GpuParamStore {
 public:
  static constexpr int kCtrlWords = 32;  // [0] global_step, [1] initialised flag

  // owner: allocate + zero; otherwise open(handle) before use
  GpuParamStore(int device, long long n, bool owner) : device_(device), n_(n), owner_(owner) {
    if (n < 1) throw std::runtime_error("gpu_ps: n must be >= 1");
    GPS_CHECK(hipSetDevice(device));
    pbytes_ = (n * 4 + 255) / 256 * 256;
    bytes_ = pbytes_ + kCtrlWords * 8;
    bytes_ = (bytes_ + (2u << 20) - 1) / (2u << 20) * (2u << 20);
    if (owner) {
      GPS_CHECK(hipExtMallocWithFlags(&base_, bytes_, hipDeviceMallocUncached));
      GPS_CHECK(hipMemset(base_, 0, bytes_));
    }
    GPS_CHECK(hipHostMalloc(&host_word_, 64, hipHostMallocDefault));
    GPS_CHECK(hipMalloc(&dev_word_, 64));
  }
  ~GpuParamStore() { close(); }

  py::bytes handle() {
    if (!owner_ || !base_) throw std::runtime_error("gpu_ps: only the owner exports a handle");
    hipIpcMemHandle_t h;
    GPS_CHECK(hipIpcGetMemHandle(&h, base_));
    return py::bytes(reinterpret_cast<const char*>(&h), sizeof(h));
  }

  static int handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

  void open(const std::string& handle) {
    if (owner_) return;
    hipIpcMemHandle_t h;
    if (handle.size() != sizeof(h)) throw std::runtime_error("gpu_ps: bad handle size");
    std::memcpy(&h, handle.data(), sizeof(h));
    GPS_CHECK(hipSetDevice(device_));
    GPS_CHECK(hipIpcOpenMemHandle(&base_, h, hipIpcMemLazyEnablePeerAccess));
  }

  uintptr_t params() const { return reinterpret_cast<uintptr_t>(base()); }
  long long numel() const { return n_; }

  void pull(uintptr_t dst, uintptr_t stream) {
    gps_pull_launch(reinterpret_cast<float*>(dst), reinterpret_cast<const float*>(base()), n_,
                    reinterpret_cast<hipStream_t>(stream));
  }

  void push_apply(uintptr_t g, float lr, bool locking, uintptr_t stream) {
    gps_apply_launch(reinterpret_cast<float*>(base()), reinterpret_cast<const float*>(g), lr, n_,
                     locking, reinterpret_cast<hipStream_t>(stream));
  }

  // control word `slot` += delta on the device (system-scope atomic); returns the old value
  long long fetch_add(int slot, long long delta, uintptr_t stream) {
    return fetch_add_impl(slot, delta, stream, 0, 0, nullptr);
  }

  // the same, also reading back `nextra` (<= 14) f32 words at device address `extra` in the
  // same copy: (old value, [floats])
  py::tuple fetch_add_read(int slot, long long delta, uintptr_t stream, uintptr_t extra,
                           int nextra) {
    float vals[14];
    const long long old = fetch_add_impl(slot, delta, stream, extra, nextra, vals);
    py::list l;
    for (int i = 0; i < nextra; ++i) l.append(vals[i]);
    return py::make_tuple(old, l);
  }

  // synchronous host <-> store copies (init / restore / checkpoint); offsets in bytes
  void read(uintptr_t host, long long off, long long nbytes) {
    check_range(off, nbytes);
    py::gil_scoped_release nogil;
    GPS_CHECK(hipSetDevice(device_));
    GPS_CHECK(hipMemcpy(reinterpret_cast<void*>(host), static_cast<char*>(base()) + off, nbytes,
                        hipMemcpyDeviceToHost));
  }
  void write(uintptr_t host, long long off, long long nbytes) {
    check_range(off, nbytes);
    py::gil_scoped_release nogil;
    GPS_CHECK(hipSetDevice(device_));
    GPS_CHECK(hipMemcpy(static_cast<char*>(base()) + off, reinterpret_cast<const void*>(host),
                        nbytes, hipMemcpyHostToDevice));
  }
  long long ctrl_offset() const { return pbytes_; }

  void close() {
    if (base_) {
      hipSetDevice(device_);
      hipDeviceSynchronize();
      if (owner_) hipFree(base_);
      else hipIpcCloseMemHandle(base_);
      base_ = nullptr;
    }
    if (host_word_) {
      hipHostFree(host_word_);
      host_word_ = nullptr;
    }
    if (dev_word_) {
      hipFree(dev_word_);
      dev_word_ = nullptr;
    }
  }

 private:
  long long fetch_add_impl(int slot, long long delta, uintptr_t stream, uintptr_t extra,
                           int nextra, float* vals) {
    if (slot < 0 || slot >= kCtrlWords) throw std::runtime_error("gpu_ps: bad control slot");
    if (nextra < 0 || nextra > 14) throw std::runtime_error("gpu_ps: at most 14 extra words");
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> lock(mu_);  // one staging buffer: the saver thread calls too
    const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    gps_fetch_add_launch(ctrl() + slot, delta, dev_word_, reinterpret_cast<const float*>(extra),
                         nextra, s);
    GPS_CHECK(hipMemcpyAsync(host_word_, dev_word_, 8 + 4 * nextra, hipMemcpyDeviceToHost, s));
    GPS_CHECK(hipStreamSynchronize(s));
    if (vals) std::memcpy(vals, host_word_ + 1, 4 * nextra);
    return (long long)*host_word_;
  }

  void* base() const {
    if (!base_) throw std::runtime_error("gpu_ps: store not allocated / opened");
    return base_;
  }
  unsigned long long* ctrl() const {
    return reinterpret_cast<unsigned long long*>(static_cast<char*>(base()) + pbytes_);
  }
  void check_range(long long off, long long nbytes) const {
    if (off < 0 || nbytes < 0 || off + nbytes > pbytes_ + kCtrlWords * 8)
      throw std::runtime_error("gpu_ps: copy out of range");
  }

  int device_;
  long long n_;
  bool owner_;
  long long pbytes_ = 0, bytes_ = 0;
  void* base_ = nullptr;
  unsigned long long* host_word_ = nullptr;
  unsigned long long* dev_word_ = nullptr;
  std::mutex mu_;
};

}  // namespace dtfx

void register_gpu_ps(py::module_& m) {
  py::class_<dtfx::GpuParamStore>(m, "GpuParamStore")
      .def(py::init<int, long long, bool>(), py::arg("device"), py::arg("n"), py::arg("owner"))
      .def("handle", &dtfx::GpuParamStore::handle)
      .def_static("handle_size", &dtfx::GpuParamStore::handle_size)
      .def("open", &dtfx::GpuParamStore::open)
      .def("params", &dtfx::GpuParamStore::params)
      .def("numel", &dtfx::GpuParamStore::numel)
      .def("pull", &dtfx::GpuParamStore::pull, py::arg("dst"), py::arg("stream"))
      .def("push_apply", &dtfx::GpuParamStore::push_apply, py::arg("g"), py::arg("lr"),
           py::arg("locking"), py::arg("stream"))
      .def("fetch_add", &dtfx::GpuParamStore::fetch_add, py::arg("slot"), py::arg("delta"),
           py::arg("stream"))
      .def("fetch_add_read", &dtfx::GpuParamStore::fetch_add_read, py::arg("slot"),
           py::arg("delta"), py::arg("stream"), py::arg("extra"), py::arg("nextra"))
      .def("read", &dtfx::GpuParamStore::read)
      .def("write", &dtfx::GpuParamStore::write)
      .def("ctrl_offset", &dtfx::GpuParamStore::ctrl_offset)
      .def("close", &dtfx::GpuParamStore::close);
}
