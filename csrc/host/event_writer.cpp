// TensorBoard event files: TFRecord framing of tensorflow.Event protos.
//
// The reference writes `loss` and `accuracy` scalars every step through
// tf.summary.FileWriter (worker.py:92-96, 139) -- TF's C++ EventsWriter with
// an async flush thread.  This is the native equivalent:
//
//   record := uint64 length | uint32 masked_crc32c(length) | data
//             | uint32 masked_crc32c(data)
//   Event  := {1: double wall_time, 2: int64 step,
//              3: string file_version | 5: Summary}
//   Summary.Value := {1: string tag, 2: float simple_value}
//
// File name events.out.tfevents.<unix seconds>.<hostname>, first record
// file_version = "brain.Event:2", exactly like TF, so TensorBoard reads it.
// Records are queued and written by a background thread every flush_secs
// (TF default 120 s) or on flush()/close().
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <ctime>
#include <deque>
#include <fstream>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "crc32c.h"
#include "proto.h"

namespace py = pybind11;
using namespace dtfx_host;

namespace {

std::string frame_record(const std::string& data) {
  std::string out;
  const uint64_t len = data.size();
  char lb[8];
  std::memcpy(lb, &len, 8);
  out.append(lb, 8);
  pb::put_fixed32(out, crc32c_mask(crc32c(lb, 8)));
  out.append(data);
  pb::put_fixed32(out, crc32c_mask(crc32c(data.data(), data.size())));
  return out;
}

double now_wall() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch())
      .count();
}

void put_double_field(std::string& o, uint32_t f, double v) {
  uint64_t b;
  std::memcpy(&b, &v, 8);
  pb::put_fixed64_field(o, f, b);
}

std::string summary_scalars(const std::vector<std::pair<std::string, float>>& vals) {
  std::string summ;
  for (auto& kv : vals) {
    std::string v;
    pb::put_bytes_field(v, 1, kv.first);
    uint32_t fb;
    std::memcpy(&fb, &kv.second, 4);
    pb::put_fixed32_field(v, 2, fb);
    pb::put_bytes_field(summ, 1, v);
  }
  return summ;
}

std::string event_proto(double wall, int64_t step, const std::string* file_version,
                        const std::string* summary) {
  std::string e;
  put_double_field(e, 1, wall);
  if (step != 0) pb::put_varint_field(e, 2, static_cast<uint64_t>(step));
  if (file_version) pb::put_bytes_field(e, 3, *file_version);
  if (summary) pb::put_bytes_field(e, 5, *summary);
  return e;
}

class EventWriter {
 public:
  EventWriter(const std::string& logdir, double flush_secs, const std::string& suffix)
      : flush_secs_(flush_secs) {
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    path_ = logdir + "/events.out.tfevents." + std::to_string((long long)std::time(nullptr)) + "." +
            host + suffix;
    f_.open(path_, std::ios::binary | std::ios::app);
    if (!f_) throw std::runtime_error("EventWriter: cannot open " + path_);
    const std::string ver = "brain.Event:2";
    f_ << frame_record(event_proto(now_wall(), 0, &ver, nullptr));
    f_.flush();
    thr_ = std::thread([this] { loop(); });
  }
  ~EventWriter() { close(); }

  void add_event(py::bytes event) { enqueue(std::string(event)); }

  void add_scalars(py::dict d, int64_t step, double wall) {
    std::vector<std::pair<std::string, float>> vals;
    for (auto kv : d) vals.emplace_back(kv.first.cast<std::string>(), kv.second.cast<float>());
    const std::string s = summary_scalars(vals);
    enqueue(event_proto(wall > 0 ? wall : now_wall(), step, nullptr, &s));
  }

  void add_summary(py::bytes summary, int64_t step, double wall) {
    const std::string s = summary;
    enqueue(event_proto(wall > 0 ? wall : now_wall(), step, nullptr, &s));
  }

  // bulk path: [n] steps x [k] tags (from the device stats ring), one lock
  void add_scalar_series(std::vector<std::string> tags, std::vector<int64_t> steps,
                         std::vector<std::vector<float>> values, double wall) {
    if (values.size() != steps.size()) throw std::runtime_error("add_scalar_series: size mismatch");
    const double w = wall > 0 ? wall : now_wall();
    std::vector<std::string> recs;
    recs.reserve(steps.size());
    for (size_t i = 0; i < steps.size(); ++i) {
      if (values[i].size() != tags.size()) throw std::runtime_error("add_scalar_series: width");
      std::vector<std::pair<std::string, float>> vals;
      for (size_t k = 0; k < tags.size(); ++k) vals.emplace_back(tags[k], values[i][k]);
      const std::string s = summary_scalars(vals);
      recs.push_back(frame_record(event_proto(w, steps[i], nullptr, &s)));
    }
    std::lock_guard<std::mutex> g(mu_);
    for (auto& r : recs) q_.push_back(std::move(r));
  }

  void flush() {
    std::deque<std::string> q;
    {
      std::lock_guard<std::mutex> g(mu_);
      q.swap(q_);
    }
    std::lock_guard<std::mutex> g(io_);
    for (auto& r : q) f_ << r;
    f_.flush();
  }

  void close() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (closed_) return;
      closed_ = true;
    }
    cv_.notify_all();
    if (thr_.joinable()) thr_.join();
    flush();
    f_.close();
  }

  std::string path() const { return path_; }

 private:
  void enqueue(const std::string& event) {
    std::lock_guard<std::mutex> g(mu_);
    if (closed_) throw std::runtime_error("EventWriter: closed");
    q_.push_back(frame_record(event));
  }
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    const auto period = std::chrono::duration_cast<std::chrono::system_clock::duration>(
        std::chrono::duration<double>(flush_secs_));
    while (!closed_) {
      // system_clock deadline: pthread_cond_timedwait, which ThreadSanitizer intercepts
      // (wait_for's steady clock maps to pthread_cond_clockwait, which GCC 11's TSan does
      // not, and then reports a false double lock -- tools/sanitize_host.py)
      cv_.wait_until(lk, std::chrono::system_clock::now() + period);
      if (closed_) break;
      lk.unlock();
      flush();
      lk.lock();
    }
  }

  std::string path_;
  std::ofstream f_;
  double flush_secs_;
  std::deque<std::string> q_;
  std::mutex mu_, io_;
  std::condition_variable cv_;
  std::thread thr_;
  bool closed_ = false;
};

py::list read_records(const std::string& path, bool verify) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw std::runtime_error("cannot open " + path);
  std::string all((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  py::list out;
  size_t p = 0;
  while (p + 12 <= all.size()) {
    uint64_t len;
    std::memcpy(&len, all.data() + p, 8);
    uint32_t lcrc;
    std::memcpy(&lcrc, all.data() + p + 8, 4);
    if (verify && crc32c_unmask(lcrc) != crc32c(all.data() + p, 8))
      throw std::runtime_error("tfrecord: length checksum mismatch");
    if (p + 12 + len + 4 > all.size()) break;  // truncated tail (writer still running)
    std::string data = all.substr(p + 12, len);
    uint32_t dcrc;
    std::memcpy(&dcrc, all.data() + p + 12 + len, 4);
    if (verify && crc32c_unmask(dcrc) != crc32c(data.data(), data.size()))
      throw std::runtime_error("tfrecord: data checksum mismatch");
    out.append(py::bytes(data));
    p += 12 + len + 4;
  }
  return out;
}

// parse_event(bytes) -> {"wall_time", "step", "file_version"?, "scalars": {tag: value}}
py::dict parse_event(py::bytes b) {
  const std::string s = b;
  pb::Reader r(s);
  py::dict out;
  py::dict scal;
  out["step"] = 0;
  while (!r.done()) {
    const uint64_t tag = r.varint();
    const uint32_t f = tag >> 3, w = tag & 7;
    if (f == 1 && w == 1) {
      const uint64_t bits = r.fixed64();
      double d;
      std::memcpy(&d, &bits, 8);
      out["wall_time"] = d;
    } else if (f == 2 && w == 0) out["step"] = static_cast<int64_t>(r.varint());
    else if (f == 3 && w == 2) out["file_version"] = r.bytes();
    else if (f == 4 && w == 2) out["graph_def"] = py::bytes(r.bytes());
    else if (f == 5 && w == 2) {
      const std::string sbuf = r.bytes();
      pb::Reader sr(sbuf);
      while (!sr.done()) {
        const uint64_t st = sr.varint();
        if ((st >> 3) == 1 && (st & 7) == 2) {
          const std::string vbuf = sr.bytes();
          pb::Reader vr(vbuf);
          std::string vtag;
          float val = 0.f;
          while (!vr.done()) {
            const uint64_t vt = vr.varint();
            if ((vt >> 3) == 1 && (vt & 7) == 2) vtag = vr.bytes();
            else if ((vt >> 3) == 2 && (vt & 7) == 5) {
              const uint32_t bits = vr.fixed32();
              std::memcpy(&val, &bits, 4);
            } else vr.skip(vt & 7);
          }
          scal[py::str(vtag)] = val;
        } else sr.skip(st & 7);
      }
    } else r.skip(w);
  }
  out["scalars"] = scal;
  return out;
}

}  // namespace

void register_events(py::module_& m) {
  py::class_<EventWriter>(m, "EventWriter")
      .def(py::init<const std::string&, double, const std::string&>(), py::arg("logdir"),
           py::arg("flush_secs") = 120.0, py::arg("filename_suffix") = "")
      .def("add_event", &EventWriter::add_event)
      .def("add_scalars", &EventWriter::add_scalars, py::arg("values"), py::arg("step"),
           py::arg("wall_time") = 0.0)
      .def("add_summary", &EventWriter::add_summary, py::arg("summary"), py::arg("step"),
           py::arg("wall_time") = 0.0)
      .def("add_scalar_series", &EventWriter::add_scalar_series, py::arg("tags"), py::arg("steps"),
           py::arg("values"), py::arg("wall_time") = 0.0)
      .def("flush", &EventWriter::flush, py::call_guard<py::gil_scoped_release>())
      .def("close", &EventWriter::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("path", &EventWriter::path);
  m.def("summary_scalars", [](py::dict d) {
    std::vector<std::pair<std::string, float>> vals;
    for (auto kv : d) vals.emplace_back(kv.first.cast<std::string>(), kv.second.cast<float>());
    return py::bytes(summary_scalars(vals));
  }, "Serialize a tensorflow.Summary of simple_value scalars.");
  m.def("read_records", &read_records, py::arg("path"), py::arg("verify") = true);
  m.def("parse_event", &parse_event);
  m.def("frame_record", [](py::bytes b) { return py::bytes(frame_record(std::string(b))); });
}
