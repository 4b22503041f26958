// TCP parameter server + client: the async between-graph-replication fabric of
// the reference (TF gRPC MasterService/WorkerService hosting /job:ps
// variables, main.py:66-75, worker.py:24-32, 75-85, 112-113, 131-141).
//
// Server (one per ps task): named variables (f32 or int64), created by the
// chief, assigned (init/restore), then served to workers:
//   PULL        -> bytes of a variable group            (sync_op, worker.py:84-85)
//   PUSH_APPLY  -> var -= lr * grad, lock-free Hogwild  (ApplyGradientDescent,
//                  use_locking=False, worker.py:79) or per-variable mutex
//   FETCH_ADD   -> atomic int64 add, returns old value  (AssignAdd global_step,
//                  worker.py:32, 141)
//   UNINIT      -> which of these are uninitialized     (report_uninitialized_
//                  variables, the Supervisor ready_op, worker.py:112-113)
//   SYNC_PUSH   -> synchronous replicas (TF's SyncReplicasOptimizer, the sync
//                  alternative of the reference's async apply): gradients tagged
//                  with the worker's local step are accumulated; stale ones
//                  (local step behind the round) are dropped, as TF's
//                  ConditionalAccumulator does; the R-th gradient of a round
//                  applies the MEAN, advances the round (and global_step, on
//                  the task that holds it) and releases every waiting pusher --
//                  the token queue of SyncReplicasOptimizer.
// Variables are placed round-robin over ps tasks by the client, like
// tf.train.replica_device_setter(ps_tasks) (worker.py:24).
//
// Wire format (little-endian): request = u32 len | u8 op | payload;
// response = u32 len | u8 status (0 ok) | payload (error text if status != 0).
// One thread per connection; the client pipelines requests to several ps
// tasks (send all, then receive all).
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/socket.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

// Timed condition-variable wait.  Normal builds use the steady clock (immune to wall-clock
// steps: NTP, a manual change).  ThreadSanitizer builds use the system clock: libstdc++'s
// steady-clock wait goes through pthread_cond_clockwait, which TSan (GCC 11) does not
// intercept -- it then misses the unlock inside the wait and reports the next lock as a
// double lock (tools/sanitize_host.py).
template <class Pred>
static bool cv_wait_ms(std::condition_variable& cv, std::unique_lock<std::mutex>& lk, long long ms,
                       Pred pred) {
#if defined(__SANITIZE_THREAD__)
  return cv.wait_until(lk, std::chrono::system_clock::now() + std::chrono::milliseconds(ms), pred);
#else
  return cv.wait_for(lk, std::chrono::milliseconds(ms), pred);
#endif
}

namespace py = pybind11;

namespace {

enum Op : uint8_t {
  OP_CREATE = 1, OP_LOOKUP = 2, OP_ASSIGN = 3, OP_PULL = 4, OP_PUSH_APPLY = 5,
  OP_FETCH_ADD = 6, OP_UNINIT = 7, OP_LIST = 8, OP_SHUTDOWN = 9, OP_PING = 10,
  OP_STATS = 11, OP_SYNC_PUSH = 12
};
constexpr uint32_t kNoVar = 0xffffffffu;
enum DType : uint8_t { DT_F32 = 0, DT_I64 = 1 };

// ---------------------------------------------------------------- io helpers
// A lost ps connection (peer closed, reset, or -- with an rpc timeout -- silent for too long):
// raised to Python as ConnectionError, so a worker whose ps died exits instead of retrying.
struct PSConnectionLost : std::runtime_error {
  using std::runtime_error::runtime_error;
};

bool read_full(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    const ssize_t r = ::recv(fd, p, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}
bool write_full(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    const ssize_t r = ::send(fd, p, n, MSG_NOSIGNAL);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= static_cast<size_t>(r);
  }
  return true;
}
// Gather-write of several buffers (sendmsg over iovecs, partial writes resumed): the push's
// gradient bytes go from the caller's (pinned) memory straight into the socket, without first
// being copied into a request string.
bool writev_full(int fd, std::vector<iovec>& iov) {
  size_t i = 0;
  while (i < iov.size()) {
    msghdr m{};
    m.msg_iov = iov.data() + i;
    m.msg_iovlen = std::min<size_t>(iov.size() - i, 1024);
    const ssize_t r = ::sendmsg(fd, &m, MSG_NOSIGNAL);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    size_t n = static_cast<size_t>(r);
    while (i < iov.size() && n >= iov[i].iov_len) n -= iov[i++].iov_len;
    if (n) {
      iov[i].iov_base = static_cast<char*>(iov[i].iov_base) + n;
      iov[i].iov_len -= n;
    }
  }
  return true;
}
void tune(int fd) {
  int one = 1, buf = 8 << 20;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

struct Writer {
  std::string b;
  template <typename T> void put(T v) { b.append(reinterpret_cast<const char*>(&v), sizeof(T)); }
  void str(const std::string& s) { put<uint16_t>(static_cast<uint16_t>(s.size())); b.append(s); }
  void raw(const void* p, size_t n) { b.append(static_cast<const char*>(p), n); }
};
struct Reader {
  const char* p;
  const char* e;
  template <typename T> T get() {
    if (e - p < static_cast<ptrdiff_t>(sizeof(T))) throw std::runtime_error("ps: short message");
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    const uint16_t n = get<uint16_t>();
    if (e - p < n) throw std::runtime_error("ps: short string");
    std::string s(p, n);
    p += n;
    return s;
  }
  const char* take(size_t n) {
    if (static_cast<size_t>(e - p) < n) throw std::runtime_error("ps: short payload");
    const char* q = p;
    p += n;
    return q;
  }
};

// ---------------------------------------------------------------- server
// The two INTENTIONAL data races of the reference's semantics live in these functions (and
// only here), so ThreadSanitizer runs (tools/sanitize_host.py) suppress exactly them:
//  * lock-free read of a variable while workers apply (TF's pull reads without locking);
//  * Hogwild apply, ApplyGradientDescent(use_locking=False) (worker.py:79).
__attribute__((noinline)) void dtfx_racy_read(Writer& w, const float* p, size_t nbytes) {
  w.raw(p, nbytes);
  // not a tail call: the string append must run under THIS frame, or the sanitizer's stack
  // (and its suppression by function name) loses it -- seen once as a reported race in
  // std::string::_M_mutate called from handle()
  asm volatile("" ::: "memory");
}
// g: the gradient bytes inside the request buffer (no alignment guarantee: loaded by memcpy)
// first: where this apply starts (it wraps around).  Every connection thread starts at its own
// offset (PSServer::serve), so concurrent Hogwild applies of several workers walk different
// cache lines at any moment instead of chasing each other through the same ones (each line
// then bounces between the cores once per apply rather than once per competing thread).
__attribute__((noinline)) void dtfx_hogwild_apply(float* p, const char* g, size_t n, float lr,
                                                  size_t first = 0) {
  first = n ? first % n : 0;
  for (size_t i = first; i < n; ++i) {
    float gi;
    std::memcpy(&gi, g + 4 * i, 4);
    p[i] -= lr * gi;
  }
  for (size_t i = 0; i < first; ++i) {
    float gi;
    std::memcpy(&gi, g + 4 * i, 4);
    p[i] -= lr * gi;
  }
}

struct Var {
  std::string name;
  uint8_t dtype;
  std::vector<int64_t> shape;
  size_t count = 0;
  std::vector<float> f;
  std::atomic<int64_t> i{0};
  std::atomic<bool> init{false};
  std::mutex mu;
  size_t nbytes() const { return dtype == DT_F32 ? count * 4 : 8; }
};

class PSServer {
 public:
  PSServer(const std::string& host, int port) : host_(host), port_(port) {}
  ~PSServer() { stop(); }

  void start() {
    lfd_ = ::socket(AF_INET, SOCK_STREAM, 0);
    if (lfd_ < 0) throw std::runtime_error("ps: socket failed");
    int one = 1;
    setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons(static_cast<uint16_t>(port_));
    a.sin_addr.s_addr = (host_.empty() || host_ == "0.0.0.0") ? INADDR_ANY : inet_addr(host_.c_str());
    if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
      ::close(lfd_);
      lfd_ = -1;
      throw std::runtime_error("ps: bind failed on port " + std::to_string(port_));
    }
    if (port_ == 0) {
      socklen_t l = sizeof(a);
      getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &l);
      port_ = ntohs(a.sin_port);
    }
    ::listen(lfd_, 256);
    running_ = true;
    acc_ = std::thread([this] { accept_loop(); });
  }

  void stop() {
    if (!running_.exchange(false)) return;
    {
      std::lock_guard<std::mutex> g(sync_mu_);  // release sync pushers blocked in a round
      sync_cv_.notify_all();
    }
    // the accept thread polls lfd_ (100 ms ticks): join it BEFORE closing the fd, so it
    // never reads a closed (and possibly reused) descriptor
    if (lfd_ >= 0) ::shutdown(lfd_, SHUT_RDWR);
    if (acc_.joinable()) acc_.join();
    if (lfd_ >= 0) {
      ::close(lfd_);
      lfd_ = -1;
    }
    std::vector<std::thread> ts;
    {
      std::lock_guard<std::mutex> g(cmu_);
      for (int fd : conns_) ::shutdown(fd, SHUT_RDWR);
      ts.swap(threads_);
    }
    for (auto& t : ts)
      if (t.joinable()) t.join();
  }

  // block until a client sends SHUTDOWN or stop() is called
  void join() {
    while (running_ && !shutdown_req_) std::this_thread::sleep_for(std::chrono::milliseconds(20));
    stop();
  }

  int port() const { return port_; }
  size_t num_vars() {
    std::lock_guard<std::mutex> g(vmu_);
    return vars_.size();
  }
  py::dict stats() {
    py::dict d;
    d["pulls"] = pulls_.load();
    d["pushes"] = pushes_.load();
    d["bytes_in"] = bytes_in_.load();
    d["bytes_out"] = bytes_out_.load();
    d["sync_rounds"] = sync_rounds_.load();
    d["sync_stale"] = sync_stale_.load();
    d["sync_withdrawn"] = sync_withdrawn_.load();
    return d;
  }

 private:
  void accept_loop() {
    while (running_) {
      pollfd p{lfd_, POLLIN, 0};
      if (::poll(&p, 1, 100) <= 0) continue;
      const int fd = ::accept(lfd_, nullptr, nullptr);
      if (fd < 0) continue;
      tune(fd);
      std::lock_guard<std::mutex> g(cmu_);
      conns_.push_back(fd);
      threads_.emplace_back([this, fd] { serve(fd); });
    }
  }

  Var* var(uint32_t id) {
    std::lock_guard<std::mutex> g(vmu_);
    if (id >= vars_.size()) throw std::runtime_error("ps: bad variable id");
    return vars_[id].get();
  }

  // this connection thread's Hogwild start offset, in eighths of a variable (dtfx_hogwild_apply)
  static thread_local size_t rot_;
  void serve(int fd) {
    rot_ = static_cast<size_t>(conn_seq_.fetch_add(1)) % 8;
    // Request and reply buffers live for the connection: a fresh 318 KB reply string per pull
    // was an mmap'd allocation (above malloc's mmap threshold) whose pages the kernel zeroed
    // and faulted in on every request, and the reply was then copied once more behind its
    // header -- both on the ps's critical path, which bounds the async cluster's step rate.
    std::string req;
    std::vector<iovec> iov(2);
    Writer w;
    while (running_) {
      uint32_t len;
      if (!read_full(fd, &len, 4)) break;
      req.resize(len);
      if (!read_full(fd, &req[0], len)) break;
      bytes_in_ += len + 4;
      w.b.clear();
      uint8_t status = 0;
      try {
        handle(req, w);
      } catch (const std::exception& e) {
        status = 1;
        w.b = e.what();
      }
      char hdr[5];
      const uint32_t rl = static_cast<uint32_t>(w.b.size() + 1);
      std::memcpy(hdr, &rl, 4);
      hdr[4] = static_cast<char>(status);
      bytes_out_ += 5 + w.b.size();
      iov.resize(2);
      iov[0] = iovec{hdr, 5};
      iov[1] = iovec{const_cast<char*>(w.b.data()), w.b.size()};
      if (w.b.empty()) iov.resize(1);
      if (!writev_full(fd, iov)) break;
    }
    // deregister before closing: stop() shuts down the fds in conns_, and a closed fd number
    // can be reused by any other socket of the process
    std::lock_guard<std::mutex> g(cmu_);
    for (auto it = conns_.begin(); it != conns_.end(); ++it)
      if (*it == fd) {
        conns_.erase(it);
        break;
      }
    ::close(fd);
  }

  void handle(const std::string& req, Writer& w) {
    Reader r{req.data(), req.data() + req.size()};
    const uint8_t op = r.get<uint8_t>();
    switch (op) {
      case OP_PING: break;
      case OP_CREATE: {
        const std::string name = r.str();
        const uint8_t dt = r.get<uint8_t>();
        const uint8_t nd = r.get<uint8_t>();
        std::vector<int64_t> shape(nd);
        size_t count = 1;
        for (auto& d : shape) {
          d = r.get<int64_t>();
          count *= static_cast<size_t>(d);
        }
        std::lock_guard<std::mutex> g(vmu_);
        auto it = by_name_.find(name);
        if (it != by_name_.end()) {
          Var* v = vars_[it->second].get();
          if (v->dtype != dt || v->shape != shape)
            throw std::runtime_error("ps: variable " + name + " re-created with another dtype/shape");
          w.put<uint32_t>(it->second);
          break;
        }
        auto v = std::make_unique<Var>();
        v->name = name;
        v->dtype = dt;
        v->shape = shape;
        v->count = dt == DT_F32 ? count : 1;
        if (dt == DT_F32) v->f.assign(count, 0.f);
        const uint32_t id = static_cast<uint32_t>(vars_.size());
        vars_.push_back(std::move(v));
        by_name_[name] = id;
        w.put<uint32_t>(id);
        break;
      }
      case OP_LOOKUP: {
        const std::string name = r.str();
        std::lock_guard<std::mutex> g(vmu_);
        auto it = by_name_.find(name);
        if (it == by_name_.end()) throw std::runtime_error("ps: no variable " + name);
        w.put<uint32_t>(it->second);
        break;
      }
      case OP_ASSIGN: {
        Var* v = var(r.get<uint32_t>());
        const char* d = r.take(v->nbytes());
        std::lock_guard<std::mutex> g(v->mu);
        if (v->dtype == DT_F32) std::memcpy(v->f.data(), d, v->nbytes());
        else {
          int64_t x;
          std::memcpy(&x, d, 8);
          v->i.store(x);
        }
        v->init.store(true);
        break;
      }
      case OP_PULL: {
        const uint32_t n = r.get<uint32_t>();
        ++pulls_;
        for (uint32_t k = 0; k < n; ++k) {
          Var* v = var(r.get<uint32_t>());
          if (!v->init.load()) throw std::runtime_error("ps: variable " + v->name + " is uninitialized");
          if (v->dtype == DT_F32) dtfx_racy_read(w, v->f.data(), v->nbytes());  // lock-free (TF)
          else w.put<int64_t>(v->i.load());
        }
        break;
      }
      case OP_PUSH_APPLY: {
        const float lr = r.get<float>();
        const uint8_t locking = r.get<uint8_t>();
        const uint32_t n = r.get<uint32_t>();
        std::vector<Var*> vs(n);
        for (auto& v : vs) v = var(r.get<uint32_t>());
        ++pushes_;
        for (Var* v : vs) {
          if (v->dtype != DT_F32) throw std::runtime_error("ps: apply on non-float variable");
          const char* g = r.take(v->nbytes());
          float* p = v->f.data();
          const size_t cnt = v->count;
          if (locking) {
            // (still races with lock-free pulls, as in TF: the apply goes through the same
            // suppressed function)
            std::lock_guard<std::mutex> lk(v->mu);
            dtfx_hogwild_apply(p, g, cnt, lr);
          } else {
            // Hogwild, as ApplyGradientDescent(use_locking=False): concurrent
            // workers may interleave element updates.
            dtfx_hogwild_apply(p, g, cnt, lr, rot_ * cnt / 8 / 16 * 16);
          }
        }
        break;
      }
      case OP_FETCH_ADD: {
        Var* v = var(r.get<uint32_t>());
        const int64_t d = r.get<int64_t>();
        if (v->dtype != DT_I64) throw std::runtime_error("ps: fetch_add on non-int variable");
        if (!v->init.load()) throw std::runtime_error("ps: variable " + v->name + " is uninitialized");
        w.put<int64_t>(v->i.fetch_add(d));
        break;
      }
      case OP_UNINIT: {
        const uint32_t n = r.get<uint32_t>();
        std::vector<uint32_t> bad;
        for (uint32_t k = 0; k < n; ++k) {
          const uint32_t id = r.get<uint32_t>();
          if (!var(id)->init.load()) bad.push_back(id);
        }
        w.put<uint32_t>(static_cast<uint32_t>(bad.size()));
        for (uint32_t id : bad) w.put<uint32_t>(id);
        break;
      }
      case OP_LIST: {
        std::lock_guard<std::mutex> g(vmu_);
        w.put<uint32_t>(static_cast<uint32_t>(vars_.size()));
        for (auto& v : vars_) {
          w.str(v->name);
          w.put<uint8_t>(v->dtype);
          w.put<uint8_t>(static_cast<uint8_t>(v->shape.size()));
          for (int64_t d : v->shape) w.put<int64_t>(d);
          w.put<uint8_t>(v->init.load() ? 1 : 0);
        }
        break;
      }
      case OP_SYNC_PUSH: sync_push(r, w); break;
      case OP_SHUTDOWN: shutdown_req_ = true; break;
      default: throw std::runtime_error("ps: unknown op " + std::to_string(op));
    }
  }

  // SYNC_PUSH: lr f32 | R u32 | local_step i64 | step var id u32 (kNoVar: not on this task) |
  // timeout_ms u32 | n u32 | n ids | n gradients.  Reply: round (global step) after the push
  // i64 | applied-in-a-round u8 (0: dropped as stale).
  void sync_push(Reader& r, Writer& w) {
    const float lr = r.get<float>();
    const uint32_t R = r.get<uint32_t>();
    const int64_t local_step = r.get<int64_t>();
    const uint32_t step_id = r.get<uint32_t>();
    const uint32_t timeout_ms = r.get<uint32_t>();
    const uint32_t n = r.get<uint32_t>();
    if (R < 1) throw std::runtime_error("ps: replicas_to_aggregate must be >= 1");
    std::vector<Var*> vs(n);
    std::vector<uint32_t> ids(n);
    for (uint32_t k = 0; k < n; ++k) vs[k] = var(ids[k] = r.get<uint32_t>());
    Var* stepv = step_id == kNoVar ? nullptr : var(step_id);
    std::unique_lock<std::mutex> lk(sync_mu_);
    if (sync_gen_ < 0 || (sync_pending_.empty() && local_step > sync_gen_))
      sync_gen_ = local_step;  // first round of a (fresh or restored) job: adopt its step
    if (local_step < sync_gen_) {  // stale: its round was applied without it
      ++sync_stale_;
      w.put<int64_t>(sync_gen_);
      w.put<uint8_t>(0);
      return;
    }
    if (local_step > sync_gen_)
      throw std::runtime_error("ps: sync push from step " + std::to_string(local_step) +
                               " while round " + std::to_string(sync_gen_) + " is open");
    // this push's gradients are kept apart until its round closes: a push whose wait times
    // out is withdrawn EXACTLY (its entry removed), so a retried push is not counted twice and
    // a round never applies an abandoned gradient
    SyncPush mine;
    mine.token = ++sync_tokens_;
    for (uint32_t k = 0; k < n; ++k) {
      Var* v = vs[k];
      if (v->dtype != DT_F32) throw std::runtime_error("ps: sync push to a non-float variable");
      const char* g = r.take(v->nbytes());
      std::vector<float> gv(v->count);
      std::memcpy(gv.data(), g, v->nbytes());
      mine.grads.emplace_back(ids[k], std::move(gv));
    }
    sync_pending_.push_back(std::move(mine));
    const uint64_t token = sync_pending_.back().token;
    const int64_t round = sync_gen_;
    if (static_cast<int>(sync_pending_.size()) >= static_cast<int>(R)) {
      // apply the mean of the round's R gradients (SyncReplicasOptimizer averages), summed in
      // arrival order
      std::map<uint32_t, std::vector<float>> acc;
      for (const SyncPush& sp : sync_pending_)
        for (const auto& kv : sp.grads) {
          std::vector<float>& a = acc[kv.first];
          if (a.empty()) a.assign(kv.second.size(), 0.f);
          for (size_t i = 0; i < a.size(); ++i) a[i] += kv.second[i];
        }
      const float scale = lr / static_cast<float>(R);
      for (auto& kv : acc) {
        Var* v = var(kv.first);
        std::lock_guard<std::mutex> vl(v->mu);
        float* p = v->f.data();
        for (size_t i = 0; i < kv.second.size(); ++i) p[i] -= scale * kv.second[i];
      }
      sync_pending_.clear();
      ++sync_gen_;
      ++sync_rounds_;
      if (stepv) stepv->i.store(sync_gen_);
      sync_cv_.notify_all();
    } else if (!cv_wait_ms(sync_cv_, lk, timeout_ms,
                           [&] { return sync_gen_ > round || !running_; })) {
      const size_t have = sync_pending_.size();
      sync_pending_.erase(std::remove_if(sync_pending_.begin(), sync_pending_.end(),
                                         [&](const SyncPush& sp) { return sp.token == token; }),
                          sync_pending_.end());
      ++sync_withdrawn_;
      throw std::runtime_error("ps: sync round " + std::to_string(round) + " timed out with " +
                               std::to_string(have) + " of " + std::to_string(R) +
                               " replicas (this push was withdrawn)");
    }
    if (sync_gen_ <= round) throw std::runtime_error("ps: server stopped during a sync round");
    w.put<int64_t>(sync_gen_);
    w.put<uint8_t>(1);
  }

  std::string host_;
  int port_;
  int lfd_ = -1;
  std::atomic<bool> running_{false}, shutdown_req_{false};
  std::thread acc_;
  std::mutex cmu_, vmu_;
  std::atomic<int> conn_seq_{0};
  std::vector<int> conns_;
  std::vector<std::thread> threads_;
  std::vector<std::unique_ptr<Var>> vars_;
  std::map<std::string, uint32_t> by_name_;
  std::atomic<uint64_t> pulls_{0}, pushes_{0}, bytes_in_{0}, bytes_out_{0};
  std::mutex sync_mu_;
  std::condition_variable sync_cv_;
  int64_t sync_gen_ = -1;
  struct SyncPush {
    uint64_t token = 0;
    std::vector<std::pair<uint32_t, std::vector<float>>> grads;
  };
  std::vector<SyncPush> sync_pending_;  // the open round's pushes, in arrival order
  uint64_t sync_tokens_ = 0;
  std::atomic<uint64_t> sync_rounds_{0}, sync_stale_{0}, sync_withdrawn_{0};
};

thread_local size_t PSServer::rot_ = 0;

// ---------------------------------------------------------------- client
class PSClient {
 public:
  // rpc_timeout_s > 0: a ps that stays silent that long on a request counts as lost (a hung or
  // stopped ps ends the worker instead of blocking it forever); 0 = wait indefinitely.
  PSClient(std::vector<std::string> addrs, double connect_timeout_s, double rpc_timeout_s = 0.0)
      : addrs_(std::move(addrs)), rpc_timeout_s_(rpc_timeout_s) {
    for (auto& a : addrs_) {
      fds_.push_back(connect_to(a, connect_timeout_s));
      set_timeout(fds_.back(), rpc_timeout_s_);
    }
  }
  ~PSClient() {
    if (psp_.active) {
      // an exchange whose end() never came (mu_ still held by the thread that began it):
      // nobody can finish it, so do not wait for mu_ -- wake the sender, join it, then close.
      // If THIS thread began it, it owns mu_ and releases it here (a mutex must not be
      // destroyed locked).  Another thread's open exchange is a caller bug: that thread
      // would call end() on a freed client, so it is refused loudly instead.
      if (psp_owner_ != std::this_thread::get_id()) {
        fprintf(stderr, "PSClient destroyed while another thread has a push_step_pull "
                        "exchange open; aborting\n");
        std::abort();
      }
      for (int fd : fds_)
        if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
      stop_sender();
      close_fds();
      psp_.active = false;
      mu_.unlock();
      return;
    }
    if (PyGILState_Check()) {  // (Python dealloc): never wait for mu_ while holding the GIL
      py::gil_scoped_release nogil;
      close();
    } else {
      close();
    }
    stop_sender();
  }

  // Bound with the GIL released (py::call_guard): an exchange that another thread has open
  // (push_step_pull_begin .. end) holds mu_ while that thread runs Python WITH the GIL
  // (next_batch, stage) before it calls end(); waiting for mu_ here with the GIL held would
  // deadlock both threads.  Without the GIL, close() simply waits for that end().
  void close() {
    std::lock_guard<std::mutex> lk(mu_);
    close_fds();
  }
  void close_fds() {
    for (int& fd : fds_)
      if (fd >= 0) {
        ::close(fd);
        fd = -1;
      }
  }
  int num_tasks() const { return static_cast<int>(fds_.size()); }
  size_t task_of(int64_t h) const {
    const size_t t = static_cast<size_t>(static_cast<uint64_t>(h) >> 32);
    if (t >= fds_.size()) throw std::runtime_error("ps: handle of an unknown ps task");
    return t;
  }

  // handle = task << 32 | id
  int64_t create(const std::string& name, const std::string& dtype, std::vector<int64_t> shape,
                 int task) {
    Writer w;
    w.put<uint8_t>(OP_CREATE);
    w.str(name);
    w.put<uint8_t>(dt(dtype));
    w.put<uint8_t>(static_cast<uint8_t>(shape.size()));
    for (int64_t d : shape) w.put<int64_t>(d);
    std::string resp = locked_call(task, w.b);
    Reader r{resp.data(), resp.data() + resp.size()};
    return (static_cast<int64_t>(task) << 32) | r.get<uint32_t>();
  }
  int64_t lookup(const std::string& name, int task) {
    Writer w;
    w.put<uint8_t>(OP_LOOKUP);
    w.str(name);
    std::string resp = locked_call(task, w.b);
    Reader r{resp.data(), resp.data() + resp.size()};
    return (static_cast<int64_t>(task) << 32) | r.get<uint32_t>();
  }
  void assign(int64_t h, uintptr_t ptr, size_t nbytes) {
    Writer w;
    w.put<uint8_t>(OP_ASSIGN);
    w.put<uint32_t>(static_cast<uint32_t>(h));
    w.raw(reinterpret_cast<const void*>(ptr), nbytes);
    locked_call(static_cast<int>(h >> 32), w.b);
  }
  // pull a group of variables into caller buffers (sizes in bytes)
  void pull(std::vector<int64_t> hs, std::vector<uintptr_t> ptrs, std::vector<size_t> sizes) {
    if (hs.size() != ptrs.size() || hs.size() != sizes.size())
      throw std::runtime_error("ps pull: argument lengths differ");
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<std::vector<size_t>> per(fds_.size());
    for (size_t k = 0; k < hs.size(); ++k) per[task_of(hs[k])].push_back(k);
    for (size_t t = 0; t < per.size(); ++t) {
      if (per[t].empty()) continue;
      Writer w;
      w.put<uint8_t>(OP_PULL);
      w.put<uint32_t>(static_cast<uint32_t>(per[t].size()));
      for (size_t k : per[t]) w.put<uint32_t>(static_cast<uint32_t>(hs[k]));
      send(static_cast<int>(t), w.b);
    }
    // drain EVERY task's response before reporting a failure: an unread reply would stay
    // queued on its socket and answer the next call on that connection
    std::string first_error;
    bool lost = false;
    for (size_t t = 0; t < per.size(); ++t) {
      if (per[t].empty()) continue;
      try {
        std::string resp = recv(static_cast<int>(t));
        size_t off = 0;
        for (size_t k : per[t]) {
          if (off + sizes[k] > resp.size()) throw std::runtime_error("ps pull: short response");
          std::memcpy(reinterpret_cast<void*>(ptrs[k]), resp.data() + off, sizes[k]);
          off += sizes[k];
        }
      } catch (const PSConnectionLost& e) {
        if (first_error.empty()) first_error = e.what();
        lost = true;
      } catch (const std::exception& e) {
        if (first_error.empty()) first_error = e.what();
      }
    }
    if (lost) throw PSConnectionLost(first_error);
    if (!first_error.empty()) throw std::runtime_error(first_error);
  }
  // push gradients (f32) and apply var -= lr * grad on the owning ps tasks
  void push_apply(std::vector<int64_t> hs, std::vector<uintptr_t> ptrs, std::vector<size_t> sizes,
                  float lr, bool locking) {
    if (hs.size() != ptrs.size() || hs.size() != sizes.size())
      throw std::runtime_error("ps push: argument lengths differ");
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> lk(mu_);
    std::vector<std::vector<size_t>> per(fds_.size());
    for (size_t k = 0; k < hs.size(); ++k) per[task_of(hs[k])].push_back(k);
    for (size_t t = 0; t < per.size(); ++t) {
      if (per[t].empty()) continue;
      Writer w;
      w.put<uint8_t>(OP_PUSH_APPLY);
      w.put<float>(lr);
      w.put<uint8_t>(locking ? 1 : 0);
      w.put<uint32_t>(static_cast<uint32_t>(per[t].size()));
      for (size_t k : per[t]) w.put<uint32_t>(static_cast<uint32_t>(hs[k]));
      for (size_t k : per[t]) w.raw(reinterpret_cast<const void*>(ptrs[k]), sizes[k]);
      send(static_cast<int>(t), w.b);
    }
    std::string first_error;  // drain every task's reply first (see pull)
      bool lost = false;
    for (size_t t = 0; t < per.size(); ++t) {
      if (per[t].empty()) continue;
      try {
        recv(static_cast<int>(t));
      } catch (const PSConnectionLost& e) {
        if (first_error.empty()) first_error = e.what();
        lost = true;
      } catch (const std::exception& e) {
        if (first_error.empty()) first_error = e.what();
      }
    }
    if (lost) throw PSConnectionLost(first_error);
    if (!first_error.empty()) throw std::runtime_error(first_error);
  }
  // One worker step's ps traffic in ONE network round trip per task: push + apply (this
  // worker's gradients), fetch_add on global_step, and the pull of the parameters for the next
  // step, pipelined on each task's connection.  The ps serves a connection's requests in
  // order, so it applies the push, then advances the step, then reads the variables --
  // exactly the reference's train_op -> counter_op -> sync_op sequence (worker.py:135-141,
  // 131), three round trips there.  Returns the old step value.
  int64_t push_step_pull(std::vector<int64_t> hs, std::vector<uintptr_t> ptrs,
                         std::vector<size_t> sizes, float lr, bool locking, int64_t step_h,
                         int64_t delta, std::vector<int64_t> phs, std::vector<uintptr_t> pptrs,
                         std::vector<size_t> psizes) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> lk(mu_);
    psp_send(hs, ptrs, sizes, lr, locking, step_h, delta, phs, pptrs, psizes);
    return psp_recv();
  }
  // The same exchange split in two (train/worker.py): ``begin`` sends every request and
  // returns at once; the ps applies the push, advances the step and reads the parameters
  // while the caller prepares its next batch; ``end`` receives the replies (the pulled
  // parameters land in ``pptrs``) and returns the old step.  The client's lock is held from
  // begin to end (same thread), so no other request can interleave on the connections; every
  // begin must be followed by end (the Python side calls it in a ``finally``).
  void push_step_pull_begin(std::vector<int64_t> hs, std::vector<uintptr_t> ptrs,
                            std::vector<size_t> sizes, float lr, bool locking, int64_t step_h,
                            int64_t delta, std::vector<int64_t> phs, std::vector<uintptr_t> pptrs,
                            std::vector<size_t> psizes) {
    py::gil_scoped_release nogil;
    mu_.lock();
    try {
      if (psp_.active) throw std::runtime_error("ps push_step_pull_begin: an exchange is already open");
      check_usable();
      start_sender();
      psp_async_ = true;  // plan only; the sender thread writes it
      psp_send(hs, ptrs, sizes, lr, locking, step_h, delta, phs, pptrs, psizes);
      psp_async_ = false;
      {
        std::lock_guard<std::mutex> lk(smu_);
        send_state_.store(1, std::memory_order_release);
      }
      scv_.notify_one();
    } catch (...) {
      psp_async_ = false;
      psp_.active = false;
      mu_.unlock();
      throw;
    }
    psp_owner_ = std::this_thread::get_id();
    psp_.active = true;
  }
  int64_t push_step_pull_end() {
    py::gil_scoped_release nogil;
    if (!psp_.active) throw std::runtime_error("ps push_step_pull_end without begin");
    struct Unlock {
      PSClient* c;
      ~Unlock() {
        c->psp_.active = false;
        c->mu_.unlock();
      }
    } unlock{this};
    // the sender thread's write of this exchange must be complete (spin: it is usually done)
    while (send_state_.load(std::memory_order_acquire) == 1) __builtin_ia32_pause();
    send_state_.store(0, std::memory_order_relaxed);
    check_usable();
    if (send_bad_ >= 0) lost(send_bad_, "send");
    return psp_recv();
  }
  // Synchronous-replicas push (see SYNC_PUSH): every task gets its variables' gradients; the
  // task holding `step_handle` (global_step) advances it with each applied round.  Returns
  // (round after the push -- the new global step --, applied (False: dropped as stale)).
  py::tuple sync_push(std::vector<int64_t> hs, std::vector<uintptr_t> ptrs,
                      std::vector<size_t> sizes, float lr, int replicas_to_aggregate,
                      int64_t local_step, int64_t step_handle, double timeout_s) {
    if (hs.size() != ptrs.size() || hs.size() != sizes.size())
      throw std::runtime_error("ps sync_push: argument lengths differ");
    if (replicas_to_aggregate < 1) throw std::runtime_error("ps sync_push: replicas_to_aggregate < 1");
    int64_t round = -1;
    bool applied = true;
    {
      py::gil_scoped_release nogil;
      std::lock_guard<std::mutex> lk(mu_);
      std::vector<std::vector<size_t>> per(fds_.size());
      for (size_t k = 0; k < hs.size(); ++k) per[task_of(hs[k])].push_back(k);
      const size_t step_task = task_of(step_handle);
      const uint32_t tmo = static_cast<uint32_t>(std::min(timeout_s, 4.0e6) * 1000.0);
      // the ps holds this reply until the round closes (up to timeout_s): the rpc timeout
      // covers the silence AFTER that wait, restored on every exit path
      struct Extend {
        PSClient* c;
        double secs;
        Extend(PSClient* c_, double s_) : c(c_), secs(s_) {
          if (c->rpc_timeout_s_ > 0) for (int fd : c->fds_) set_timeout(fd, secs + c->rpc_timeout_s_);
        }
        ~Extend() {
          if (c->rpc_timeout_s_ > 0) for (int fd : c->fds_) set_timeout(fd, c->rpc_timeout_s_);
        }
      } extend(this, timeout_s);
      std::vector<bool> sent(fds_.size(), false);
      for (size_t t = 0; t < per.size(); ++t) {
        if (per[t].empty() && t != step_task) continue;
        Writer w;
        w.put<uint8_t>(OP_SYNC_PUSH);
        w.put<float>(lr);
        w.put<uint32_t>(static_cast<uint32_t>(replicas_to_aggregate));
        w.put<int64_t>(local_step);
        w.put<uint32_t>(t == step_task ? static_cast<uint32_t>(step_handle) : kNoVar);
        w.put<uint32_t>(tmo);
        w.put<uint32_t>(static_cast<uint32_t>(per[t].size()));
        for (size_t k : per[t]) w.put<uint32_t>(static_cast<uint32_t>(hs[k]));
        for (size_t k : per[t]) w.raw(reinterpret_cast<const void*>(ptrs[k]), sizes[k]);
        send(static_cast<int>(t), w.b);
        sent[t] = true;
      }
      std::string first_error;  // drain every task's reply first (see pull)
      bool lost = false;
      for (size_t t = 0; t < per.size(); ++t) {
        if (!sent[t]) continue;
        try {
          std::string resp = recv(static_cast<int>(t));
          Reader r{resp.data(), resp.data() + resp.size()};
          const int64_t g = r.get<int64_t>();
          const bool a = r.get<uint8_t>() != 0;
          if (t == step_task || round < 0) round = g;
          applied = applied && a;
        } catch (const PSConnectionLost& e) {
          if (first_error.empty()) first_error = e.what();
          lost = true;
        } catch (const std::exception& e) {
          if (first_error.empty()) first_error = e.what();
        }
      }
      if (lost) throw PSConnectionLost(first_error);
    if (!first_error.empty()) throw std::runtime_error(first_error);
    }
    return py::make_tuple(round, applied);
  }
  int64_t fetch_add(int64_t h, int64_t delta) {
    Writer w;
    w.put<uint8_t>(OP_FETCH_ADD);
    w.put<uint32_t>(static_cast<uint32_t>(h));
    w.put<int64_t>(delta);
    std::string resp = locked_call(static_cast<int>(h >> 32), w.b);
    Reader r{resp.data(), resp.data() + resp.size()};
    return r.get<int64_t>();
  }
  std::vector<int64_t> uninitialized(std::vector<int64_t> hs) {
    std::vector<int64_t> out;
    std::vector<std::vector<int64_t>> per(fds_.size());
    for (int64_t h : hs) per[task_of(h)].push_back(h);
    for (size_t t = 0; t < per.size(); ++t) {
      if (per[t].empty()) continue;
      Writer w;
      w.put<uint8_t>(OP_UNINIT);
      w.put<uint32_t>(static_cast<uint32_t>(per[t].size()));
      for (int64_t h : per[t]) w.put<uint32_t>(static_cast<uint32_t>(h));
      std::string resp = locked_call(static_cast<int>(t), w.b);
      Reader r{resp.data(), resp.data() + resp.size()};
      const uint32_t n = r.get<uint32_t>();
      for (uint32_t k = 0; k < n; ++k)
        out.push_back((static_cast<int64_t>(t) << 32) | r.get<uint32_t>());
    }
    return out;
  }
  py::list list_vars(int task) {
    Writer w;
    w.put<uint8_t>(OP_LIST);
    std::string resp = locked_call(task, w.b);
    Reader r{resp.data(), resp.data() + resp.size()};
    py::list out;
    const uint32_t n = r.get<uint32_t>();
    for (uint32_t k = 0; k < n; ++k) {
      std::string name = r.str();
      const uint8_t d = r.get<uint8_t>();
      const uint8_t nd = r.get<uint8_t>();
      std::vector<int64_t> shape(nd);
      for (auto& s : shape) s = r.get<int64_t>();
      const bool init = r.get<uint8_t>() != 0;
      out.append(py::make_tuple(name, d == DT_F32 ? "float32" : "int64", shape, init));
    }
    return out;
  }
  void ping(int task) {
    Writer w;
    w.put<uint8_t>(OP_PING);
    locked_call(task, w.b);
  }
  void shutdown_server(int task) {
    Writer w;
    w.put<uint8_t>(OP_SHUTDOWN);
    locked_call(task, w.b);
  }

 private:
  // push_step_pull, send half (mu_ held by the caller): per task, the push + apply of its
  // gradients, the fetch_add on global_step (its task only) and the pull of its variables,
  // framed back to back and written with one call.  The reply plan stays in psp_.
  void psp_send(const std::vector<int64_t>& hs, const std::vector<uintptr_t>& ptrs,
                const std::vector<size_t>& sizes, float lr, bool locking, int64_t step_h,
                int64_t delta, const std::vector<int64_t>& phs, const std::vector<uintptr_t>& pptrs,
                const std::vector<size_t>& psizes) {
    if (hs.size() != ptrs.size() || hs.size() != sizes.size() || phs.size() != pptrs.size() ||
        phs.size() != psizes.size())
      throw std::runtime_error("ps push_step_pull: argument lengths differ");
    check_usable();
    const size_t T = fds_.size();
    psp_.step_task = task_of(step_h);
    psp_.per.assign(T, {});
    psp_.pper.assign(T, {});
    psp_.pptrs = pptrs;
    psp_.psizes = psizes;
    auto& per = psp_.per;
    auto& pper = psp_.pper;
    for (size_t k = 0; k < hs.size(); ++k) per[task_of(hs[k])].push_back(k);
    for (size_t k = 0; k < phs.size(); ++k) pper[task_of(phs[k])].push_back(k);
    psp_.hdrs.assign(T, std::string());
    psp_.tails.assign(T, std::string());
    psp_.iov.assign(T, {});
    for (size_t t = 0; t < T; ++t) {
      // the task's requests, framed, sent with ONE gather-write: the headers from small
      // strings, the gradient payload straight from the caller's buffers (no copy).  The plan
      // lives in psp_ until it is sent (inline, or by the sender thread: psp_begin_async)
      std::string& hdr = psp_.hdrs[t];
      std::vector<iovec>& iov = psp_.iov[t];
      if (!per[t].empty()) {
        size_t payload = 0;
        for (size_t k : per[t]) payload += sizes[k];
        Writer w;
        w.put<uint8_t>(OP_PUSH_APPLY);
        w.put<float>(lr);
        w.put<uint8_t>(locking ? 1 : 0);
        w.put<uint32_t>(static_cast<uint32_t>(per[t].size()));
        for (size_t k : per[t]) w.put<uint32_t>(static_cast<uint32_t>(hs[k]));
        const uint32_t len = static_cast<uint32_t>(w.b.size() + payload);
        hdr.assign(reinterpret_cast<const char*>(&len), 4);
        hdr.append(w.b);
        iov.push_back({const_cast<char*>(hdr.data()), hdr.size()});
        for (size_t k : per[t])
          if (sizes[k]) iov.push_back({reinterpret_cast<void*>(ptrs[k]), sizes[k]});
      }
      std::string& tail = psp_.tails[t];  // fetch_add + pull frames
      auto frame = [&](const Writer& w) {
        const uint32_t len = static_cast<uint32_t>(w.b.size());
        tail.append(reinterpret_cast<const char*>(&len), 4);
        tail.append(w.b);
      };
      if (t == psp_.step_task) {
        Writer w;
        w.put<uint8_t>(OP_FETCH_ADD);
        w.put<uint32_t>(static_cast<uint32_t>(step_h));
        w.put<int64_t>(delta);
        frame(w);
      }
      if (!pper[t].empty()) {
        Writer w;
        w.put<uint8_t>(OP_PULL);
        w.put<uint32_t>(static_cast<uint32_t>(pper[t].size()));
        for (size_t k : pper[t]) w.put<uint32_t>(static_cast<uint32_t>(phs[k]));
        frame(w);
      }
      if (!tail.empty()) iov.push_back({const_cast<char*>(tail.data()), tail.size()});
    }
    if (!psp_async_) psp_write();
  }
  // The planned writes (the caller's thread, or the sender thread; mu_ held by the exchange).
  // Returns the index of a task whose connection failed, or -1.
  int psp_write_tasks() {
    for (size_t t = 0; t < psp_.iov.size(); ++t)
      if (!psp_.iov[t].empty() && !writev_full(fds_[t], psp_.iov[t])) return static_cast<int>(t);
    return -1;
  }
  void psp_write() {
    check_usable();
    const int bad = psp_write_tasks();
    if (bad >= 0) lost(bad, "send");
  }
  // Sender thread of the split-phase exchange (push_step_pull_begin with a background send):
  // the request bytes -- 318 KB of gradient for the reference MLP -- are copied into the
  // socket by this thread while the caller stages its next batch; push_step_pull_end waits
  // for it.  It spins briefly between exchanges (they come every ~0.1 ms), then sleeps.
  // Spins before the sender sleeps (DTFX_PS_SENDER_SPINS, default 20000): several workers per
  // host each spinning a sender thread compete with the ps threads for the CPU share.
  static int sender_spins() {
    static const int n = [] {
      const char* e = getenv("DTFX_PS_SENDER_SPINS");
      return e ? std::max(0, atoi(e)) : 20000;
    }();
    return n;
  }
  void sender_loop() {
    const int max_spins = sender_spins();
    while (true) {
      int spins = 0;
      while (send_state_.load(std::memory_order_acquire) != 1) {
        if (sender_stop_.load(std::memory_order_acquire)) return;
        if (++spins < max_spins) {
          __builtin_ia32_pause();
        } else {
          std::unique_lock<std::mutex> lk(smu_);
          cv_wait_ms(scv_, lk, 5, [this] {
            return send_state_.load(std::memory_order_acquire) == 1 ||
                   sender_stop_.load(std::memory_order_acquire);
          });
          spins = 0;
        }
      }
      send_bad_ = psp_write_tasks();
      send_state_.store(2, std::memory_order_release);
    }
  }
  void start_sender() {
    if (sender_.joinable()) return;
    sender_stop_.store(false, std::memory_order_release);
    sender_ = std::thread([this] { sender_loop(); });
  }
  void stop_sender() {
    if (!sender_.joinable()) return;
    {
      std::lock_guard<std::mutex> lk(smu_);
      sender_stop_.store(true, std::memory_order_release);
    }
    scv_.notify_all();
    sender_.join();
  }
  // A pull reply read straight into the destination buffers (status byte, then the variables'
  // bytes in request order): no intermediate response string.
  void recv_pull_into(int task, const std::vector<size_t>& ks) {
    check_usable();
    uint32_t len;
    if (!read_full(fds_[task], &len, 4)) lost(task, "recv");
    if (len < 1) throw std::runtime_error("ps: empty response");
    uint8_t status;
    if (!read_full(fds_[task], &status, 1)) lost(task, "recv body");
    size_t want = 0;
    for (size_t k : ks) want += psp_.psizes[k];
    if (status != 0 || len - 1 != want) {  // an error string (or an unexpected size): drain it
      std::string rest(len - 1, '\0');
      if (len > 1 && !read_full(fds_[task], &rest[0], len - 1)) lost(task, "recv body");
      if (status != 0) throw std::runtime_error(rest);
      throw std::runtime_error("ps pull: response size mismatch");
    }
    for (size_t k : ks)
      if (psp_.psizes[k] && !read_full(fds_[task], reinterpret_cast<void*>(psp_.pptrs[k]),
                                       psp_.psizes[k]))
        lost(task, "recv body");
  }
  // push_step_pull, receive half: drains every reply (see pull) and returns the old step.
  int64_t psp_recv() {
    const size_t T = fds_.size(), step_task = psp_.step_task;
    const auto& per = psp_.per;
    const auto& pper = psp_.pper;
    int64_t old = -1;
    std::string first_error;
    bool lost_conn = false;
    for (size_t t = 0; t < T; ++t) {
      const int n_req = (per[t].empty() ? 0 : 1) + (t == step_task ? 1 : 0) + (pper[t].empty() ? 0 : 1);
      for (int q = 0; q < n_req; ++q) {
        try {
          const bool is_push = q == 0 && !per[t].empty();
          const bool is_step = t == step_task && q == (per[t].empty() ? 0 : 1);
          if (!is_push && !is_step) {  // the pull: straight into the caller's buffers
            recv_pull_into(static_cast<int>(t), pper[t]);
            continue;
          }
          std::string resp = recv(static_cast<int>(t));
          if (is_push) continue;
          Reader r{resp.data(), resp.data() + resp.size()};
          old = r.get<int64_t>();
        } catch (const PSConnectionLost& e) {
          if (first_error.empty()) first_error = e.what();
          lost_conn = true;
          break;  // nothing more arrives on a lost connection
        } catch (const std::exception& e) {
          if (first_error.empty()) first_error = e.what();
        }
      }
    }
    if (lost_conn) throw PSConnectionLost(first_error);
    if (!first_error.empty()) throw std::runtime_error(first_error);
    return old;
  }
  struct PendingPSP {
    bool active = false;
    size_t step_task = 0;
    std::vector<std::vector<size_t>> per, pper;
    std::vector<uintptr_t> pptrs;
    std::vector<size_t> psizes;
    std::vector<std::string> hdrs, tails;  // the planned writes' own bytes, per task
    std::vector<std::vector<iovec>> iov;
  } psp_;
  std::thread::id psp_owner_;  // the thread holding mu_ for the open exchange
  bool psp_async_ = false;
  std::thread sender_;
  std::mutex smu_;
  std::condition_variable scv_;
  std::atomic<int> send_state_{0};  // 0 idle, 1 planned (sender writes), 2 written
  int send_bad_ = -1;
  std::atomic<bool> sender_stop_{false};

  static uint8_t dt(const std::string& s) {
    if (s == "float32") return DT_F32;
    if (s == "int64" || s == "int32") return DT_I64;
    throw std::runtime_error("ps: unsupported dtype " + s);
  }
  static void set_timeout(int fd, double secs) {
    timeval tv{};
    if (secs > 0) {
      tv.tv_sec = static_cast<time_t>(secs);
      tv.tv_usec = static_cast<suseconds_t>((secs - static_cast<double>(tv.tv_sec)) * 1e6);
    }
    setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
    setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
  }
  static int connect_to(const std::string& addr, double timeout_s) {
    const auto c = addr.rfind(':');
    if (c == std::string::npos) throw std::runtime_error("ps: bad address " + addr);
    const std::string host = addr.substr(0, c), port = addr.substr(c + 1);
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    while (true) {
      addrinfo hints{}, *res = nullptr;
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      if (getaddrinfo(host.c_str(), port.c_str(), &hints, &res) == 0 && res) {
        const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
        if (fd >= 0 && ::connect(fd, res->ai_addr, res->ai_addrlen) == 0) {
          freeaddrinfo(res);
          tune(fd);
          return fd;
        }
        if (fd >= 0) ::close(fd);
        freeaddrinfo(res);
      }
      if (std::chrono::steady_clock::now() > deadline)
        throw std::runtime_error("ps: cannot connect to " + addr);
      std::this_thread::sleep_for(std::chrono::milliseconds(50));  // ps not up yet (run_*.sh sleep 1)
    }
  }
  // A lost or timed-out connection (SO_RCVTIMEO can fire in the middle of a frame) makes the
  // whole client unusable: every socket is closed, so a later call -- e.g. the Supervisor's
  // saver thread on the same client -- can never read the late or partial reply of the
  // abandoned request as its own response; it throws PSConnectionLost at once instead.
  [[noreturn]] void lost(int task, const char* what) {
    if (broken_.empty()) broken_ = "ps: connection to " + addrs_[task] + " lost (" + what + ")";
    for (int& fd : fds_)
      if (fd >= 0) {
        ::close(fd);
        fd = -1;
      }
    throw PSConnectionLost(broken_);
  }
  void check_usable() const {
    if (!broken_.empty())
      throw PSConnectionLost("ps: client unusable after an earlier connection loss: " + broken_);
  }
  void send(int task, const std::string& payload) {
    check_usable();
    if (task < 0 || task >= static_cast<int>(fds_.size()) || fds_[task] < 0)
      throw std::runtime_error("ps: bad task");
    const uint32_t len = static_cast<uint32_t>(payload.size());
    if (!write_full(fds_[task], &len, 4) || !write_full(fds_[task], payload.data(), payload.size()))
      lost(task, "send");
  }
  std::string recv(int task) {
    check_usable();
    uint32_t len;
    if (!read_full(fds_[task], &len, 4)) lost(task, "recv");
    std::string resp(len, '\0');
    if (!read_full(fds_[task], &resp[0], len)) lost(task, "recv body");
    if (resp.empty()) throw std::runtime_error("ps: empty response");
    if (resp[0] != 0) throw std::runtime_error(resp.substr(1));
    return resp.substr(1);
  }
  std::string call(int task, const std::string& payload) {
    send(task, payload);
    return recv(task);
  }
  // Thread-safe exchange; drops the GIL while blocked on the mutex and the socket.
  std::string locked_call(int task, const std::string& payload) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::mutex> lk(mu_);
    return call(task, payload);
  }

  std::vector<std::string> addrs_;
  double rpc_timeout_s_ = 0.0;
  std::vector<int> fds_;
  std::string broken_;  // set by the first connection loss (see lost())
  std::mutex mu_;  // one request/response exchange at a time (shared by Python threads)
};

}  // namespace

void register_ps(py::module_& m) {
  py::register_exception<PSConnectionLost>(m, "PSConnectionLost", PyExc_ConnectionError);
  py::class_<PSServer>(m, "PSServer")
      .def(py::init<const std::string&, int>(), py::arg("host") = "127.0.0.1", py::arg("port") = 0)
      .def("start", &PSServer::start)
      .def("stop", &PSServer::stop, py::call_guard<py::gil_scoped_release>())
      .def("join", &PSServer::join, py::call_guard<py::gil_scoped_release>())
      .def("num_vars", &PSServer::num_vars)
      .def("stats", &PSServer::stats)
      .def_property_readonly("port", &PSServer::port);
  py::class_<PSClient>(m, "PSClient")
      .def(py::init<std::vector<std::string>, double, double>(), py::arg("addresses"),
           py::arg("connect_timeout") = 60.0, py::arg("rpc_timeout") = 0.0)
      .def("create", &PSClient::create, py::arg("name"), py::arg("dtype"), py::arg("shape"),
           py::arg("task"))
      .def("lookup", &PSClient::lookup, py::arg("name"), py::arg("task"))
      .def("assign", &PSClient::assign)
      .def("pull", &PSClient::pull)
      .def("push_apply", &PSClient::push_apply, py::arg("handles"), py::arg("ptrs"),
           py::arg("sizes"), py::arg("lr"), py::arg("use_locking") = false)
      .def("sync_push", &PSClient::sync_push, py::arg("handles"), py::arg("ptrs"),
           py::arg("sizes"), py::arg("lr"), py::arg("replicas_to_aggregate"),
           py::arg("local_step"), py::arg("step_handle"), py::arg("timeout_s") = 600.0)
      .def("fetch_add", &PSClient::fetch_add)
      .def("push_step_pull", &PSClient::push_step_pull, py::arg("handles"), py::arg("ptrs"),
           py::arg("sizes"), py::arg("lr"), py::arg("use_locking"), py::arg("step_handle"),
           py::arg("delta"), py::arg("pull_handles"), py::arg("pull_ptrs"),
           py::arg("pull_sizes"))
      .def("push_step_pull_begin", &PSClient::push_step_pull_begin, py::arg("handles"),
           py::arg("ptrs"), py::arg("sizes"), py::arg("lr"), py::arg("use_locking"),
           py::arg("step_handle"), py::arg("delta"), py::arg("pull_handles"),
           py::arg("pull_ptrs"), py::arg("pull_sizes"))
      .def("push_step_pull_end", &PSClient::push_step_pull_end)
      .def("uninitialized", &PSClient::uninitialized)
      .def("list_vars", &PSClient::list_vars)
      .def("ping", &PSClient::ping)
      .def("shutdown_server", &PSClient::shutdown_server)
      .def("close", &PSClient::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("num_tasks", &PSClient::num_tasks);
}
