// CPU collective backend over a TCP full mesh (gloo's role in the reference stack,
// SURVEY.md §2.2 T5b). Ring reduce-scatter + all-gather for all-reduce, ring all-gather,
// pipelined chain broadcast, pairwise all-to-all. Collectives run strictly in submission
// order on one worker thread per communicator, so every rank issues the same wire sequence.
// Device (GPU) tensors are staged through host memory, so the same backend also runs
// multi-rank DDP on GPU tensors where RCCL cannot (e.g. several ranks sharing one GPU).
#include <arpa/inet.h>
#include <fcntl.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <thread>

#include "comm/comm.h"

namespace xddp {

namespace {

class CpuWork : public Work {
 public:
  bool is_completed() override {
    std::lock_guard<std::mutex> g(mu);
    return done;
  }
  void wait() override {
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return done; });
    if (err) std::rethrow_exception(err);
  }
  void finish(std::exception_ptr e) {
    {
      std::lock_guard<std::mutex> g(mu);
      done = true;
      err = e;
    }
    cv.notify_all();
  }
  Timing timing_state() override {
    if (!timed) return Timing::kNone;
    std::lock_guard<std::mutex> g(mu);
    return done ? Timing::kReady : Timing::kPending;
  }
  double comm_ms() override { return (t1 - t0) * 1e-6; }
  double comm_ms_before(const TimeRef& ref) override {
    return std::max<double>(0.0, std::min<int64_t>(ref.ns, t1) - t0) * 1e-6;
  }
  std::mutex mu;
  std::condition_variable cv;
  bool done = false;
  std::exception_ptr err;
  bool timed = false;
  int64_t t0 = 0, t1 = 0;  // worker-thread clock around the collective (timed works)
};

// A host-staged collective on device tensors: wait() finishes the host collective, then copies
// each host result back into its device tensor on the waiter's current stream (once).
class StagedWork : public Work {
 public:
  bool is_completed() override { return inner->is_completed(); }
  Timing timing_state() override { return inner->timing_state(); }
  double comm_ms() override { return inner->comm_ms(); }
  double comm_ms_before(const TimeRef& ref) override { return inner->comm_ms_before(ref); }
  void wait() override {
    inner->wait();
    std::lock_guard<std::mutex> g(mu);
    if (copied) return;
    for (auto& p : back) p.first.copy_(p.second);
    copied = true;
  }
  std::shared_ptr<Work> inner;
  std::vector<std::pair<at::Tensor, at::Tensor>> back;  // (device tensor, host result)
  std::mutex mu;
  bool copied = false;
};

void set_nonblock(int fd, bool nb) {
  int fl = ::fcntl(fd, F_GETFL, 0);
  ::fcntl(fd, F_SETFL, nb ? (fl | O_NONBLOCK) : (fl & ~O_NONBLOCK));
}

}  // namespace

class TcpComm : public Comm {
 public:
  TcpComm(std::shared_ptr<Store> store, int rank, int size, std::chrono::milliseconds timeout, std::string host)
      : Comm(rank, size), store_(std::move(store)), timeout_(timeout) {
    peers_.assign(size, -1);
    if (size > 1) connect_mesh(host);
    worker_ = std::thread([this] { run(); });
  }
  ~TcpComm() override { shutdown(); }

  std::string backend() const override { return "cpu"; }

  void shutdown() override {
    {
      std::lock_guard<std::mutex> g(qmu_);
      if (stop_) return;
      stop_ = true;
    }
    qcv_.notify_all();
    if (worker_.joinable()) worker_.join();
    for (int fd : peers_)
      if (fd >= 0) ::close(fd);
    peers_.assign(size_, -1);
  }

  // Device tensors (gloo's CUDA support): staged through host memory. The device-to-host copy
  // runs on the caller's current stream (ordered after the producer kernels); the copy back runs
  // in wait() on the waiter's current stream, so consumers are ordered after it.
  std::shared_ptr<Work> allreduce(at::Tensor t, RedOp op, double premul) override {
    if (t.is_cuda()) {
      auto h = t.cpu();
      return staged(host_allreduce(h, op, premul), {{t, h}});
    }
    return host_allreduce(t, op, premul);
  }
  std::shared_ptr<Work> broadcast(at::Tensor t, int root) override {
    if (t.is_cuda()) {
      auto h = t.cpu();
      return staged(host_broadcast(h, root), {{t, h}});
    }
    return host_broadcast(t, root);
  }
  std::shared_ptr<Work> allgather(at::Tensor out, at::Tensor in) override {
    TORCH_CHECK(out.numel() == in.numel() * size_, "allgather: output must hold size*input elements");
    if (out.is_cuda() || in.is_cuda()) {
      auto ho = at::empty(out.sizes(), out.options().device(at::kCPU));
      return staged(host_allgather(ho, in.cpu()), {{out, ho}});
    }
    return host_allgather(out, in);
  }
  std::shared_ptr<Work> reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) override {
    TORCH_CHECK(in.numel() == out.numel() * size_, "reduce_scatter: input must hold size*output elements");
    if (out.is_cuda() || in.is_cuda()) {
      auto ho = at::empty(out.sizes(), out.options().device(at::kCPU));
      return staged(host_reduce_scatter(ho, in.cpu(), op), {{out, ho}});
    }
    return host_reduce_scatter(out, in, op);
  }
  std::shared_ptr<Work> alltoall(at::Tensor out, at::Tensor in) override {
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % size_ == 0, "alltoall: equal splits required");
    if (out.is_cuda() || in.is_cuda()) {
      auto ho = at::empty(out.sizes(), out.options().device(at::kCPU));
      return staged(host_alltoall(ho, in.cpu()), {{out, ho}});
    }
    return host_alltoall(out, in);
  }
  std::shared_ptr<Work> send(at::Tensor t, int dst) override {
    auto h = t.is_cuda() ? t.cpu() : t;
    auto w = enqueue("send", h, {h}, [=]() mutable {
      auto c = h.contiguous();
      send_all(peers_.at(dst), c.data_ptr(), c.nbytes());
    });
    return t.is_cuda() ? staged(w, {}) : w;
  }
  std::shared_ptr<Work> recv(at::Tensor t, int src) override {
    auto h = t.is_cuda() ? at::empty(t.sizes(), t.options().device(at::kCPU)) : t;
    auto w = enqueue("recv", h, {h}, [=]() mutable {
      auto c = h.is_contiguous() ? h : at::empty_like(h, at::MemoryFormat::Contiguous);
      recv_all(peers_.at(src), c.data_ptr(), c.nbytes());
      if (!h.is_contiguous()) h.copy_(c);
    });
    return t.is_cuda() ? staged(w, {{t, h}}) : w;
  }
  std::shared_ptr<Work> barrier() override {
    auto t = at::ones({1}, at::kInt);
    return enqueue("barrier", t, {}, [=]() mutable { do_allreduce(t, RedOp::SUM, 1.0); });
  }

 private:
  std::shared_ptr<Work> host_allreduce(at::Tensor t, RedOp op, double premul) {
    return enqueue("allreduce", t, {t}, [=]() mutable { do_allreduce(t, op, premul); });
  }
  std::shared_ptr<Work> host_broadcast(at::Tensor t, int root) {
    return enqueue("broadcast", t, {t}, [=]() mutable { do_broadcast(t, root); });
  }
  std::shared_ptr<Work> host_allgather(at::Tensor out, at::Tensor in) {
    return enqueue("allgather", in, {out}, [=]() mutable { do_allgather(out, in); });
  }
  std::shared_ptr<Work> host_reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) {
    return enqueue("reduce_scatter", in, {out}, [=]() mutable { do_reduce_scatter(out, in, op); });
  }
  std::shared_ptr<Work> host_alltoall(at::Tensor out, at::Tensor in) {
    return enqueue("alltoall", in, {out}, [=]() mutable { do_alltoall(out, in); });
  }

  std::shared_ptr<Work> staged(std::shared_ptr<Work> inner, std::vector<std::pair<at::Tensor, at::Tensor>> back) {
    auto w = std::make_shared<StagedWork>();
    w->inner = std::move(inner);
    w->back = std::move(back);
    w->seq = w->inner->seq;
    w->collective = w->inner->collective;
    for (auto& p : w->back) w->outputs.push_back(p.first);
    return w;
  }

  // ---------------- mesh setup ----------------
  void connect_mesh(const std::string& host) {
    int lfd = ::socket(AF_INET, SOCK_STREAM, 0);
    int one = 1;
    ::setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_addr.s_addr = htonl(INADDR_ANY);
    a.sin_port = 0;
    TORCH_CHECK(::bind(lfd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0, "xddp cpu comm: bind failed");
    TORCH_CHECK(::listen(lfd, size_) == 0, "xddp cpu comm: listen failed");
    socklen_t sl = sizeof(a);
    ::getsockname(lfd, reinterpret_cast<sockaddr*>(&a), &sl);
    const int port = ntohs(a.sin_port);
    store_->set("tcpcomm/addr/" + std::to_string(rank_), host + ":" + std::to_string(port));
    // connect to lower ranks
    for (int p = 0; p < rank_; ++p) {
      std::string addr = store_->get("tcpcomm/addr/" + std::to_string(p));
      auto colon = addr.rfind(':');
      int fd = dial(addr.substr(0, colon), std::stoi(addr.substr(colon + 1)));
      int32_t me = rank_;
      send_all(fd, &me, sizeof(me));
      peers_[p] = fd;
    }
    // accept higher ranks
    for (int k = rank_ + 1; k < size_; ++k) {
      pollfd pf{lfd, POLLIN, 0};
      int pr = ::poll(&pf, 1, static_cast<int>(timeout_.count()));
      TORCH_CHECK(pr > 0, "xddp cpu comm: timed out waiting for peer connections");
      int fd = ::accept(lfd, nullptr, nullptr);
      TORCH_CHECK(fd >= 0, "xddp cpu comm: accept failed");
      int32_t who = -1;
      recv_all(fd, &who, sizeof(who));
      TORCH_CHECK(who > rank_ && who < size_ && peers_[who] < 0, "xddp cpu comm: bad handshake");
      peers_[who] = fd;
    }
    ::close(lfd);
    for (int fd : peers_) {
      if (fd < 0) continue;
      ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      int buf = 4 << 20;
      ::setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
      ::setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
    }
  }

  int dial(const std::string& host, int port) {
    auto deadline = std::chrono::steady_clock::now() + timeout_;
    while (std::chrono::steady_clock::now() < deadline) {
      addrinfo hints{};
      hints.ai_family = AF_INET;
      hints.ai_socktype = SOCK_STREAM;
      addrinfo* res = nullptr;
      if (::getaddrinfo(host.c_str(), std::to_string(port).c_str(), &hints, &res) == 0) {
        for (addrinfo* r = res; r; r = r->ai_next) {
          int fd = ::socket(r->ai_family, r->ai_socktype, r->ai_protocol);
          if (fd >= 0 && ::connect(fd, r->ai_addr, r->ai_addrlen) == 0) {
            ::freeaddrinfo(res);
            return fd;
          }
          if (fd >= 0) ::close(fd);
        }
        ::freeaddrinfo(res);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    TORCH_CHECK(false, "xddp cpu comm: could not connect to peer ", host, ":", port);
  }

  // ---------------- raw transfer ----------------
  void send_all(int fd, const void* p, size_t n) { exchange(fd, p, n, -1, nullptr, 0); }
  void recv_all(int fd, void* p, size_t n) { exchange(-1, nullptr, 0, fd, p, n); }

  // Concurrently send `sn` bytes on sfd and receive `rn` bytes on rfd (fds may coincide).
  void exchange(int sfd, const void* sbuf, size_t sn, int rfd, void* rbuf, size_t rn) {
    size_t so = 0, ro = 0;
    if (sfd >= 0) set_nonblock(sfd, true);
    if (rfd >= 0) set_nonblock(rfd, true);
    auto last_progress = std::chrono::steady_clock::now();
    while (so < sn || ro < rn) {
      pollfd fds[2];
      int nf = 0;
      if (sfd >= 0 && sfd == rfd) {
        fds[nf++] = {sfd, static_cast<short>((so < sn ? POLLOUT : 0) | (ro < rn ? POLLIN : 0)), 0};
      } else {
        if (so < sn) fds[nf++] = {sfd, POLLOUT, 0};
        if (ro < rn) fds[nf++] = {rfd, POLLIN, 0};
      }
      int pr = ::poll(fds, nf, 1000);
      if (pr < 0 && errno != EINTR) TORCH_CHECK(false, "xddp cpu comm: poll failed: ", std::strerror(errno));
      bool progressed = false;
      for (int i = 0; i < nf; ++i) {
        if ((fds[i].revents & POLLOUT) && so < sn) {
          ssize_t w = ::send(fds[i].fd, static_cast<const char*>(sbuf) + so, sn - so, MSG_NOSIGNAL);
          if (w > 0) {
            so += w;
            progressed = true;
          } else if (w < 0 && errno != EAGAIN && errno != EINTR) {
            TORCH_CHECK(false, "xddp cpu comm: send failed (peer gone?): ", std::strerror(errno));
          }
        }
        if ((fds[i].revents & (POLLIN | POLLHUP | POLLERR)) && ro < rn) {
          ssize_t r = ::recv(fds[i].fd, static_cast<char*>(rbuf) + ro, rn - ro, 0);
          if (r > 0) {
            ro += r;
            progressed = true;
          } else if (r == 0) {
            TORCH_CHECK(false, "xddp cpu comm: peer closed connection");
          } else if (errno != EAGAIN && errno != EINTR) {
            TORCH_CHECK(false, "xddp cpu comm: recv failed: ", std::strerror(errno));
          }
        }
      }
      auto now = std::chrono::steady_clock::now();
      if (progressed) {
        last_progress = now;
      } else if (now - last_progress > timeout_) {
        TORCH_CHECK(false, "xddp cpu comm: collective timed out after ", timeout_.count(), " ms (rank ", rank_, ")");
      }
    }
  }

  // ---------------- worker ----------------
  std::shared_ptr<Work> enqueue(const char* name, const at::Tensor& meta, std::vector<at::Tensor> outs,
                                std::function<void()> fn) {
    TORCH_CHECK(!meta.defined() || meta.device().is_cpu(), "xddp cpu backend: tensors must live on the CPU");
    auto w = std::make_shared<CpuWork>();
    w->outputs = std::move(outs);
    w->collective = size_ > 1;
    w->timed = timing_.load();
    if (w->timed && w->collective) log_timed(w);
    w->seq = flight_.record(name, meta.defined() ? meta.numel() : 0, meta.defined() ? meta.scalar_type() : at::kByte);
    {
      std::lock_guard<std::mutex> g(qmu_);
      TORCH_CHECK(!stop_, "xddp cpu comm: communicator was shut down");
      if (error_) std::rethrow_exception(error_);
      q_.push_back([this, w, fn = std::move(fn)] {
        try {
          w->t0 = now_ns();
          fn();
          w->t1 = now_ns();
          flight_.finish(w->seq, "completed");
          w->finish(nullptr);
        } catch (...) {
          flight_.finish(w->seq, "failed");
          dump_flight("collective failed");
          w->finish(std::current_exception());
        }
      });
    }
    qcv_.notify_one();
    return w;
  }

  void run() {
    for (;;) {
      std::function<void()> job;
      {
        std::unique_lock<std::mutex> g(qmu_);
        qcv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        job = std::move(q_.front());
        q_.pop_front();
      }
      job();
    }
  }

  // ---------------- collectives ----------------
  static void reduce_into(at::Tensor dst, const at::Tensor& src, RedOp op) {
    switch (op) {
      case RedOp::SUM:
      case RedOp::AVG:
      case RedOp::PREMUL_SUM:
        if (dst.scalar_type() == at::kBool) dst.logical_or_(src); else dst.add_(src);
        break;
      case RedOp::PRODUCT:
        if (dst.scalar_type() == at::kBool) dst.logical_and_(src); else dst.mul_(src);
        break;
      case RedOp::MIN: at::minimum_out(dst, dst, src); break;
      case RedOp::MAX: at::maximum_out(dst, dst, src); break;
      case RedOp::BAND: dst.bitwise_and_(src); break;
      case RedOp::BOR: dst.bitwise_or_(src); break;
      case RedOp::BXOR: dst.bitwise_xor_(src); break;
    }
  }

  std::vector<int64_t> seg_bounds(int64_t n) const {
    std::vector<int64_t> b(size_ + 1, 0);
    for (int i = 0; i < size_; ++i) b[i + 1] = b[i] + n / size_ + (i < n % size_ ? 1 : 0);
    return b;
  }

  // ring reduce-scatter over `flat` (contiguous 1-D); afterwards segment `rank_` is reduced.
  void ring_reduce_scatter(at::Tensor flat, const std::vector<int64_t>& b, RedOp op) {
    const int right = (rank_ + 1) % size_, left = (rank_ - 1 + size_) % size_;
    const int64_t es = flat.element_size();
    int64_t maxseg = 0;
    for (int i = 0; i < size_; ++i) maxseg = std::max(maxseg, b[i + 1] - b[i]);
    auto tmp = at::empty({maxseg}, flat.options());
    char* base = static_cast<char*>(flat.data_ptr());
    for (int s = 0; s < size_ - 1; ++s) {
      const int ss = ((rank_ - s - 1) % size_ + size_) % size_;
      const int rs = ((rank_ - s - 2) % size_ + size_) % size_;
      const int64_t rn = b[rs + 1] - b[rs];
      exchange(peers_[right], base + b[ss] * es, (b[ss + 1] - b[ss]) * es, peers_[left], tmp.data_ptr(), rn * es);
      reduce_into(flat.narrow(0, b[rs], rn), tmp.narrow(0, 0, rn), op);
    }
  }

  // ring all-gather: rank r starts owning segment r.
  void ring_allgather(at::Tensor flat, const std::vector<int64_t>& b) {
    const int right = (rank_ + 1) % size_, left = (rank_ - 1 + size_) % size_;
    const int64_t es = flat.element_size();
    char* base = static_cast<char*>(flat.data_ptr());
    for (int s = 0; s < size_ - 1; ++s) {
      const int ss = ((rank_ - s) % size_ + size_) % size_;
      const int rs = ((rank_ - s - 1) % size_ + size_) % size_;
      exchange(peers_[right], base + b[ss] * es, (b[ss + 1] - b[ss]) * es, peers_[left], base + b[rs] * es,
               (b[rs + 1] - b[rs]) * es);
    }
  }

  void do_allreduce(at::Tensor t, RedOp op, double premul) {
    at::Tensor work = t.is_contiguous() ? t : t.contiguous();
    at::Tensor flat = work.view({-1});
    if (op == RedOp::PREMUL_SUM && premul != 1.0) flat.mul_(premul);
    if (size_ > 1 && flat.numel() > 0) {
      auto b = seg_bounds(flat.numel());
      ring_reduce_scatter(flat, b, op);
      ring_allgather(flat, b);
    }
    if (op == RedOp::AVG) {
      if (at::isFloatingType(flat.scalar_type())) flat.div_(size_);
      else flat.div_(size_, "trunc");
    }
    if (!work.is_same(t)) t.copy_(work);
  }

  void do_broadcast(at::Tensor t, int root) {
    if (size_ == 1) return;
    at::Tensor work = t.is_contiguous() ? t : t.contiguous();
    const int64_t nb = work.nbytes();
    char* p = static_cast<char*>(work.data_ptr());
    // chain: root -> root+1 -> ... pipelined in 4 MiB chunks
    const int pos = (rank_ - root + size_) % size_;
    const int right = (rank_ + 1) % size_, left = (rank_ - 1 + size_) % size_;
    const int64_t chunk = 4 << 20;
    for (int64_t off = 0; off < nb; off += chunk) {
      const int64_t n = std::min(chunk, nb - off);
      if (pos != 0) recv_all(peers_[left], p + off, n);
      if (pos != size_ - 1) send_all(peers_[right], p + off, n);
    }
    if (!work.is_same(t)) t.copy_(work);
  }

  void do_allgather(at::Tensor out, at::Tensor in) {
    at::Tensor o = out.is_contiguous() ? out : at::empty_like(out, at::MemoryFormat::Contiguous);
    auto flat = o.view({-1});
    const int64_t n = in.numel();
    flat.narrow(0, rank_ * n, n).copy_(in.reshape({-1}));
    if (size_ > 1 && n > 0) {
      std::vector<int64_t> b(size_ + 1);
      for (int i = 0; i <= size_; ++i) b[i] = i * n;
      ring_allgather(flat, b);
    }
    if (!o.is_same(out)) out.copy_(o);
  }

  void do_reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) {
    auto flat = in.reshape({-1}).clone();
    const int64_t n = out.numel();
    std::vector<int64_t> b(size_ + 1);
    for (int i = 0; i <= size_; ++i) b[i] = i * n;
    if (size_ > 1 && n > 0) ring_reduce_scatter(flat, b, op);
    auto mine = flat.narrow(0, rank_ * n, n);
    if (op == RedOp::AVG) {
      if (at::isFloatingType(mine.scalar_type())) mine.div_(size_); else mine.div_(size_, "trunc");
    }
    out.copy_(mine.view(out.sizes()));
  }

  void do_alltoall(at::Tensor out, at::Tensor in) {
    auto src = in.reshape({-1}).contiguous();
    at::Tensor o = out.is_contiguous() ? out : at::empty_like(out, at::MemoryFormat::Contiguous);
    auto dst = o.view({-1});
    const int64_t n = src.numel() / size_;
    const int64_t es = src.element_size();
    dst.narrow(0, rank_ * n, n).copy_(src.narrow(0, rank_ * n, n));
    char* sp = static_cast<char*>(src.data_ptr());
    char* dp = static_cast<char*>(dst.data_ptr());
    for (int k = 1; k < size_; ++k) {
      const int to = (rank_ + k) % size_, from = (rank_ - k + size_) % size_;
      exchange(peers_[to], sp + to * n * es, n * es, peers_[from], dp + from * n * es, n * es);
    }
    if (!o.is_same(out)) out.copy_(o);
  }

  std::shared_ptr<Store> store_;
  std::chrono::milliseconds timeout_;
  std::vector<int> peers_;
  std::thread worker_;
  std::mutex qmu_;
  std::condition_variable qcv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false;
  std::exception_ptr error_;
};

std::shared_ptr<Comm> make_tcp_comm_host(std::shared_ptr<Store> store, int rank, int size,
                                         std::chrono::milliseconds timeout, const std::string& host) {
  return std::make_shared<TcpComm>(std::move(store), rank, size, timeout, host);
}

std::shared_ptr<Comm> make_tcp_comm(std::shared_ptr<Store> store, int rank, int size,
                                    std::chrono::milliseconds timeout) {
  return make_tcp_comm_host(std::move(store), rank, size, timeout, "127.0.0.1");
}

}  // namespace xddp
