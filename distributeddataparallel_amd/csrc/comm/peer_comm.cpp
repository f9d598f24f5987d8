// PeerComm: an RCCL-free single-node communicator for device tensors, built on the peer-memory
// kernels of peer_allreduce.hip (IPC-mapped staging buffers, xGMI loads). Backend "peer" of
// init_process_group.
//
// Every collective runs on one dedicated HIP stream that first waits for the caller's stream
// (event), so it is ordered after the producer of its input; Work.wait() makes the caller's stream
// wait for the collective's completion event (no host blocking). All-reduce takes the two-shot
// kernel (reduce-scatter + all-gather over all links) from XDDP_PEER_TWO_SHOT_MIN_BYTES (default
// 256 KiB) up and the one-shot kernel below; messages larger than a lane's staging capacity are
// walked in capacity-sized chunks. Broadcast, all-gather, reduce-scatter (all-reduce + own slice)
// and barrier are supported; all-to-all and point-to-point are not (use the RCCL backend).
//
// Failure handling: a watchdog thread polls the in-flight completion events (flight records are
// marked completed only when their event has fired) and the peer kernels' host-mapped status word.
// A peer that never arrived (XDDP_PEER_TIMEOUT_MS, default = the process-group timeout) puts the
// communicator in an error state: the flight record is dumped, the error is posted to the store so
// the other ranks fail too, and every later Work query / launch raises.
//
// Why it exists: on a 1-GPU box several ranks can share the device through it (RCCL refuses
// duplicate devices), so the W > 1 DDP path — bucket launches, stream ordering, Work semantics —
// runs against device-side collectives, not the host-staged CPU backend; on a node it is the same
// peer-memory protocol the RCCL communicator can route messages to (XDDP_PEER_ALLREDUCE).
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <iostream>
#include <list>
#include <memory>
#include <thread>

#include "comm/comm.h"
#include "comm/peer.h"

namespace xddp {

namespace {

// Shared error state of one communicator: 0 ok, 1 peer timeout, 3 a peer rank reported an error.
struct PeerState {
  std::atomic<int> err{0};
  std::shared_ptr<PeerAllReduce> peer;  // shared: a Work may outlive its communicator
  void check() {
    int e = err.load();
    if (e == 0 && peer && peer->status() != 0) {
      e = 1;
      err.store(1);
    }
    TORCH_CHECK(e == 0, "xddp peer: communicator is in error state (",
                e == 1 ? "a peer rank did not arrive within XDDP_PEER_TIMEOUT_MS; the collective's output is invalid"
                       : "a peer rank reported a communicator error",
                "); re-create the process group");
  }
};

class PeerWork : public Work {
 public:
  PeerWork(int device, hipEvent_t ev, hipEvent_t t0, hipEvent_t t1, std::shared_ptr<PeerState> st)
      : device_(device), ev_(ev), t0_(t0), t1_(t1), st_(std::move(st)) {}
  ~PeerWork() override {
    for (auto e : {ev_, t0_, t1_})
      if (e) (void)hipEventDestroy(e);
  }
  bool is_completed() override {
    st_->check();
    const bool done = hipEventQuery(ev_) == hipSuccess;
    if (done) st_->check();
    return done;
  }
  void wait() override {
    st_->check();
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    XDDP_HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(device_).stream(), ev_, 0));
  }
  void synchronize() override {
    st_->check();
    XDDP_HIP_CHECK(hipEventSynchronize(ev_));
    st_->check();
  }
  Timing timing_state() override {
    if (!t0_) return Timing::kNone;
    return hipEventQuery(t1_) == hipSuccess ? Timing::kReady : Timing::kPending;
  }
  double comm_ms() override {
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, t0_, t1_);
    return ms;
  }
  double comm_ms_before(const TimeRef& ref) override {
    if (!ref.ev) return 0.0;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, t0_, ref.ev) != hipSuccess) return 0.0;
    return std::max(0.0, std::min<double>(ms, comm_ms()));
  }
  hipEvent_t event() const { return ev_; }

 private:
  int device_;
  hipEvent_t ev_, t0_, t1_;
  std::shared_ptr<PeerState> st_;
};

class PeerComm : public Comm {
 public:
  PeerComm(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity, int64_t two_shot_capacity,
           std::chrono::milliseconds timeout)
      : Comm(rank, size),
        store_(store),
        device_(device),
        stream_(c10::hip::getStreamFromPool(true, static_cast<c10::DeviceIndex>(device))),
        peer_(std::make_shared<PeerAllReduce>(std::move(store), rank, size, device, capacity, two_shot_capacity,
                                              timeout)),
        st_(std::make_shared<PeerState>()) {
    st_->peer = peer_;
    const char* m = std::getenv("XDDP_PEER_TWO_SHOT_MIN_BYTES");
    two_shot_min_ = m ? std::atoll(m) : (256 << 10);
    watchdog_ = std::thread([this] { watchdog_loop(); });
  }
  ~PeerComm() override { stop_watchdog(); }

  std::string backend() const override { return "peer"; }
  std::map<std::string, std::string> info() const override {
    return {{"backend", "peer"},
            {"one_shot_capacity_bytes", std::to_string(peer_->capacity())},
            {"two_shot_capacity_bytes", std::to_string(peer_->two_shot_capacity())},
            {"two_shot_min_bytes", std::to_string(two_shot_min_)},
            {"timeout_ms", std::to_string(peer_->timeout_ms())}};
  }

  std::shared_ptr<Work> allreduce(at::Tensor t, RedOp op, double premul) override {
    TORCH_CHECK(op == RedOp::SUM || op == RedOp::AVG || op == RedOp::MAX || op == RedOp::PREMUL_SUM,
                "peer backend: all-reduce supports SUM, AVG, MAX and PREMUL_SUM");
    const RedOp kop = op == RedOp::PREMUL_SUM ? RedOp::SUM : op;
    const bool two = use_two_shot(t, kop);
    return launch(two ? "allreduce_two_shot" : "allreduce", t, {t}, [&](hipStream_t s) {
      if (two) {
        peer_->allreduce_two_shot(t, kop, s);
      } else {
        for_chunks(t, [&](at::Tensor c) { peer_->allreduce(c, kop, s); });
      }
      if (op == RedOp::PREMUL_SUM) t.mul_(premul);  // (on the comm stream: the guard below)
    });
  }

  // Routes: base / one-shot = one-shot chunks, two-shot = the two-shot lane. The route table
  // (calibration) replaces the XDDP_PEER_TWO_SHOT_MIN_BYTES threshold; dropping the two-shot lane
  // after a failed self-check (finish_peer_probation(false)) leaves the one-shot chunks.
  std::shared_ptr<Work> allreduce_via(at::Tensor t, RedOp op, int route) override {
    if (route == kRouteAuto) return allreduce(t, op, 1.0);
    TORCH_CHECK(op == RedOp::SUM || op == RedOp::AVG || op == RedOp::MAX, "peer backend: allreduce_via op");
    const bool two = route == kRouteTwoShot;
    TORCH_CHECK(!two || (two_shot_ok_ && peer_->supports_two_shot(t, op)), "peer backend: two-shot route unavailable");
    return launch(two ? "allreduce_two_shot" : "allreduce", t, {t}, [&](hipStream_t s) {
      if (two) peer_->allreduce_two_shot(t, op, s);
      else for_chunks(t, [&](at::Tensor c) { peer_->allreduce(c, op, s); });
    });
  }
  std::vector<int> routes() const override {
    if (two_shot_ok_ && peer_->two_shot_capacity() > 0) return {kRouteOneShot, kRouteTwoShot};
    return {kRouteOneShot};
  }
  int64_t one_shot_capacity() const override { return peer_->capacity(); }
  void set_route_table(const std::vector<int64_t>& bounds, const std::vector<int>& routes) override {
    TORCH_CHECK(bounds.size() == routes.size(), "route table: bounds and routes differ in length");
    route_bounds_ = bounds;
    route_ids_ = routes;
  }
  std::vector<std::vector<int64_t>> route_table() const override {
    return {route_bounds_, std::vector<int64_t>(route_ids_.begin(), route_ids_.end())};
  }
  int peer_status() const override { return peer_->status(); }
  void set_peer_timeout_ms(double ms) override { peer_->set_timeout_ms(ms); }
  void finish_peer_probation(bool keep) override {
    if (keep) return;
    two_shot_ok_ = false;
    route_bounds_.clear();
    route_ids_.clear();
  }

  std::shared_ptr<Work> broadcast(at::Tensor t, int root) override {
    return launch("broadcast", t, {t}, [&](hipStream_t s) {
      for_chunks(t, [&](at::Tensor c) { peer_->broadcast(c, root, s); });
    });
  }

  std::shared_ptr<Work> allgather(at::Tensor out, at::Tensor in) override {
    TORCH_CHECK(out.numel() == in.numel() * size_ && out.scalar_type() == in.scalar_type() && out.is_contiguous() &&
                    in.is_contiguous(),
                "peer backend: all-gather needs contiguous out of size * in.numel() elements");
    return launch("allgather", in, {out, in}, [&](hipStream_t s) {
      const int64_t n = in.numel();
      const int64_t step = chunk_elems(in);
      auto o2 = out.view({size_, n});
      for (int64_t off = 0; off < n; off += step) {
        const int64_t len = std::min(step, n - off);
        auto src = in.view(-1).narrow(0, off, len);
        if (off == 0 && len == n) {
          peer_->allgather(out.view(-1), src, s);
        } else {  // chunk: gather into a staging tensor, then scatter the rows
          auto tmp = at::empty({size_ * len}, in.options());
          peer_->allgather(tmp, src, s);
          o2.narrow(1, off, len).copy_(tmp.view({size_, len}));
        }
      }
    });
  }

  std::shared_ptr<Work> reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) override {
    TORCH_CHECK(in.numel() == out.numel() * size_, "reduce_scatter: input must hold size*output elements");
    TORCH_CHECK(op == RedOp::SUM || op == RedOp::AVG || op == RedOp::MAX, "peer backend: reduce_scatter op");
    auto tmp = in.contiguous().clone();  // (on the caller's stream: the launch orders after it)
    return launch("reduce_scatter", in, {out, tmp}, [&](hipStream_t s) {
      for_chunks(tmp, [&](at::Tensor c) { peer_->allreduce(c, op, s); });
      out.view(-1).copy_(tmp.view(-1).narrow(0, (int64_t)rank_ * out.numel(), out.numel()));
    });
  }

  std::shared_ptr<Work> alltoall(at::Tensor, at::Tensor) override {
    TORCH_CHECK(false, "peer backend: all_to_all is not supported (use the rccl backend)");
  }
  std::shared_ptr<Work> send(at::Tensor, int) override {
    TORCH_CHECK(false, "peer backend: send/recv are not supported (use the rccl backend)");
  }
  std::shared_ptr<Work> recv(at::Tensor, int) override {
    TORCH_CHECK(false, "peer backend: send/recv are not supported (use the rccl backend)");
  }

  std::shared_ptr<Work> barrier() override {
    if (!barrier_buf_.defined())
      barrier_buf_ = at::zeros({4}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, device_));
    auto w = allreduce(barrier_buf_, RedOp::SUM, 1.0);
    w->synchronize();
    return w;
  }

  void shutdown() override {
    stop_watchdog();
    {
      c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
      (void)hipStreamSynchronize(stream_.stream());
    }
    peer_quiesce(store_, rank_, size_, std::chrono::seconds(10));
    peer_->close();
  }

 private:
  bool use_two_shot(const at::Tensor& t, RedOp op) const {
    if (!two_shot_ok_ || !peer_->supports_two_shot(t, op)) return false;
    const int64_t nb = static_cast<int64_t>(t.nbytes());
    if (route_bounds_.empty()) return nb >= two_shot_min_;
    for (size_t i = 0; i < route_bounds_.size(); ++i)
      if (nb <= route_bounds_[i]) return route_ids_[i] == kRouteTwoShot;
    return false;
  }

  int64_t chunk_elems(const at::Tensor& t) const {
    const int64_t esz = t.element_size();
    return std::max<int64_t>(16 / esz, (peer_->capacity() / esz) / (16 / esz) * (16 / esz));
  }

  template <typename F>
  void for_chunks(const at::Tensor& t, F&& f) {
    TORCH_CHECK(t.is_cuda() && t.is_contiguous() && t.device().index() == device_,
                "peer backend: contiguous tensors on this rank's device only");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, "peer backend: 16-B aligned tensors only");
    const int64_t n = t.numel(), step = chunk_elems(t);
    auto flat = t.view(-1);
    for (int64_t off = 0; off < n; off += step) f(flat.narrow(0, off, std::min(step, n - off)));
  }

  static hipEvent_t make_event(bool timed) {
    hipEvent_t e;
    XDDP_HIP_CHECK(hipEventCreateWithFlags(&e, timed ? hipEventDefault : hipEventDisableTiming));
    return e;
  }

  template <typename F>
  std::shared_ptr<Work> launch(const char* name, const at::Tensor& meta, std::vector<at::Tensor> keep, F&& body) {
    st_->check();
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    auto cur = c10::hip::getCurrentHIPStream(device_);
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    XDDP_HIP_CHECK(hipStreamIsCapturing(cur.stream(), &cap));
    const bool capturing = cap == hipStreamCaptureStatusActive;
    hipEvent_t pre = make_event(false);
    XDDP_HIP_CHECK(hipEventRecord(pre, cur.stream()));
    XDDP_HIP_CHECK(hipStreamWaitEvent(stream_.stream(), pre, 0));
    XDDP_HIP_CHECK(hipEventDestroy(pre));
    const int64_t seq = flight_.record(name, meta.numel(), meta.scalar_type());
    const bool timed = timing_.load() && !capturing;
    hipEvent_t t0 = timed ? make_event(true) : nullptr, t1 = timed ? make_event(true) : nullptr;
    if (t0) XDDP_HIP_CHECK(hipEventRecord(t0, stream_.stream()));
    {
      c10::hip::HIPStreamGuard sg(stream_);  // torch ops in the body (chunk copies, scaling) too
      body(stream_.stream());
    }
    if (t1) XDDP_HIP_CHECK(hipEventRecord(t1, stream_.stream()));
    if (!capturing) {
      for (auto& t : keep)
        if (t.defined() && t.is_cuda()) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_);
    }
    hipEvent_t done = make_event(false);
    XDDP_HIP_CHECK(hipEventRecord(done, stream_.stream()));
    auto w = std::make_shared<PeerWork>(device_, done, t0, t1, st_);
    w->outputs = std::move(keep);
    w->seq = seq;
    w->collective = size_ > 1;
    if (timed && w->collective) log_timed(w);
    if (capturing) {
      flight_.finish(seq, "captured");  // a graph node, not a live collective
    } else {
      std::lock_guard<std::mutex> g(wd_mu_);
      inflight_.push_back(w);
    }
    return w;
  }

  void watchdog_loop() {
    int64_t last_store_poll = 0;
    while (!wd_stop_) {
      std::vector<std::shared_ptr<PeerWork>> done;
      {
        std::unique_lock<std::mutex> g(wd_mu_);
        wd_cv_.wait_for(g, std::chrono::milliseconds(50), [&] { return wd_stop_.load(); });
        if (wd_stop_) break;
        for (auto it = inflight_.begin(); it != inflight_.end();) {
          if (hipEventQuery((*it)->event()) == hipSuccess) {
            done.push_back(*it);
            it = inflight_.erase(it);
          } else {
            ++it;
          }
        }
      }
      const bool timed_out = peer_->status() != 0;
      for (auto& w : done) flight_.finish(w->seq, timed_out ? "failed" : "completed");
      if (timed_out && !reported_) {  // (a Work query may have set the error state first)
        reported_ = true;
        int z = 0;
        st_->err.compare_exchange_strong(z, 1);
        const std::string reason = "a peer did not arrive within " + std::to_string((int64_t)peer_->timeout_ms()) +
                                   " ms (XDDP_PEER_TIMEOUT_MS)";
        std::cerr << "[xddp rank " << rank_ << "] peer watchdog: " << reason << "; communicator is in error state\n";
        {
          std::lock_guard<std::mutex> g(wd_mu_);
          for (auto& w : inflight_) flight_.finish(w->seq, "failed");
        }
        dump_flight(reason);
        try {
          store_->set("peer/error", "rank " + std::to_string(rank_) + ": " + reason);
        } catch (...) {
        }
      }
      // a collective in flight for over a second: has a peer already failed?
      const int64_t now = now_ns();
      bool busy;
      {
        std::lock_guard<std::mutex> g(wd_mu_);
        busy = !inflight_.empty();
      }
      if (st_->err.load() == 0 && busy && now - last_store_poll > 1000000000LL) {
        last_store_poll = now;
        try {
          if (store_->check({"peer/error"})) {
            std::cerr << "[xddp rank " << rank_ << "] peer watchdog: " << store_->get("peer/error") << "\n";
            st_->err.store(3);
            dump_flight("peer error: " + store_->get("peer/error"));
          }
        } catch (...) {
        }
      }
    }
  }

  void stop_watchdog() {
    wd_stop_ = true;
    wd_cv_.notify_all();
    if (watchdog_.joinable()) watchdog_.join();
  }

  std::shared_ptr<Store> store_;
  int device_;
  c10::hip::HIPStream stream_;
  std::shared_ptr<PeerAllReduce> peer_;
  std::shared_ptr<PeerState> st_;
  int64_t two_shot_min_ = 0;
  bool two_shot_ok_ = true;
  std::vector<int64_t> route_bounds_;
  std::vector<int> route_ids_;
  at::Tensor barrier_buf_;
  std::thread watchdog_;
  std::atomic<bool> wd_stop_{false};
  bool reported_ = false;  // watchdog thread only
  std::mutex wd_mu_;
  std::condition_variable wd_cv_;
  std::list<std::shared_ptr<PeerWork>> inflight_;
};

}  // namespace

std::shared_ptr<Comm> make_peer_comm(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity,
                                     int64_t two_shot_capacity, std::chrono::milliseconds timeout) {
  return std::make_shared<PeerComm>(std::move(store), rank, size, device, capacity, two_shot_capacity, timeout);
}

}  // namespace xddp
