// RCCL communicator over xGMI.
//
// Design (MI355X-first, not a ProcessGroupNCCL translation):
//  * one communicator per process/GPU, created eagerly at init (no lazy first-collective
//    stall inside the DDP constructor), unique id exchanged through the xddp store;
//  * all collectives go on ONE dedicated high-priority HIP stream obtained from torch's
//    stream pool, so backward kernels keep the CUs and the caching allocator knows the
//    stream (recordStream on every buffer handed to RCCL);
//  * Work completion = a timing-free hipEvent recorded after the RCCL call; wait() makes the
//    caller's current stream wait on it (no host block);
//  * ncclGroupStart/End coalescing for bucket bursts;
//  * a watchdog thread polls in-flight events + ncclCommGetAsyncError and aborts the
//    communicator on timeout/error so a hung peer surfaces as an exception, not a hang;
//    on error it dumps the flight record and posts the error to the store, and while a
//    collective is overdue (>1 s) it polls the store for errors posted by peers, so every
//    rank fails fast instead of each waiting out its own timeout;
//  * a heartbeat monitor thread aborts the process (after a flight dump) if the watchdog
//    itself stops ticking, e.g. stuck inside a driver call (XDDP_HEARTBEAT_TIMEOUT_SEC).
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <iostream>
#include <list>
#include <thread>

#include "comm/comm.h"
#include "comm/peer.h"

#define XDDP_NCCL_CHECK(expr)                                                                  \
  do {                                                                                         \
    ncclResult_t _r = (expr);                                                                  \
    TORCH_CHECK(_r == ncclSuccess, "RCCL error: ", ncclGetErrorString(_r), " (" #expr ")");    \
  } while (0)

namespace xddp {

namespace {

ncclDataType_t to_nccl(at::ScalarType t) {
  switch (t) {
    case at::kFloat: return ncclFloat32;
    case at::kHalf: return ncclFloat16;
    case at::kBFloat16: return ncclBfloat16;
    case at::kDouble: return ncclFloat64;
    case at::kInt: return ncclInt32;
    case at::kLong: return ncclInt64;
    case at::kByte: return ncclUint8;
    case at::kChar: return ncclInt8;
    case at::kBool: return ncclUint8;
    case at::kFloat8_e4m3fn: return ncclFloat8e4m3;
    case at::kFloat8_e5m2: return ncclFloat8e5m2;
    default: TORCH_CHECK(false, "xddp rccl: unsupported dtype ", t);
  }
}

ncclRedOp_t to_nccl(RedOp op, at::ScalarType t) {
  if (t == at::kBool) {
    if (op == RedOp::SUM || op == RedOp::MAX || op == RedOp::BOR) return ncclMax;
    if (op == RedOp::PRODUCT || op == RedOp::MIN || op == RedOp::BAND) return ncclMin;
  }
  switch (op) {
    case RedOp::SUM: return ncclSum;
    case RedOp::AVG: return ncclAvg;
    case RedOp::PRODUCT: return ncclProd;
    case RedOp::MIN: return ncclMin;
    case RedOp::MAX: return ncclMax;
    default: TORCH_CHECK(false, "xddp rccl: unsupported reduce op ", static_cast<int>(op));
  }
}

class EventPool {
 public:
  explicit EventPool(bool timing = false) : timing_(timing) {}
  hipEvent_t get() {
    std::lock_guard<std::mutex> g(mu_);
    if (!free_.empty()) {
      auto e = free_.back();
      free_.pop_back();
      return e;
    }
    hipEvent_t e;
    XDDP_HIP_CHECK(hipEventCreateWithFlags(&e, timing_ ? hipEventDefault : hipEventDisableTiming));
    return e;
  }
  void put(hipEvent_t e) {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(e);
  }

 private:
  bool timing_;
  std::mutex mu_;
  std::vector<hipEvent_t> free_;
};

// Comm-stream interval of one (or one group of) RCCL launches, shared by the works it covers.
struct Interval {
  Interval(std::shared_ptr<EventPool> p) : pool(std::move(p)), t0(pool->get()), t1(pool->get()) {}
  ~Interval() {
    pool->put(t0);
    pool->put(t1);
  }
  std::shared_ptr<EventPool> pool;
  hipEvent_t t0, t1;
};

}  // namespace

class RcclComm;

class RcclWork : public Work {
 public:
  RcclWork(std::shared_ptr<EventPool> pool, int device, std::shared_ptr<std::atomic<int>> err,
           std::shared_ptr<PeerAllReduce> peer)
      : pool_(std::move(pool)), device_(device), err_(std::move(err)), peer_(std::move(peer)) {
    ev = pool_->get();
    t_start = now_ns();
  }
  ~RcclWork() override { pool_->put(ev); }
  bool is_completed() override {
    check_error();
    if (captured) return true;
    if (!launched) return false;  // still inside an open group: nothing enqueued yet
    const bool done = hipEventQuery(ev) == hipSuccess;
    if (done) check_error();
    return done;
  }
  void wait() override {
    check_error();
    check_launched("wait");
    auto cur = c10::hip::getCurrentHIPStream(device_);
    XDDP_HIP_CHECK(hipStreamWaitEvent(cur.stream(), ev, 0));
  }
  void synchronize() override {
    check_error();
    if (captured) return;  // host sync inside a capture is illegal; replay ordering is by stream
    check_launched("synchronize");
    XDDP_HIP_CHECK(hipEventSynchronize(ev));
    check_error();
  }
  void check_error() {
    int e = err_->load();
    if (e == 0 && peer_ && peer_->status() != 0) {  // host-mapped word: no device sync
      int z = 0;
      err_->compare_exchange_strong(z, 4);
      e = err_->load();
    }
    TORCH_CHECK(e == 0, "xddp rccl: communicator is in error state (",
                e == 1   ? "collective timed out; watchdog aborted the communicator"
                : e == 3 ? "a peer rank reported a communicator error"
                : e == 4 ? "a peer-memory collective timed out (a rank did not arrive within XDDP_PEER_TIMEOUT_MS); "
                           "its output is invalid"
                         : "asynchronous RCCL error",
                ")");
  }
  Timing timing_state() override {
    if (!iv) return Timing::kNone;
    return hipEventQuery(iv->t1) == hipSuccess ? Timing::kReady : Timing::kPending;
  }
  double comm_ms() override {
    if (!iv || !owns_interval) return 0.0;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, iv->t0, iv->t1);
    return ms;
  }
  double comm_ms_before(const TimeRef& ref) override {
    if (!iv || !owns_interval || !ref.ev) return 0.0;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, iv->t0, ref.ev) != hipSuccess) return 0.0;
    return std::max(0.0, std::min<double>(ms, comm_ms()));
  }
  // A work issued inside an open ncclGroupStart has no kernels and no recorded event until the
  // group ends: its event (a pooled one, possibly recorded for an earlier collective) says nothing
  // about it, so waiting on it before group_end is an error rather than a silent no-op.
  void check_launched(const char* what) const {
    TORCH_CHECK(launched.load(), "xddp rccl: ", what, "() on a collective issued inside an open group; ",
                "the collective is launched at group_end() (close the coalescing block first)");
  }
  hipEvent_t ev;
  int64_t t_start;
  std::atomic<bool> launched{false};
  bool captured = false;
  std::shared_ptr<Interval> iv;  // timed works only
  bool owns_interval = true;     // false for the 2nd.. works of a grouped launch

 private:
  std::shared_ptr<EventPool> pool_;
  int device_;
  std::shared_ptr<std::atomic<int>> err_;
  std::shared_ptr<PeerAllReduce> peer_;
};

class RcclComm : public Comm {
 public:
  RcclComm(std::shared_ptr<Store> store, int rank, int size, int device, std::chrono::milliseconds timeout,
           bool high_priority)
      : Comm(rank, size),
        store_(store),
        device_(device),
        timeout_(timeout),
        stream_(c10::hip::getStreamFromPool(high_priority, static_cast<c10::DeviceIndex>(device))),
        pool_(std::make_shared<EventPool>()),
        tpool_(std::make_shared<EventPool>(true)),
        err_(std::make_shared<std::atomic<int>>(0)) {
    high_priority_ = high_priority;
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device));
    ncclUniqueId id;
    if (rank == 0) {
      XDDP_NCCL_CHECK(ncclGetUniqueId(&id));
      store->set("rccl/uid", std::string(reinterpret_cast<const char*>(&id), sizeof(id)));
    } else {
      std::string s = store->get("rccl/uid");
      TORCH_CHECK(s.size() == sizeof(id), "xddp rccl: bad unique id size");
      std::memcpy(&id, s.data(), sizeof(id));
    }
    XDDP_NCCL_CHECK(ncclCommInitRank(&comm_, size, id, rank));
    // XDDP_RCCL_FORCE_LAUNCH=1: issue real RCCL kernels even on one rank, so the multi-rank
    // launch path (comm-stream ordering, events, allocator stream records) runs on a 1-GPU box
    const char* fl = std::getenv("XDDP_RCCL_FORCE_LAUNCH");
    force_launch_ = fl && std::string(fl) == "1";
    init_peer(store);
    heartbeat_ = now_ns();
    watchdog_ = std::thread([this] { watchdog_loop(); });
    const char* hb = std::getenv("XDDP_HEARTBEAT_TIMEOUT_SEC");
    hb_timeout_s_ = hb ? std::atof(hb) : 480.0;
    if (hb_timeout_s_ > 0) monitor_ = std::thread([this] { monitor_loop(); });
  }

  ~RcclComm() override {
    stop_watchdog();
    // Deliberately no ncclCommDestroy here: at interpreter exit the HIP runtime may already
    // be torn down. destroy_process_group() calls shutdown() explicitly.
  }

  std::string backend() const override { return "rccl"; }

  std::shared_ptr<Work> allreduce(at::Tensor t, RedOp op, double premul) override {
    check_tensor(t);
    if (size_ == 1 && !force_launch_ && op != RedOp::PREMUL_SUM) return local_noop("allreduce", t);  // identity
    switch (peer_route(t, op, false)) {
      case PeerRoute::kOneShot:
        return launch_peer("allreduce_peer", t, {t}, [&](hipStream_t s) { peer_->allreduce(t, op, s); });
      case PeerRoute::kTwoShot:
        return launch_peer("allreduce_two_shot", t, {t}, [&](hipStream_t s) { peer_->allreduce_two_shot(t, op, s); });
      default: break;
    }
    return launch("allreduce", t, {t}, [&](hipStream_t s) {
      if (op == RedOp::PREMUL_SUM) {
        TORCH_CHECK(at::isFloatingType(t.scalar_type()), "PREMUL_SUM needs a floating-point tensor");
        // the host-immediate scalar must be in the tensor's dtype
        ncclRedOp_t rop;
        double d = premul;
        float f = static_cast<float>(premul);
        uint16_t half_bits = t.scalar_type() == at::kHalf ? at::Half(f).x : at::BFloat16(f).x;
        void* sp = t.scalar_type() == at::kDouble  ? static_cast<void*>(&d)
                   : t.scalar_type() == at::kFloat ? static_cast<void*>(&f)
                                                   : static_cast<void*>(&half_bits);
        XDDP_NCCL_CHECK(ncclRedOpCreatePreMulSum(&rop, sp, to_nccl(t.scalar_type()), ncclScalarHostImmediate, comm_));
        XDDP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), rop, comm_, s));
        XDDP_NCCL_CHECK(ncclRedOpDestroy(rop, comm_));
      } else {
        XDDP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()),
                                      to_nccl(op, t.scalar_type()), comm_, s));
      }
    });
  }

  std::shared_ptr<Work> allreduce_via(at::Tensor t, RedOp op, int route) override {
    check_tensor(t);
    if (route == kRouteAuto) return allreduce(t, op, 1.0);
    if (size_ == 1 && !force_launch_) return local_noop("allreduce", t);
    auto pr = std::atomic_load(&peer_);
    if (route == kRouteOneShot) {
      TORCH_CHECK(pr && pr->supports(t, op, false), "xddp rccl: one-shot route unavailable for this tensor");
      return launch_peer("allreduce_peer", t, {t}, [&](hipStream_t s) { pr->allreduce(t, op, s); });
    }
    if (route == kRouteTwoShot) {
      TORCH_CHECK(pr && pr->supports_two_shot(t, op), "xddp rccl: two-shot route unavailable for this tensor");
      return launch_peer("allreduce_two_shot", t, {t}, [&](hipStream_t s) { pr->allreduce_two_shot(t, op, s); });
    }
    TORCH_CHECK(op != RedOp::PREMUL_SUM, "allreduce_via: PREMUL_SUM takes the auto route");
    return launch("allreduce", t, {t}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclAllReduce(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()),
                                    to_nccl(op, t.scalar_type()), comm_, s));
    });
  }

  std::vector<int> routes() const override {
    auto pr = std::atomic_load(&peer_);
    if (!pr) return {};
    std::vector<int> r{kRouteOneShot};
    if (pr->two_shot_capacity() > 0) r.push_back(kRouteTwoShot);
    return r;
  }
  int64_t one_shot_capacity() const override {
    auto pr = std::atomic_load(&peer_);
    return pr ? pr->capacity() : 0;
  }
  void set_route_table(const std::vector<int64_t>& bounds, const std::vector<int>& routes) override {
    TORCH_CHECK(bounds.size() == routes.size(), "route table: bounds and routes differ in length");
    route_bounds_ = bounds;
    route_ids_ = routes;
  }
  std::vector<std::vector<int64_t>> route_table() const override {
    return {route_bounds_, std::vector<int64_t>(route_ids_.begin(), route_ids_.end())};
  }
  int peer_status() const override {
    auto pr = std::atomic_load(&peer_);
    return pr ? pr->status() : 0;
  }
  void set_peer_timeout_ms(double ms) override {
    if (auto pr = std::atomic_load(&peer_)) pr->set_timeout_ms(ms);
  }
  void finish_peer_probation(bool keep) override {
    auto pr = std::atomic_load(&peer_);
    if (!pr) return;
    if (keep && pr->status() == 0) {
      probation_ = false;
      return;
    }
    // every launched peer kernel drains (its grid always exits, also after a timeout); then the
    // lanes go away and every collective takes the RCCL ring
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    XDDP_HIP_CHECK(hipStreamSynchronize(stream_.stream()));
    route_bounds_.clear();
    route_ids_.clear();
    peer_mode_ = 0;
    std::atomic_store(&peer_, std::shared_ptr<PeerAllReduce>());
    pr->close();
    probation_ = false;
  }

  std::shared_ptr<Work> broadcast(at::Tensor t, int root) override {
    check_tensor(t);
    if (size_ == 1 && !force_launch_) return local_noop("broadcast", t);
    if (peer_route(t, RedOp::SUM, true) == PeerRoute::kOneShot)
      return launch_peer("broadcast_peer", t, {t}, [&](hipStream_t s) { peer_->broadcast(t, root, s); });
    return launch("broadcast", t, {t}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclBroadcast(t.data_ptr(), t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), root, comm_, s));
    });
  }

  std::shared_ptr<Work> allgather(at::Tensor out, at::Tensor in) override {
    check_contig(out);
    check_contig(in);
    TORCH_CHECK(out.numel() == in.numel() * size_, "allgather: output must hold size*input elements");
    return launch("allgather", in, {out, in}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclAllGather(in.data_ptr(), out.data_ptr(), in.numel(), to_nccl(in.scalar_type()), comm_, s));
    });
  }

  std::shared_ptr<Work> reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) override {
    check_contig(out);
    check_contig(in);
    TORCH_CHECK(in.numel() == out.numel() * size_, "reduce_scatter: input must hold size*output elements");
    return launch("reduce_scatter", in, {out, in}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclReduceScatter(in.data_ptr(), out.data_ptr(), out.numel(), to_nccl(in.scalar_type()),
                                        to_nccl(op, in.scalar_type()), comm_, s));
    });
  }

  std::shared_ptr<Work> alltoall(at::Tensor out, at::Tensor in) override {
    check_contig(out);
    check_contig(in);
    TORCH_CHECK(in.numel() == out.numel() && in.numel() % size_ == 0, "alltoall: equal splits required");
    return launch("alltoall", in, {out, in}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclAllToAll(in.data_ptr(), out.data_ptr(), in.numel() / size_, to_nccl(in.scalar_type()),
                                   comm_, s));
    });
  }

  std::shared_ptr<Work> send(at::Tensor t, int dst) override {
    check_contig(t);
    return launch("send", t, {t}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclSend(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), dst, comm_, s));
    });
  }

  std::shared_ptr<Work> recv(at::Tensor t, int src) override {
    check_contig(t);
    return launch("recv", t, {t}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclRecv(t.data_ptr(), t.numel(), to_nccl(t.scalar_type()), src, comm_, s));
    });
  }

  std::shared_ptr<Work> barrier() override {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    if (!barrier_buf_.defined())
      barrier_buf_ = at::zeros({1}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA, device_));
    auto w = launch("barrier", barrier_buf_, {barrier_buf_}, [&](hipStream_t s) {
      XDDP_NCCL_CHECK(ncclAllReduce(barrier_buf_.data_ptr(), barrier_buf_.data_ptr(), 1, ncclInt32, ncclSum, comm_, s));
    });
    w->synchronize();
    return w;
  }

  void group_start() override {
    XDDP_NCCL_CHECK(ncclGroupStart());
    in_group_++;
  }
  void group_end() override {
    if (in_group_ == 1) {
      end_group_launch(1);
    } else {
      XDDP_NCCL_CHECK(ncclGroupEnd());
    }
    --in_group_;
  }

  void abort() override {
    std::lock_guard<std::mutex> g(comm_mu_);
    if (comm_ && !aborted_) {
      ncclCommAbort(comm_);
      aborted_ = true;
    }
  }

  void shutdown() override {
    stop_watchdog();
    std::lock_guard<std::mutex> g(comm_mu_);
    if (comm_ && !aborted_ && !destroyed_) {
      c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
      XDDP_HIP_CHECK(hipStreamSynchronize(stream_.stream()));
      ncclCommDestroy(comm_);
      destroyed_ = true;
    }
    if (auto pr = std::atomic_load(&peer_)) {
      peer_quiesce(store_, rank_, size_, std::chrono::seconds(10));
      pr->close();
    }
  }

  // Peer-memory routing (comm/peer_allreduce.hip), node-local groups of 2..8 ranks:
  //   XDDP_PEER_ALLREDUCE=1: messages up to XDDP_PEER_ALLREDUCE_BYTES (default 256 KiB) take the
  //     one-shot kernel instead of an RCCL ring — the latency-bound per-forward buffer broadcast,
  //     find-unused bitmap and small first bucket;
  //   XDDP_PEER_ALLREDUCE=2: additionally, fp32/bf16/fp16 SUM/AVG all-reduces from
  //     XDDP_PEER_TWO_SHOT_MIN_BYTES (default 1 MiB) up to XDDP_PEER_TWO_SHOT_MAX_BYTES (default
  //     unlimited) take the two-shot kernel, which reads from all seven xGMI links at once
  //     (staging XDDP_PEER_TWO_SHOT_MB per slot, default 64; larger messages are chunked).
  // The route depends only on facts identical on every rank (size, dtype, op) — never on group
  // state — so all ranks issue the same sequence. Every rank must agree the path works: each
  // posts whether its IPC mapping succeeded and the path is used only if all did.
  //   XDDP_PEER_ALLREDUCE=auto: both lanes are created but on probation — nothing is routed to them
  //     and their timeouts are not communicator errors — until comm calibration
  //     (distributed/calibrate.py) has self-checked them on every rank and installed a route table
  //     from measured timings (finish_peer_probation: keep them or close them).
  void init_peer(const std::shared_ptr<Store>& store) {
    const char* e = std::getenv("XDDP_PEER_ALLREDUCE");
    const bool autom = e && std::string(e) == "auto";
    const int mode = autom ? 2 : (e ? std::atoi(e) : 0);
    // (one rank: only with XDDP_RCCL_FORCE_LAUNCH, so a one-GPU box runs the peer / calibration path)
    if (mode <= 0 || size_ > kPeerMaxRanks || (size_ < 2 && !force_launch_)) return;
    auto env_i64 = [](const char* k, int64_t d) {
      const char* v = std::getenv(k);
      return v ? static_cast<int64_t>(std::atof(v)) : d;
    };
    peer_bytes_ = env_i64("XDDP_PEER_ALLREDUCE_BYTES", 256 << 10);
    const int64_t cap = std::max<int64_t>(4096, (peer_bytes_ + 4095) / 4096 * 4096);
    int64_t cap2 = 0;
    if (mode >= 2) {
      two_shot_min_ = env_i64("XDDP_PEER_TWO_SHOT_MIN_BYTES", 1 << 20);
      two_shot_max_ = env_i64("XDDP_PEER_TWO_SHOT_MAX_BYTES", INT64_MAX);
      cap2 = std::max<int64_t>(4096, static_cast<int64_t>(env_i64("XDDP_PEER_TWO_SHOT_MB", 64) * (1 << 20)) / 4096 * 4096);
    }
    std::string ok = "1";
    try {
      peer_ = std::make_shared<PeerAllReduce>(store, rank_, size_, device_, cap, cap2, timeout_);
    } catch (const std::exception& ex) {
      ok = "0";
      peer_.reset();
      fprintf(stderr, "[xddp rccl] rank %d: peer all-reduce unavailable (%s)\n", rank_, ex.what());
    }
    store->set("peer/use/" + std::to_string(rank_), ok);
    bool all = true;
    for (int r = 0; r < size_; ++r) all = all && store->get("peer/use/" + std::to_string(r)) == "1";
    if (!all) peer_.reset();
    peer_mode_ = peer_ && !autom ? mode : 0;
    probation_ = peer_ && autom;
  }

  enum class PeerRoute { kRccl, kOneShot, kTwoShot };
  PeerRoute peer_route(const at::Tensor& t, RedOp op, bool bcast) const {
    if (!peer_) return PeerRoute::kRccl;
    const int64_t nb = static_cast<int64_t>(t.nbytes());
    if (!route_bounds_.empty()) {  // calibrated: the measured fastest route for this size
      for (size_t i = 0; i < route_bounds_.size(); ++i) {
        if (nb > route_bounds_[i]) continue;
        if (route_ids_[i] == kRouteOneShot && peer_->supports(t, op, bcast)) return PeerRoute::kOneShot;
        if (route_ids_[i] == kRouteTwoShot && !bcast && peer_->supports_two_shot(t, op)) return PeerRoute::kTwoShot;
        return PeerRoute::kRccl;
      }
      return PeerRoute::kRccl;
    }
    if (probation_) return PeerRoute::kRccl;
    if (nb <= peer_bytes_ && peer_->supports(t, op, bcast)) return PeerRoute::kOneShot;
    if (!bcast && peer_mode_ >= 2 && nb >= two_shot_min_ && nb <= two_shot_max_ && peer_->supports_two_shot(t, op))
      return PeerRoute::kTwoShot;
    return PeerRoute::kRccl;
  }

  std::map<std::string, std::string> info() const override {
    int dev = -1;
    if (comm_) ncclCommCuDevice(comm_, &dev);
    return {{"backend", "rccl"},
            {"rccl_version", rccl_version()},
            {"nranks", std::to_string(size_)},
            {"rank", std::to_string(rank_)},
            {"device", std::to_string(dev)},
            {"high_priority_stream", high_priority_ ? "1" : "0"},
            {"peer_mode", std::to_string(peer_mode_)},
            {"peer_one_shot_max_bytes", std::to_string(peer_ ? peer_bytes_ : 0)},
            {"peer_two_shot_min_bytes", std::to_string(peer_mode_ >= 2 ? two_shot_min_ : 0)},
            {"peer_probation", probation_ ? "1" : "0"},
            {"route_table_entries", std::to_string(route_bounds_.size())}};
  }

  hipStream_t stream() const { return stream_.stream(); }

 private:
  void check_tensor(const at::Tensor& t) {
    TORCH_CHECK(t.is_cuda(), "xddp rccl backend: tensor must be on a GPU");
    TORCH_CHECK(t.device().index() == device_, "xddp rccl backend: tensor on device ", t.device().index(),
                " but communicator is bound to device ", device_);
    TORCH_CHECK(t.is_non_overlapping_and_dense(), "xddp rccl backend: tensor must be dense");
  }
  void check_contig(const at::Tensor& t) {
    check_tensor(t);
    TORCH_CHECK(t.is_contiguous(), "xddp rccl backend: tensor must be contiguous");
  }

  template <typename F>
  std::shared_ptr<Work> launch(const char* name, const at::Tensor& meta, std::vector<at::Tensor> keep, F&& body) {
    TORCH_CHECK(err_->load() == 0, "xddp rccl: communicator is in error state; re-create the process group");
    TORCH_CHECK(!destroyed_, "xddp rccl: communicator was shut down");
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    auto cur = c10::hip::getCurrentHIPStream(device_);
    // HIP-graph capture: the comm stream joins the capture through the event wait below; works
    // recorded inside a capture are graph nodes, so the watchdog must not poll them.
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    XDDP_HIP_CHECK(hipStreamIsCapturing(cur.stream(), &cap));
    capturing_ = cap == hipStreamCaptureStatusActive;
    hipEvent_t pre = pool_->get();
    XDDP_HIP_CHECK(hipEventRecord(pre, cur.stream()));
    XDDP_HIP_CHECK(hipStreamWaitEvent(stream_.stream(), pre, 0));
    pool_->put(pre);
    auto w = std::make_shared<RcclWork>(pool_, device_, err_, probation_ ? nullptr : std::atomic_load(&peer_));
    w->seq = flight_.record(name, meta.numel(), meta.scalar_type());
    const bool timed = timing_.load() && !capturing_;
    // Inside a group the RCCL kernels are enqueued at ncclGroupEnd: the group is timed there.
    if (timed && in_group_ == 0) {
      w->iv = std::make_shared<Interval>(tpool_);
      XDDP_HIP_CHECK(hipEventRecord(w->iv->t0, stream_.stream()));
    }
    body(stream_.stream());
    if (w->iv) XDDP_HIP_CHECK(hipEventRecord(w->iv->t1, stream_.stream()));
    if (!capturing_) {
      for (auto& t : keep) {
        if (t.defined() && t.is_cuda())
          c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_);
      }
    }
    w->outputs = std::move(keep);
    w->captured = capturing_;
    if (timed) log_timed(w);
    if (in_group_ > 0) {
      if (timed) timed_group_ = true;
      group_works_.push_back(w);
    } else {
      finish_launch(w);
    }
    return w;
  }

  // A peer-memory collective issued inside an RCCL group: the group's pending RCCL launches go
  // out first (ncclGroupEnd down to depth 0, then reopened at the same depth), so the stream
  // order of peer and RCCL kernels is the issue order — identical on every rank, whatever the
  // local grouping (a joined rank shadows all buckets in one group while training ranks launch
  // them one by one).
  template <typename F>
  std::shared_ptr<Work> launch_peer(const char* name, const at::Tensor& meta, std::vector<at::Tensor> keep,
                                    F&& body) {
    const int depth = in_group_;
    if (depth > 0) {
      end_group_launch(depth);
      in_group_ = 0;
    }
    auto w = launch(name, meta, std::move(keep), std::forward<F>(body));
    for (int k = 0; k < depth; ++k) XDDP_NCCL_CHECK(ncclGroupStart());
    in_group_ = depth;
    return w;
  }

  // Close `depth` levels of ncclGroupStart (RCCL launches the group's kernels when the depth
  // reaches 0) and hand the grouped works to the watchdog; with timing on, the whole grouped
  // launch is one comm-stream interval reported by its first work.
  void end_group_launch(int depth) {
    std::shared_ptr<Interval> iv;
    if (timed_group_ && !group_works_.empty()) {
      c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
      iv = std::make_shared<Interval>(tpool_);
      XDDP_HIP_CHECK(hipEventRecord(iv->t0, stream_.stream()));
    }
    for (int k = 0; k < depth; ++k) XDDP_NCCL_CHECK(ncclGroupEnd());
    if (iv) XDDP_HIP_CHECK(hipEventRecord(iv->t1, stream_.stream()));
    for (size_t i = 0; i < group_works_.size(); ++i) {
      if (iv) {
        group_works_[i]->iv = iv;
        group_works_[i]->owns_interval = i == 0;
      }
      finish_launch(group_works_[i]);
    }
    group_works_.clear();
    timed_group_ = false;
  }

  // One-rank collectives that are identities: no RCCL launch, a Work that is already ordered.
  std::shared_ptr<Work> local_noop(const char* name, const at::Tensor& t) {
    TORCH_CHECK(err_->load() == 0, "xddp rccl: communicator is in error state");
    auto w = std::make_shared<RcclWork>(pool_, device_, err_, probation_ ? nullptr : std::atomic_load(&peer_));
    w->seq = flight_.record(name, t.numel(), t.scalar_type());
    XDDP_HIP_CHECK(hipEventRecord(w->ev, c10::hip::getCurrentHIPStream(device_).stream()));
    w->launched = true;
    flight_.finish(w->seq, "completed");
    w->outputs = {t};
    w->collective = false;  // one rank: nothing crossed a link
    return w;
  }

  void finish_launch(const std::shared_ptr<RcclWork>& w) {
    XDDP_HIP_CHECK(hipEventRecord(w->ev, stream_.stream()));
    w->launched = true;
    if (w->captured) return;  // a graph node, not a live collective
    std::lock_guard<std::mutex> g(wd_mu_);
    inflight_.push_back(w);
  }

  void watchdog_loop() {
    std::string reason;
    int64_t last_peer_poll = 0;
    while (!wd_stop_) {
      heartbeat_ = now_ns();
      bool poll_peers = false;
      {
        std::unique_lock<std::mutex> g(wd_mu_);
        wd_cv_.wait_for(g, std::chrono::milliseconds(100), [&] { return wd_stop_.load(); });
        if (wd_stop_) break;
        const int64_t now = now_ns();
        int64_t oldest = now;
        for (auto it = inflight_.begin(); it != inflight_.end();) {
          hipError_t q = hipEventQuery((*it)->ev);
          if (q == hipSuccess) {
            flight_.finish((*it)->seq, "completed");
            it = inflight_.erase(it);
          } else if (now - (*it)->t_start > static_cast<int64_t>(timeout_.count()) * 1000000LL) {
            flight_.finish((*it)->seq, "timeout");
            reason = "collective seq " + std::to_string((*it)->seq) + " exceeded timeout of " +
                     std::to_string(timeout_.count()) + " ms";
            std::cerr << "[xddp rank " << rank_ << "] watchdog: " << reason << "; aborting communicator\n";
            err_->store(1);
            it = inflight_.erase(it);
          } else {
            oldest = std::min(oldest, (*it)->t_start);
            ++it;
          }
        }
        // a healthy step never has a collective in flight for a second: only then ask the
        // store whether a peer has already failed
        if (err_->load() == 0 && now - oldest > 1000000000LL && now - last_peer_poll > 1000000000LL) {
          last_peer_poll = now;
          poll_peers = true;
        }
      }
      // the store round trip runs without wd_mu_: collectives launched meanwhile
      // (finish_launch) must not wait on a slow or vanished store host
      if (poll_peers) {
        try {
          if (store_->check({"rccl/error"})) {
            reason = "peer error: " + store_->get("rccl/error");
            std::cerr << "[xddp rank " << rank_ << "] watchdog: " << reason << "; aborting communicator\n";
            err_->store(3);
          }
        } catch (...) {
        }
      }
      auto pr = std::atomic_load(&peer_);
      if ((err_->load() == 0 || err_->load() == 4) && reason.empty() && pr && !probation_ && pr->status() != 0) {
        // (a Work query may have flagged it first; the watchdog still dumps, posts and aborts)
        reason = "peer-memory collective: a rank did not arrive within " +
                 std::to_string(static_cast<int64_t>(pr->timeout_ms())) + " ms (XDDP_PEER_TIMEOUT_MS)";
        std::cerr << "[xddp rank " << rank_ << "] watchdog: " << reason << "; aborting communicator\n";
        int z = 0;
        err_->compare_exchange_strong(z, 4);
      }
      if (err_->load() == 0 && comm_ && !aborted_ && !destroyed_) {
        ncclResult_t ae = ncclSuccess;
        if (ncclCommGetAsyncError(comm_, &ae) == ncclSuccess && ae != ncclSuccess && ae != ncclInProgress) {
          reason = std::string("async RCCL error ") + ncclGetErrorString(ae);
          std::cerr << "[xddp rank " << rank_ << "] watchdog: " << reason << "\n";
          err_->store(2);
        }
      }
      if (err_->load() != 0 && !aborted_) {
        dump_flight(reason);
        if (err_->load() != 3) {
          try {
            store_->set("rccl/error", "rank " + std::to_string(rank_) + ": " + reason);
          } catch (...) {
          }
        }
        abort();
      }
    }
  }

  void monitor_loop() {
    std::unique_lock<std::mutex> g(hb_mu_);
    while (!wd_stop_) {
      hb_cv_.wait_for(g, std::chrono::seconds(1), [&] { return wd_stop_.load(); });
      if (wd_stop_) break;
      const double idle_s = (now_ns() - heartbeat_.load()) * 1e-9;
      if (idle_s > hb_timeout_s_) {
        std::cerr << "[xddp rank " << rank_ << "] heartbeat monitor: watchdog silent for " << idle_s
                  << " s (XDDP_HEARTBEAT_TIMEOUT_SEC=" << hb_timeout_s_ << "); aborting the process\n";
        dump_flight("watchdog heartbeat lost", true);
        std::abort();
      }
    }
  }

  void stop_watchdog() {
    wd_stop_ = true;
    wd_cv_.notify_all();
    hb_cv_.notify_all();
    if (watchdog_.joinable()) watchdog_.join();
    if (monitor_.joinable()) monitor_.join();
  }

  std::shared_ptr<Store> store_;
  int device_;
  std::chrono::milliseconds timeout_;
  c10::hip::HIPStream stream_;
  std::shared_ptr<EventPool> pool_;
  std::shared_ptr<EventPool> tpool_;  // timing-enabled events (Comm::set_timing)
  std::shared_ptr<std::atomic<int>> err_;
  ncclComm_t comm_ = nullptr;
  std::mutex comm_mu_;
  bool aborted_ = false;
  bool destroyed_ = false;
  std::shared_ptr<PeerAllReduce> peer_;
  int peer_mode_ = 0;
  std::atomic<bool> probation_{false};
  std::vector<int64_t> route_bounds_;
  std::vector<int> route_ids_;
  int64_t peer_bytes_ = 0;
  int64_t two_shot_min_ = 0;
  int64_t two_shot_max_ = 0;
  bool high_priority_ = true;
  bool timed_group_ = false;
  bool force_launch_ = false;
  int in_group_ = 0;
  bool capturing_ = false;
  std::vector<std::shared_ptr<RcclWork>> group_works_;
  at::Tensor barrier_buf_;
  std::thread watchdog_;
  std::atomic<bool> wd_stop_{false};
  std::mutex wd_mu_;
  std::condition_variable wd_cv_;
  std::list<std::shared_ptr<RcclWork>> inflight_;
  std::atomic<int64_t> heartbeat_{0};
  double hb_timeout_s_ = 480.0;
  std::thread monitor_;
  std::mutex hb_mu_;
  std::condition_variable hb_cv_;
};

std::shared_ptr<Comm> make_rccl_comm(std::shared_ptr<Store> store, int rank, int size, int device,
                                     std::chrono::milliseconds timeout, bool high_priority_stream) {
  return std::make_shared<RcclComm>(std::move(store), rank, size, device, timeout, high_priority_stream);
}

std::string rccl_version() {
  int v = 0;
  ncclGetVersion(&v);
  return std::to_string(v / 10000) + "." + std::to_string((v % 10000) / 100) + "." + std::to_string(v % 100);
}

int64_t rccl_stream_handle(const std::shared_ptr<Comm>& c) {
  auto r = std::dynamic_pointer_cast<RcclComm>(c);
  TORCH_CHECK(r, "not an RCCL communicator");
  return reinterpret_cast<int64_t>(r->stream());
}

}  // namespace xddp
