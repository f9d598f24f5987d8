// Communicator abstraction for xddp.
//
// Two native backends implement it:
//   * RcclComm — RCCL over xGMI on a dedicated high-priority HIP stream, hipEvent-based Work,
//                group coalescing, watchdog thread (timeout + async-error → ncclCommAbort).
//   * TcpComm  — CPU ring collectives over a TCP full mesh, executed in FIFO order on a
//                worker thread (the GPU-free multi-process test backend; gloo's role).
// Every collective is recorded in a bounded ring buffer ("flight recorder", T20) that
// Python can dump for desync/timeout triage.
#pragma once

#include <ATen/ATen.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <exception>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "common.h"
#include "store/tcp_store.h"

namespace xddp {

// A point in time a collective's interval can be compared against: a hipEvent recorded on the
// same device (device backends) or a steady-clock timestamp (CPU backend).
struct TimeRef {
  hipEvent_t ev = nullptr;
  int64_t ns = 0;
};

class Work {
 public:
  enum class Timing { kNone, kPending, kReady };
  virtual ~Work() = default;
  // Non-blocking completion query.
  virtual bool is_completed() = 0;
  // GPU: make the caller's current stream wait for the collective (no host block).
  // CPU: block until done. Re-throws a collective error.
  virtual void wait() = 0;
  // Block the host until the collective has finished on the device.
  virtual void synchronize() { wait(); }
  virtual std::vector<at::Tensor> result() { return outputs; }

  // Collective timing, measured where the collective ran (timing-enabled hipEvents around the
  // launch on the comm stream; the worker thread's clock on the CPU backend). Only works issued
  // while Comm::set_timing(true) are timed. A grouped launch (RCCL group) is timed as one interval
  // reported by the first work of the group; the others report 0 ms.
  virtual Timing timing_state() { return Timing::kNone; }
  virtual double comm_ms() { return 0.0; }
  // Milliseconds of the collective's interval that lie before `ref` (clamped to [0, comm_ms]).
  virtual double comm_ms_before(const TimeRef& /*ref*/) { return 0.0; }

  std::vector<at::Tensor> outputs;
  int64_t seq = -1;
  // false: nothing crossed a link (a one-rank identity; the fake backend)
  bool collective = true;
};

struct FlightEntry {
  int64_t seq;
  std::string op;
  int64_t numel;
  std::string dtype;
  int64_t t_enqueue_ns;
  int64_t t_done_ns;  // 0 while in flight
  std::string state;  // "scheduled" | "completed" | "failed" | "timeout"
};

class FlightRecorder {
 public:
  explicit FlightRecorder(size_t cap = 2048) : cap_(cap) {}
  int64_t record(const std::string& op, int64_t numel, at::ScalarType dt) {
    std::lock_guard<std::mutex> g(mu_);
    int64_t s = next_++;
    if (ring_.size() == cap_) ring_.pop_front();
    ring_.push_back(FlightEntry{s, op, numel, std::string(c10::toString(dt)), now_ns(), 0, "scheduled"});
    return s;
  }
  void finish(int64_t seq, const char* state) {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = ring_.rbegin(); it != ring_.rend(); ++it) {
      if (it->seq == seq) {
        it->t_done_ns = now_ns();
        it->state = state;
        return;
      }
    }
  }
  std::vector<FlightEntry> dump() {
    std::lock_guard<std::mutex> g(mu_);
    return std::vector<FlightEntry>(ring_.begin(), ring_.end());
  }
  // JSON document of the ring (newest last), for post-mortem desync/timeout triage.
  std::string to_json(int rank, const std::string& backend, const std::string& reason);
  int64_t count() const { return next_; }

 private:
  size_t cap_;
  std::mutex mu_;
  std::deque<FlightEntry> ring_;
  std::atomic<int64_t> next_{0};
};

class Comm : public std::enable_shared_from_this<Comm> {
 public:
  Comm(int rank, int size) : rank_(rank), size_(size) {}
  virtual ~Comm() = default;
  int rank() const { return rank_; }
  int size() const { return size_; }
  virtual std::string backend() const = 0;

  virtual std::shared_ptr<Work> allreduce(at::Tensor t, RedOp op, double premul = 1.0) = 0;
  virtual std::shared_ptr<Work> broadcast(at::Tensor t, int root) = 0;
  // out.numel() == size * in.numel(); rank r's input lands at out[r*n:(r+1)*n].
  virtual std::shared_ptr<Work> allgather(at::Tensor out, at::Tensor in) = 0;
  // in.numel() == size * out.numel()
  virtual std::shared_ptr<Work> reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) = 0;
  // equal splits: in/out numel divisible by size
  virtual std::shared_ptr<Work> alltoall(at::Tensor out, at::Tensor in) = 0;
  virtual std::shared_ptr<Work> send(at::Tensor t, int dst) = 0;
  virtual std::shared_ptr<Work> recv(at::Tensor t, int src) = 0;
  virtual std::shared_ptr<Work> barrier() = 0;
  // Coalescing window (RCCL group); CPU backend runs ops in order anyway.
  virtual void group_start() {}
  virtual void group_end() {}
  virtual void abort() {}
  virtual void shutdown() {}
  // Time the collectives issued from now on (see Work::comm_ms). Off by default: the events
  // cost a little on every launch, so the Reducer turns it on only for its sampled iterations.
  virtual void set_timing(bool on) { timing_ = on; }
  bool timing() const { return timing_; }
  // The works issued while timing was on, in launch order (cleared by the call). The Reducer
  // drains them after a sampled backward: bucket all-reduces, comm-hook collectives, the
  // find-unused bitmap — everything that crossed a link during that backward.
  virtual std::vector<std::shared_ptr<Work>> drain_timed_works() {
    std::lock_guard<std::mutex> g(timed_mu_);
    std::vector<std::shared_ptr<Work>> out;
    out.swap(timed_log_);
    return out;
  }
  // ---- route control for comm calibration (distributed/calibrate.py) ----------
  // Routes of an all-reduce: 0 = the communicator's own choice (route table), 1 = its base path
  // (the RCCL ring; one-shot chunks on the peer backend), 2 = the one-shot peer kernel, 3 = the
  // two-shot peer kernel.
  enum Route { kRouteAuto = 0, kRouteBase = 1, kRouteOneShot = 2, kRouteTwoShot = 3 };
  virtual std::shared_ptr<Work> allreduce_via(at::Tensor t, RedOp op, int /*route*/) { return allreduce(t, op, 1.0); }
  // Routes besides auto/base this communicator can run now (RCCL: {2, 3} once the peer lanes exist).
  virtual std::vector<int> routes() const { return {}; }
  // Largest message the one-shot lane takes in one launch (0: none).
  virtual int64_t one_shot_capacity() const { return 0; }
  // Route table: an all-reduce of nb bytes takes routes[i] for the first bounds[i] >= nb, the
  // base path beyond the last bound; a route the tensor/op cannot take falls back to the base path.
  // Must be identical on every rank (it is computed from MAX-reduced timings).
  virtual void set_route_table(const std::vector<int64_t>& /*bounds*/, const std::vector<int>& /*routes*/) {}
  virtual std::vector<std::vector<int64_t>> route_table() const { return {}; }
  // Peer lanes' host-mapped status word: 0 ok, 1 a peer kernel timed out.
  virtual int peer_status() const { return 0; }
  // Device-side wait bound of the peer kernels from now on (calibration uses a short one).
  virtual void set_peer_timeout_ms(double /*ms*/) {}
  // End of the peer lanes' probation: keep=false closes them (everything takes the base path);
  // keep=true arms them (their failures become communicator errors from now on).
  virtual void finish_peer_probation(bool /*keep*/) {}

  // Backend facts for logs/benchmarks (RCCL: version, channel count seen at init, ...).
  virtual std::map<std::string, std::string> info() const { return {{"backend", backend()}}; }

  virtual FlightRecorder& flight() { return flight_; }
  // Writes the flight record to $XDDP_FLIGHT_DUMP_PREFIX<rank>.json (default
  // /tmp/xddp_flight_rank_<rank>.json) unless XDDP_FLIGHT_DUMP_ON_ERROR=0 and !force;
  // returns the path ("" if skipped). Called by the backends on timeout / comm error.
  std::string dump_flight(const std::string& reason, bool force = false);
  // Debug: TORCH_DISTRIBUTED_DEBUG=DETAIL-style fingerprint check before each collective.
  bool debug_fingerprint = false;

 protected:
  void log_timed(std::shared_ptr<Work> w) {
    std::lock_guard<std::mutex> g(timed_mu_);
    if (timed_log_.size() < 4096) timed_log_.push_back(std::move(w));
  }
  int rank_, size_;
  FlightRecorder flight_;
  std::atomic<bool> timing_{false};
  std::mutex timed_mu_;
  std::vector<std::shared_ptr<Work>> timed_log_;
};

// CPU backend ---------------------------------------------------------------------------
std::shared_ptr<Comm> make_tcp_comm(std::shared_ptr<Store> store, int rank, int size,
                                    std::chrono::milliseconds timeout);
// `host` = address peers use to reach this rank's listening socket.
std::shared_ptr<Comm> make_tcp_comm_host(std::shared_ptr<Store> store, int rank, int size,
                                         std::chrono::milliseconds timeout, const std::string& host);

// RCCL backend --------------------------------------------------------------------------
std::shared_ptr<Comm> make_rccl_comm(std::shared_ptr<Store> store, int rank, int size, int device,
                                     std::chrono::milliseconds timeout, bool high_priority_stream);

// Peer-memory backend (single node, device tensors; comm/peer_comm.cpp). capacity = one-shot
// staging bytes, two_shot_capacity = two-shot staging bytes (0: one-shot only).
std::shared_ptr<Comm> make_peer_comm(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity,
                                     int64_t two_shot_capacity, std::chrono::milliseconds timeout);

// Debug wrapper: per-collective cross-rank fingerprint check and/or NaN check. `helper` (a CPU
// communicator over the same ranks) carries the fingerprints; required for device backends.
std::shared_ptr<Comm> make_debug_comm(std::shared_ptr<Comm> inner, bool fingerprint, bool nan_check,
                                      std::shared_ptr<Comm> helper = nullptr);

// Extra RCCL-only entry points (no-ops / errors for other backends).
std::string rccl_version();
// Stream the RCCL comm runs on (raw handle as int64) — for tests/profiling.
int64_t rccl_stream_handle(const std::shared_ptr<Comm>& c);

}  // namespace xddp
