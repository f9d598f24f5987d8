// Debug communicator (TORCH_DISTRIBUTED_DEBUG=DETAIL / ProcessGroupWrapper and
// TORCH_NCCL_NAN_CHECK analogues). Wraps any Comm:
//  * fingerprint mode: before every collective, all-gather (seq, op, numel, dtype, arg) from all
//    ranks and raise a readable desync report on mismatch — turns a silent RCCL hang (ranks
//    issuing different collectives) into an exception. The fingerprints travel over a separate
//    host-side communicator (the CPU TCP ring on its own store prefix; ProcessGroupWrapper's gloo
//    helper group in the reference stack), never through the wrapped device communicator: an RCCL
//    collective issued inside an open ncclGroupStart (the Reducer's bucket bursts, coalescing()
//    blocks) is only enqueued at ncclGroupEnd, so a fingerprint sent through it could not complete
//    before the check reads it. The host exchange is synchronous and group-agnostic, so the check
//    runs before every collective, grouped or not;
//  * NaN check: before a reduction, scan the input with the multi-tensor non-finite kernel
//    (GPU) or at::isfinite (CPU) and raise naming the collective.
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#include <functional>
#include <sstream>

#include "comm/comm.h"
#include "kernels/multi_tensor.h"

namespace xddp {

class DebugComm : public Comm {
 public:
  DebugComm(std::shared_ptr<Comm> inner, bool fingerprint, bool nan_check, std::shared_ptr<Comm> helper)
      : Comm(inner->rank(), inner->size()),
        inner_(std::move(inner)),
        helper_(std::move(helper)),
        fingerprint_(fingerprint),
        nan_(nan_check) {
    TORCH_CHECK(!fingerprint_ || helper_ || (inner_->backend() != "rccl" && inner_->backend() != "peer"),
                "xddp debug comm: fingerprints of a device communicator need a host-side helper communicator");
    TORCH_CHECK(!helper_ || (helper_->rank() == rank_ && helper_->size() == size_),
                "xddp debug comm: helper communicator rank/size differ from the wrapped one");
  }

  std::string backend() const override { return inner_->backend(); }

  std::shared_ptr<Work> allreduce(at::Tensor t, RedOp op, double premul) override {
    pre("allreduce", t, static_cast<int64_t>(op), true);
    return inner_->allreduce(t, op, premul);
  }
  std::shared_ptr<Work> broadcast(at::Tensor t, int root) override {
    pre("broadcast", t, root, false);
    return inner_->broadcast(t, root);
  }
  std::shared_ptr<Work> allgather(at::Tensor out, at::Tensor in) override {
    pre("allgather", in, 0, false);
    return inner_->allgather(out, in);
  }
  std::shared_ptr<Work> reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) override {
    pre("reduce_scatter", in, static_cast<int64_t>(op), true);
    return inner_->reduce_scatter(out, in, op);
  }
  std::shared_ptr<Work> alltoall(at::Tensor out, at::Tensor in) override {
    pre("alltoall", in, 0, false);
    return inner_->alltoall(out, in);
  }
  // point-to-point ops are not collective: no fingerprint
  std::shared_ptr<Work> send(at::Tensor t, int dst) override { return inner_->send(t, dst); }
  std::shared_ptr<Work> recv(at::Tensor t, int src) override { return inner_->recv(t, src); }
  std::shared_ptr<Work> barrier() override {
    pre("barrier", at::Tensor(), 0, false);
    return inner_->barrier();
  }
  void group_start() override { inner_->group_start(); }
  void group_end() override { inner_->group_end(); }
  void abort() override { inner_->abort(); }
  void shutdown() override {
    inner_->shutdown();
    if (helper_) helper_->shutdown();
  }
  void set_timing(bool on) override {
    Comm::set_timing(on);
    inner_->set_timing(on);
  }
  std::map<std::string, std::string> info() const override { return inner_->info(); }
  std::shared_ptr<Work> allreduce_via(at::Tensor t, RedOp op, int route) override {
    pre("allreduce", t, static_cast<int64_t>(op), true);
    return inner_->allreduce_via(t, op, route);
  }
  std::vector<int> routes() const override { return inner_->routes(); }
  int64_t one_shot_capacity() const override { return inner_->one_shot_capacity(); }
  void set_route_table(const std::vector<int64_t>& b, const std::vector<int>& r) override { inner_->set_route_table(b, r); }
  std::vector<std::vector<int64_t>> route_table() const override { return inner_->route_table(); }
  int peer_status() const override { return inner_->peer_status(); }
  void set_peer_timeout_ms(double ms) override { inner_->set_peer_timeout_ms(ms); }
  void finish_peer_probation(bool keep) override { inner_->finish_peer_probation(keep); }
  std::vector<std::shared_ptr<Work>> drain_timed_works() override { return inner_->drain_timed_works(); }
  std::shared_ptr<Comm> inner() const { return inner_; }
  FlightRecorder& flight() override { return inner_->flight(); }

 private:
  static int64_t op_code(const char* op) {
    return static_cast<int64_t>(std::hash<std::string>{}(op) & 0x7fffffff);
  }

  void pre(const char* op, const at::Tensor& t, int64_t arg, bool reduction) {
    if (nan_ && reduction && t.defined() && at::isFloatingType(t.scalar_type()) && t.numel() > 0) check_nan(op, t);
    if (fingerprint_) check_fingerprint(op, t, arg);
    seq_++;
  }

  void check_nan(const char* op, const at::Tensor& t) {
    bool bad;
    if (t.is_cuda() && t.is_non_overlapping_and_dense()) {
      auto flag = at::empty({1}, t.options().dtype(at::kInt));
      kernels::mt_nonfinite({t}, flag, c10::hip::getCurrentHIPStream(t.device().index()).stream());
      bad = flag.item<int>() != 0;
    } else {
      bad = !at::isfinite(t).all().item<bool>();
    }
    TORCH_CHECK(!bad, "xddp NaN check: rank ", rank_, " is about to ", op, " a tensor with NaN/Inf values (seq ",
                seq_, ", numel ", t.numel(), ")");
  }

  void check_fingerprint(const char* op, const at::Tensor& t, int64_t arg) {
    const int64_t numel = t.defined() ? t.numel() : 0;
    const int64_t dt = t.defined() ? static_cast<int64_t>(t.scalar_type()) : -1;
    auto fp = at::tensor(std::vector<int64_t>{seq_, op_code(op), numel, dt, arg}, at::kLong);
    auto all = at::zeros({size_ * 5}, at::kLong);
    // host tensors over a host communicator: wait() returns once every rank's record is in `all`
    (helper_ ? helper_ : inner_)->allgather(all, fp)->wait();
    const int64_t* a = all.data_ptr<int64_t>();
    bool same = true;
    for (int r = 1; r < size_; ++r)
      for (int k = 0; k < 5; ++k) same = same && a[r * 5 + k] == a[k];
    if (!same) {
      std::ostringstream os;
      os << "xddp collective desync detected (XDDP_DEBUG=DETAIL) at rank " << rank_ << ":\n";
      for (int r = 0; r < size_; ++r)
        os << "  rank " << r << ": seq=" << a[r * 5] << " op_hash=" << a[r * 5 + 1] << " numel=" << a[r * 5 + 2]
           << " dtype=" << a[r * 5 + 3] << " arg=" << a[r * 5 + 4] << (r == rank_ ? "  <- this rank (" : "")
           << (r == rank_ ? op : "") << (r == rank_ ? ")" : "") << "\n";
      TORCH_CHECK(false, os.str());
    }
  }

  std::shared_ptr<Comm> inner_;
  std::shared_ptr<Comm> helper_;  // host-side fingerprint exchange (device backends)
  bool fingerprint_, nan_;
  int64_t seq_ = 0;
};

std::shared_ptr<Comm> make_debug_comm(std::shared_ptr<Comm> inner, bool fingerprint, bool nan_check,
                                      std::shared_ptr<Comm> helper) {
  return std::make_shared<DebugComm>(std::move(inner), fingerprint, nan_check, std::move(helper));
}

}  // namespace xddp
