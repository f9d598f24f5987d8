// "fake" backend: every collective completes immediately without touching peers (the
// reference stack's FakeProcessGroup). One process can then pretend to be
// rank r of a world of any size — e.g. to test bucket assignment, reducer bookkeeping and
// hook plumbing at world_size=64 without 64 processes. Semantics: all-reduce/broadcast leave
// the tensor as is, all-gather replicates the local input into every slot, reduce-scatter
// copies this rank's shard, all-to-all copies in -> out, send/recv/barrier are no-ops.
#include "comm/comm.h"

namespace xddp {

namespace {

class DoneWork : public Work {
 public:
  bool is_completed() override { return true; }
  void wait() override {}
};

class FakeComm : public Comm {
 public:
  FakeComm(int rank, int size) : Comm(rank, size) {}
  std::string backend() const override { return "fake"; }
  std::shared_ptr<Work> allreduce(at::Tensor t, RedOp, double) override { return done("allreduce", t, {t}); }
  std::shared_ptr<Work> broadcast(at::Tensor t, int) override { return done("broadcast", t, {t}); }
  std::shared_ptr<Work> allgather(at::Tensor out, at::Tensor in) override {
    TORCH_CHECK(out.numel() == in.numel() * size_, "allgather: output must hold size*input elements");
    out.view({size_, in.numel()}).copy_(in.reshape({1, -1}).expand({size_, in.numel()}));
    return done("allgather", in, {out});
  }
  std::shared_ptr<Work> reduce_scatter(at::Tensor out, at::Tensor in, RedOp) override {
    TORCH_CHECK(in.numel() == out.numel() * size_, "reduce_scatter: input must hold size*output elements");
    out.reshape({-1}).copy_(in.reshape({-1}).narrow(0, rank_ * out.numel(), out.numel()));
    return done("reduce_scatter", in, {out});
  }
  std::shared_ptr<Work> alltoall(at::Tensor out, at::Tensor in) override {
    out.copy_(in);
    return done("alltoall", in, {out});
  }
  std::shared_ptr<Work> send(at::Tensor t, int) override { return done("send", t, {}); }
  std::shared_ptr<Work> recv(at::Tensor t, int) override { return done("recv", t, {t}); }
  std::shared_ptr<Work> barrier() override { return done("barrier", at::Tensor(), {}); }

 private:
  std::shared_ptr<Work> done(const char* name, const at::Tensor& meta, std::vector<at::Tensor> outs) {
    auto w = std::make_shared<DoneWork>();
    w->collective = false;
    w->seq = flight_.record(name, meta.defined() ? meta.numel() : 0, meta.defined() ? meta.scalar_type() : at::kByte);
    flight_.finish(w->seq, "completed");
    w->outputs = std::move(outs);
    return w;
  }
};

}  // namespace

std::shared_ptr<Comm> make_fake_comm(int rank, int size) { return std::make_shared<FakeComm>(rank, size); }

}  // namespace xddp
