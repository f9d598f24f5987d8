// PeerComm: an RCCL-free single-node communicator for device tensors, built on the one-shot
// peer-memory kernels of peer_allreduce.hip (IPC-mapped staging buffers, xGMI loads). Backend
// "peer" of init_process_group.
//
// Every collective runs on one dedicated HIP stream that first waits for the caller's stream
// (event), so it is ordered after the producer of its input; Work.wait() makes the caller's stream
// wait for the collective's completion event (no host blocking). Messages larger than the staging
// capacity (XDDP_PEER_CAPACITY_MB, default 16 MiB) are walked in capacity-sized chunks, each one a
// kernel with its own flag barrier. All-reduce (SUM / AVG / MAX; PREMUL_SUM as SUM + scale),
// broadcast, all-gather, reduce-scatter (all-reduce + own slice) and barrier are supported;
// all-to-all and point-to-point are not (use the RCCL backend).
//
// Why it exists: on a 1-GPU box two ranks can share the device through it (RCCL refuses duplicate
// devices), so the W > 1 DDP path — bucket launches, stream ordering, Work semantics — runs
// against device-side collectives, not the host-staged CPU backend; on a node it is the same
// peer-memory protocol the RCCL communicator uses for small messages (XDDP_PEER_ALLREDUCE).
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>

#include <memory>

#include "comm/comm.h"
#include "comm/peer.h"

namespace xddp {

namespace {

class PeerWork : public Work {
 public:
  PeerWork(int device, hipEvent_t ev) : device_(device), ev_(ev) {}
  ~PeerWork() override {
    if (ev_) (void)hipEventDestroy(ev_);
  }
  bool is_completed() override { return hipEventQuery(ev_) == hipSuccess; }
  void wait() override {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    XDDP_HIP_CHECK(hipStreamWaitEvent(c10::hip::getCurrentHIPStream(device_).stream(), ev_, 0));
  }
  void synchronize() override { XDDP_HIP_CHECK(hipEventSynchronize(ev_)); }

 private:
  int device_;
  hipEvent_t ev_;
};

class PeerComm : public Comm {
 public:
  PeerComm(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity)
      : Comm(rank, size),
        device_(device),
        stream_(c10::hip::getStreamFromPool(true, static_cast<c10::DeviceIndex>(device))),
        peer_(std::make_unique<PeerAllReduce>(std::move(store), rank, size, device, capacity)) {}

  std::string backend() const override { return "peer"; }

  std::shared_ptr<Work> allreduce(at::Tensor t, RedOp op, double premul) override {
    TORCH_CHECK(op == RedOp::SUM || op == RedOp::AVG || op == RedOp::MAX || op == RedOp::PREMUL_SUM,
                "peer backend: all-reduce supports SUM, AVG, MAX and PREMUL_SUM");
    const RedOp kop = op == RedOp::PREMUL_SUM ? RedOp::SUM : op;
    return launch("allreduce", t, {t}, [&](hipStream_t s) {
      for_chunks(t, [&](at::Tensor c) { peer_->allreduce(c, kop, s); });
      if (op == RedOp::PREMUL_SUM) t.mul_(premul);  // (on the comm stream: the guard below)
    });
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

  void shutdown() override { peer_->close(); }

 private:
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

  template <typename F>
  std::shared_ptr<Work> launch(const char* name, const at::Tensor& meta, std::vector<at::Tensor> keep, F&& body) {
    c10::hip::HIPGuard guard(static_cast<c10::DeviceIndex>(device_));
    auto cur = c10::hip::getCurrentHIPStream(device_);
    hipEvent_t pre;
    XDDP_HIP_CHECK(hipEventCreateWithFlags(&pre, hipEventDisableTiming));
    XDDP_HIP_CHECK(hipEventRecord(pre, cur.stream()));
    XDDP_HIP_CHECK(hipStreamWaitEvent(stream_.stream(), pre, 0));
    XDDP_HIP_CHECK(hipEventDestroy(pre));
    const int64_t seq = flight_.record(name, meta.numel(), meta.scalar_type());
    {
      c10::hip::HIPStreamGuard sg(stream_);  // torch ops in the body (chunk copies, scaling) too
      body(stream_.stream());
    }
    for (auto& t : keep)
      if (t.defined() && t.is_cuda()) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), stream_);
    hipEvent_t done;
    XDDP_HIP_CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
    XDDP_HIP_CHECK(hipEventRecord(done, stream_.stream()));
    flight_.finish(seq, "completed");  // (enqueued; completion is the event)
    auto w = std::make_shared<PeerWork>(device_, done);
    w->outputs = std::move(keep);
    w->seq = seq;
    return w;
  }

  int device_;
  c10::hip::HIPStream stream_;
  std::unique_ptr<PeerAllReduce> peer_;
  at::Tensor barrier_buf_;
};

}  // namespace

std::shared_ptr<Comm> make_peer_comm(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity) {
  return std::make_shared<PeerComm>(std::move(store), rank, size, device, capacity);
}

}  // namespace xddp
