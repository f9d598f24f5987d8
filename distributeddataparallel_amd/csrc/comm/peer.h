// One-shot small-message all-reduce / broadcast over IPC-mapped peer buffers (xGMI).
// See peer_allreduce.hip for the protocol.
#pragma once

#include <ATen/ATen.h>
#include <hip/hip_runtime.h>

#include <memory>

#include "common.h"
#include "store/tcp_store.h"

namespace xddp {

constexpr int kPeerMaxRanks = 8;
constexpr int kPeerMaxBlocks = 64;

class PeerAllReduce {
 public:
  // Collective over `size` ranks of one node (all must construct it; IPC handles go through
  // `store`). capacity: largest message in bytes (a multiple of 4 KiB).
  PeerAllReduce(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity);
  ~PeerAllReduce();
  PeerAllReduce(const PeerAllReduce&) = delete;
  PeerAllReduce& operator=(const PeerAllReduce&) = delete;

  // Contiguous, 16-B aligned CUDA tensor on this device of at most capacity bytes; all-reduce:
  // SUM / MAX of fp64/fp32/bf16/fp16/int32/int64 or AVG of the floating types; broadcast: any dtype.
  bool supports(const at::Tensor& t, RedOp op, bool bcast = false) const;
  // In-place on stream s (identical sequence of calls on every rank).
  void run(at::Tensor t, RedOp op, int root, bool bcast, hipStream_t s);
  // out [size * in.numel()] <- every rank's in (in within capacity)
  void allgather(at::Tensor out, at::Tensor in, hipStream_t s);
  void allreduce(at::Tensor t, RedOp op, hipStream_t s) { run(t, op, 0, false, s); }
  void broadcast(at::Tensor t, int root, hipStream_t s) { run(t, RedOp::SUM, root, true, s); }
  // 0 = ok; 1 = a peer never arrived within XDDP_PEER_TIMEOUT_MS (synchronizes the device).
  int status();
  void close();
  int64_t capacity() const { return cap_; }

 private:
  void launch(at::Tensor t, at::Tensor out, RedOp op, int root, int mode, hipStream_t s);
  struct Impl;
  int rank_, size_, device_;
  int64_t cap_;
  std::unique_ptr<Impl> impl_;
};

}  // namespace xddp
