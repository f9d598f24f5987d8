// Peer-memory collectives over IPC-mapped staging buffers (xGMI): a one-shot all-reduce /
// broadcast / all-gather for latency-bound small messages and a two-shot (reduce-scatter +
// all-gather) all-reduce for bucket-sized messages. See peer_allreduce.hip for the protocols.
#pragma once

#include <ATen/ATen.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <memory>

#include "common.h"
#include "store/tcp_store.h"

namespace xddp {

constexpr int kPeerMaxRanks = 8;
// Workgroups of a one-shot launch. EVERY launch of a lane runs its full grid (idle workgroups
// only take part in the flag barrier), so each workgroup's call counter — which picks the
// double-buffer slot — advances in lockstep with every other workgroup's.
constexpr int kPeerMaxBlocks = 64;
// Workgroups of a two-shot launch (at most kPeerTwoShotBlocks, XDDP_PEER_TWO_SHOT_BLOCKS; default
// 64 = 8 per XCD): each rank pulls its slice from W - 1 peers concurrently, so the xGMI reads of
// one launch are spread over every link.
constexpr int kPeerTwoShotBlocks = 256;
constexpr int kPeerTwoShotDefaultBlocks = 64;

// Before a rank frees its peer lanes at shutdown: a peer may still be reading this rank's staging
// slot (a two-shot peer gathers the reduced slices after this rank's own kernel has finished), so
// every rank posts "closing" and waits — bounded, a shutdown on an error path is not collective —
// until all ranks have posted it: then no rank runs a peer kernel any more.
inline void peer_quiesce(const std::shared_ptr<Store>& store, int rank, int size, std::chrono::milliseconds timeout) {
  try {
    store->set("peer/closing/" + std::to_string(rank), "1");
    std::vector<std::string> keys;
    for (int r = 0; r < size; ++r) keys.push_back("peer/closing/" + std::to_string(r));
    store->wait(keys, timeout);
  } catch (...) {
  }
}

class PeerAllReduce {
 public:
  // Collective over `size` ranks of one node (all must construct it; IPC handles go through
  // `store`). capacity: largest one-shot message in bytes (a multiple of 4 KiB);
  // two_shot_capacity: staging bytes of the two-shot lane (0 = no two-shot lane; larger
  // messages are walked in chunks of this size). timeout: how long a workgroup waits for a
  // peer before it gives up (XDDP_PEER_TIMEOUT_MS overrides).
  PeerAllReduce(std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity,
                int64_t two_shot_capacity = 0, std::chrono::milliseconds timeout = std::chrono::minutes(10));
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

  // Two-shot all-reduce (SUM / AVG of fp32 / bf16 / fp16, any size: chunks of
  // two_shot_capacity): each rank reduces 1/W of the message from all peers at once, then
  // gathers the other ranks' reduced slices. 2 (W-1)/W * S bytes cross the links per rank.
  bool supports_two_shot(const at::Tensor& t, RedOp op) const;
  void allreduce_two_shot(at::Tensor t, RedOp op, hipStream_t s);

  // 0 = ok; 1 = a peer never arrived within the timeout (the collective's output is invalid and
  // the communicator must be torn down). Host-mapped: reading it never synchronizes the device.
  int status() const;
  void close();
  int64_t capacity() const { return cap_; }
  int64_t two_shot_capacity() const { return cap2_; }
  double timeout_ms() const { return timeout_ms_; }
  // Wait bound of the launches issued from now on (kernel argument: no effect on queued ones).
  void set_timeout_ms(double ms);

 private:
  void launch(at::Tensor t, at::Tensor out, RedOp op, int root, int mode, hipStream_t s);
  struct Impl;
  int rank_, size_, device_;
  int64_t cap_, cap2_;
  double timeout_ms_ = 0;
  std::unique_ptr<Impl> impl_;
};

}  // namespace xddp
