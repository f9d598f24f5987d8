// xddp Reducer: gradient bucketing engine driven by autograd AccumulateGrad post-hooks.
//
// Behavioural contract = the reference stack's c10d::Reducer:
// per-bucket flat buffers with per-parameter views, strictly in-order bucket launch,
// finalize at end of backward via Engine::queue_callback, one rebuild after iteration 0
// in grad-ready order (rank 0's order broadcast), unused-parameter bitmap, static graph,
// no_sync accumulation, gradient_as_bucket_view, a comm-hook slot, prior-reduction and
// marked-twice checks.
//
// MI355X-specific design (not a translation):
//  * grads are gathered into a bucket by ONE multi-tensor HIP launch when the bucket
//    completes (not one `mul_out` per parameter), with the 1/W division folded into the
//    RCCL all-reduce (ncclAvg) and an optional fused cast to a lower comm dtype (bf16);
//  * bucket offsets are padded to 16 elements so every view is 16-B aligned and all
//    pack/unpack kernels take the dwordx4 path;
//  * bucket→grad copy-out is one multi-tensor launch per bucket (or nothing at all with
//    gradient_as_bucket_view).
#pragma once

#include <ATen/ATen.h>
#include <torch/csrc/autograd/function.h>

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "comm/comm.h"

namespace xddp {

// What a comm hook sees (c10d::GradBucket analogue).
struct GradBucket {
  int64_t index = 0;
  int64_t bucket_count = 0;
  at::Tensor buffer;                 // flat buffer to communicate (comm dtype)
  std::vector<int64_t> offsets;      // element offset of each gradient in `buffer`
  std::vector<int64_t> lengths;      // numel of each gradient
  std::vector<std::vector<int64_t>> sizes;
  std::vector<at::Tensor> gradients; // views into `buffer`, shaped like the params
  std::vector<at::Tensor> parameters;
  bool is_last() const { return index == bucket_count - 1; }
};

// Result handle of a (Python or native) comm hook.
struct HookResult {
  virtual ~HookResult() = default;
  virtual at::Tensor wait() = 0;
};
using CommHookFn = std::function<std::shared_ptr<HookResult>(std::shared_ptr<GradBucket>)>;

struct ReducerOptions {
  bool find_unused_parameters = false;
  bool gradient_as_bucket_view = false;
  bool static_graph = false;
  int64_t bucket_bytes_cap = 25 * 1024 * 1024;
  int64_t first_bucket_bytes_cap = 1024 * 1024;
  // Dtype gradients are communicated in (kUndefined = same as the param).
  at::ScalarType comm_dtype = at::ScalarType::Undefined;
  // With find_unused_parameters: a bucket whose parameters were all unused this iteration is
  // not all-reduced (caller guarantees the unused set is identical on every rank).
  bool skip_all_reduce_unused_params = false;
  // xGMI tail policy (0 = off): after the rebuild, the LAST-launched bucket holds only the
  // trailing gradients up to this many bytes, so the all-reduce left exposed after backward
  // (the one that cannot overlap anything) is short. See parallel/bucket_policy.py.
  int64_t tail_bucket_bytes_cap = 0;
  // Per-parameter: gradient is sparse (nn.Embedding(sparse=True)). Such a parameter gets a
  // bucket of its own and is reduced by an all-gather of (indices, values) at finalize.
  std::vector<bool> expect_sparse;
};

class Reducer : public std::enable_shared_from_this<Reducer> {
 public:
  Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> bucket_indices,
          std::vector<int64_t> per_bucket_size_limits, std::shared_ptr<Comm> comm, ReducerOptions opts,
          std::vector<std::string> param_names);
  ~Reducer();

  // Must be called once after construction (needs shared_from_this for hook lifetimes).
  void install_hooks();
  void remove_autograd_hooks();

  void prepare_for_forward();
  void prepare_for_backward(const std::vector<at::Tensor>& outputs);
  bool should_rebuild_buckets() const;
  bool rebuild_buckets();  // returns true iff a rebuild happened

  void set_comm_hook(CommHookFn fn);
  bool has_comm_hook() const { return static_cast<bool>(hook_); }
  void set_comm_dtype(at::ScalarType t);
  void set_static_graph();
  // Join(divide_by_initial_world_size=False): divide by the number of ranks still training,
  // for the NEXT backward only (reset at every finalize, like the reference's div_factor_).
  void set_gradient_divide_factor(double f) { divide_factor_ = f; }
  void set_comm(std::shared_ptr<Comm> c) { comm_ = std::move(c); }
  void set_runtime_logging_sample_rate(int64_t r) { sample_rate_ = std::max<int64_t>(1, r); }

  // Join support: zero buffers shaped like each bucket, used to shadow all-reduces.
  std::vector<at::Tensor> zeros_like_buckets() const;
  // Join support: all-reduce a zero buffer per bucket with the SAME op the training ranks use
  // (AVG, or PREMUL_SUM when `premul_sum`), one RCCL group; returns when the device is done.
  void shadow_allreduce_buckets(bool premul_sum);
  // Join support (reference `_push_all_rebuilt_params`): a rank that joined before finishing an
  // iteration has no grad-ready order; seed it so it still takes part in the rebuild broadcast.
  void push_all_rebuilt_params();
  void reset_runtime_stats();
  void install_post_backward_futures(std::vector<std::shared_ptr<HookResult>> futs);
  at::Tensor local_used_map() const { return local_used_.clone(); }
  std::vector<std::vector<int64_t>> bucket_indices() const;
  std::vector<int64_t> bucket_sizes_bytes() const;
  // per parameter (constructor order): its view into its bucket's flat gradient buffer
  std::vector<at::Tensor> param_bucket_views() const;
  std::vector<int64_t> grad_ready_order() const { return prev_ready_order_; }
  int64_t num_iterations() const { return num_iterations_; }
  bool finalized() const { return !require_finalize_; }
  bool static_graph() const { return opts_.static_graph; }
  void check_finalized() const;

  // Timing/logging (c10d::Logger analogue); values in ns.
  std::map<std::string, double> runtime_stats() const;
  // Average comm-stream duration (ns) of each bucket's collective over the timed iterations.
  std::vector<double> bucket_comm_times() const;
  std::map<std::string, std::string> construction_data() const;

  // Test hook: number of native multi-tensor launches issued so far.
  int64_t native_launches() const { return native_launches_; }

 private:
  struct Bucket {
    std::vector<int64_t> vars;            // param indices
    std::vector<int64_t> offsets;         // element offsets (padded to 16)
    std::vector<int64_t> lengths;
    at::Tensor flat;                      // grad-dtype buffer holding bucket views
    at::Tensor comm;                      // comm-dtype buffer (== flat if same dtype)
    std::vector<at::Tensor> views;        // views into flat with param strides
    std::vector<at::Tensor> comm_views;   // views into comm (only when comm != flat)
    int64_t pending = 0;
    int64_t size_limit = 0;
    std::shared_ptr<Work> work;
    std::shared_ptr<HookResult> hook_result;
    std::shared_ptr<GradBucket> grad_bucket;
    bool launched = false;
    bool sparse = false;                  // one sparse-gradient parameter, reduced at finalize
    bool skipped = false;                 // skip_all_reduce_unused_params: not reduced this iter
  };

  void initialize_buckets(const std::vector<std::vector<int64_t>>& indices, const std::vector<int64_t>& limits);
  void autograd_hook(int64_t index);
  void mark_variable_ready(int64_t index);
  void mark_bucket_ready(int64_t b);
  void launch_bucket(int64_t b);
  void launch_bucket_impl(int64_t b);
  void finalize_backward();
  void search_unused_parameters(const std::vector<at::Tensor>& outputs);
  void all_reduce_local_used_map();
  at::Tensor sparse_allreduce(const at::Tensor& grad);
  std::pair<std::vector<std::vector<int64_t>>, std::vector<int64_t>> assign_rebuilt(
      const std::vector<int64_t>& order) const;
  std::vector<std::vector<int64_t>> sync_bucket_indices(std::vector<std::vector<int64_t>> indices,
                                                       std::vector<int64_t>& limits);
  hipStream_t current_stream() const;
  bool on_gpu() const { return device_.is_cuda(); }
  void timer_record(int slot);

  std::vector<at::Tensor> params_;
  std::vector<std::string> names_;
  std::shared_ptr<Comm> comm_;
  ReducerOptions opts_;
  at::Device device_;
  std::vector<std::shared_ptr<torch::autograd::Node>> grad_accs_;
  std::vector<uintptr_t> hook_keys_;
  bool hooks_installed_ = false;

  std::vector<Bucket> buckets_;
  std::vector<std::pair<int64_t, int64_t>> var_loc_;  // param -> (bucket, slot)
  std::vector<int64_t> cur_limits_;
  int64_t next_bucket_ = 0;
  bool expect_hooks_ = false;
  bool require_finalize_ = false;
  bool finalize_queued_ = false;
  bool has_marked_unused_ = false;
  std::vector<char> ready_;
  std::vector<int64_t> unused_;  // locally unused this iteration
  std::vector<char> unused_mask_;
  at::Tensor local_used_;        // int32 CPU bitmap
  CommHookFn hook_;
  std::vector<std::shared_ptr<HookResult>> post_bwd_futs_;
  double divide_factor_ = 0.0;   // 0 => world size (AVG)

  // rebuild
  bool has_rebuilt_ = false;
  std::vector<int64_t> ready_order_;
  std::vector<int64_t> prev_ready_order_;
  std::vector<int64_t> initial_bucket_bytes_;

  // static graph
  bool static_first_iter_done_ = false;
  std::vector<int64_t> hook_count_expected_;
  std::vector<int64_t> hook_count_;

  int64_t num_iterations_ = 0;
  int64_t native_launches_ = 0;
  int64_t grouped_launches_ = 0;
  mutable std::mutex mu_;

  // timers: slots 0 fwd start, 1 bwd compute start, 2 bwd compute end, 3 comm start, 4 comm end
  int64_t sample_rate_ = 100;
  bool timing_this_iter_ = false;
  std::vector<hipEvent_t> gpu_ev_;
  std::vector<int64_t> cpu_ts_;
  bool timing_pending_ = false;
  double sum_fwd_ = 0, sum_bwd_ = 0, sum_comm_ = 0, sum_overlap_ = 0, sum_tail_ = 0;
  int64_t n_timed_ = 0;
  int64_t n_comm_timed_ = 0;          // timed iterations that launched >= 1 collective
  int64_t collectives_launched_ = 0;  // over the timed iterations
  // (launch index, work) awaiting harvest: the collectives of a sampled backward in launch order
  // (= bucket order for the built-in all-reduce)
  std::vector<std::pair<int64_t, std::shared_ptr<Work>>> timed_works_;
  std::vector<double> bucket_comm_sum_;  // ns, per launch index
  void harvest_timings();

  // fault injection (tests of the replica check): XDDP_FAULT_CORRUPT="rank=R,iter=I" adds 1 to the
  // first element of the first dense bucket AFTER its all-reduce completed, on rank R in iteration I
  // — a silent transport / ordering bug that leaves the loss falling and replicas diverging
  int fault_rank_ = -1;
  int64_t fault_iter_ = -1;
  // XDDP_TSAN_CANARY=1 (ThreadSanitizer self-test, tests/test_sanitizers_cpu.py): a counter written
  // by the hook side on another thread (as the autograd engine's device thread runs the hooks of
  // GPU parameters) and by prepare_for_backward, with no lock in common — a real data race the TSan
  // run must report, proving reports from the Reducer's hook path are not suppressed
  bool tsan_canary_ = false;
  int64_t canary_count_ = 0;
  std::thread canary_thread_;
};

// Bucket assignment with the reference stack's semantics: group by
// (dtype, device); a bucket closes once its byte size reaches the current limit, and the
// limit advances through `limits`. Sparse tensors get their own bucket. If tensor_indices
// is empty the buckets are sorted by their smallest index.
std::pair<std::vector<std::vector<int64_t>>, std::vector<int64_t>> compute_bucket_assignment_by_size(
    const std::vector<at::Tensor>& tensors, const std::vector<int64_t>& limits,
    const std::vector<bool>& expect_sparse, const std::vector<int64_t>& tensor_indices);

// Cross-rank param shape check (T9): all-gather the count, broadcast sizes+strides from 0.
void verify_params_across_processes(const std::shared_ptr<Comm>& comm, const std::vector<at::Tensor>& params);

// Broadcast a tensor list from `src` in flattened per-dtype chunks of <= buffer_bytes (T10).
void broadcast_coalesced(const std::shared_ptr<Comm>& comm, std::vector<at::Tensor> tensors, int64_t buffer_bytes,
                         int src);

}  // namespace xddp
