// xddp Reducer implementation. See reducer.h for the contract and the MI355X design notes.
#include "reducer/reducer.h"

#include <cstring>

#include <ATen/hip/HIPContext.h>
#include <ATen/record_function.h>
#include <c10/hip/HIPGuard.h>
#include <roctracer/roctx.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/utils/lambda_post_hook.h>
#include <torch/csrc/autograd/variable.h>

#include <algorithm>
#include <deque>
#include <limits>
#include <sstream>
#include <unordered_set>

#include "kernels/multi_tensor.h"

namespace xddp {

namespace {

// Scoped marker visible in both torch.profiler (RECORD_FUNCTION) and rocprofv3 (roctx range).
struct Range {
  explicit Range(const char* name) { roctxRangePushA(name); }
  ~Range() { roctxRangePop(); }
};

constexpr int64_t kPad = 16;  // element alignment of every gradient slot in a bucket

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

at::Tensor make_view(const at::Tensor& flat, int64_t off, const at::Tensor& p) {
  if (p.is_non_overlapping_and_dense()) return flat.as_strided(p.sizes(), p.strides(), flat.storage_offset() + off);
  return flat.narrow(0, off, p.numel()).view(p.sizes());
}

bool same_layout(const at::Tensor& a, const at::Tensor& b) {
  if (a.numel() <= 1) return true;
  if (a.is_contiguous() && b.is_contiguous()) return true;
  return a.is_non_overlapping_and_dense() && b.is_non_overlapping_and_dense() && a.strides() == b.strides();
}

}  // namespace

// =======================================================================================
// bucket assignment
// =======================================================================================
std::pair<std::vector<std::vector<int64_t>>, std::vector<int64_t>> compute_bucket_assignment_by_size(
    const std::vector<at::Tensor>& tensors, const std::vector<int64_t>& limits,
    const std::vector<bool>& expect_sparse, const std::vector<int64_t>& tensor_indices) {
  TORCH_CHECK(!limits.empty(), "bucket size limits must not be empty");
  // expect_sparse is indexed by tensor index (tensor_indices[i] when given, else i)
  TORCH_CHECK(expect_sparse.empty() || !tensor_indices.empty() || expect_sparse.size() == tensors.size(),
              "expect_sparse length mismatch");
  for (auto ti : tensor_indices)
    TORCH_CHECK(expect_sparse.empty() || (ti >= 0 && ti < (int64_t)expect_sparse.size()),
                "expect_sparse does not cover tensor index ", ti);
  TORCH_CHECK(tensor_indices.empty() || tensor_indices.size() == tensors.size(), "tensor_indices length mismatch");
  struct Acc {
    std::vector<int64_t> idx;
    int64_t bytes = 0;
    int64_t limit = 0;
    size_t limit_pos = 0;
  };
  std::vector<std::pair<std::vector<int64_t>, int64_t>> out;
  std::vector<std::string> key_order;
  std::map<std::string, Acc> accs;
  for (size_t i = 0; i < tensors.size(); ++i) {
    const auto& t = tensors[i];
    const int64_t ti = tensor_indices.empty() ? static_cast<int64_t>(i) : tensor_indices[i];
    if (!expect_sparse.empty() && expect_sparse[ti]) {
      out.push_back({{ti}, 0});
      continue;
    }
    TORCH_CHECK(!t.is_sparse(), "xddp: sparse tensors need expect_sparse_gradient");
    std::string key = std::string(c10::toString(t.scalar_type())) + "@" + t.device().str();
    auto it = accs.find(key);
    if (it == accs.end()) {
      it = accs.emplace(key, Acc{}).first;
      key_order.push_back(key);
    }
    Acc& a = it->second;
    a.idx.push_back(ti);
    a.bytes += t.numel() * t.element_size();
    a.limit = limits[a.limit_pos];
    if (a.bytes >= a.limit) {
      out.push_back({std::move(a.idx), a.limit});
      a.idx.clear();
      a.bytes = 0;
      if (a.limit_pos + 1 < limits.size()) a.limit_pos++;
    }
  }
  for (auto& k : key_order) {
    Acc& a = accs[k];
    if (!a.idx.empty()) out.push_back({std::move(a.idx), a.limit});
  }
  if (tensor_indices.empty()) {
    std::stable_sort(out.begin(), out.end(), [](const auto& x, const auto& y) {
      return *std::min_element(x.first.begin(), x.first.end()) < *std::min_element(y.first.begin(), y.first.end());
    });
  }
  std::vector<std::vector<int64_t>> idx;
  std::vector<int64_t> lim;
  for (auto& o : out) {
    idx.push_back(std::move(o.first));
    lim.push_back(o.second);
  }
  return {idx, lim};
}

// =======================================================================================
// construction / hooks
// =======================================================================================
Reducer::Reducer(std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> bucket_indices,
                 std::vector<int64_t> per_bucket_size_limits, std::shared_ptr<Comm> comm, ReducerOptions opts,
                 std::vector<std::string> param_names)
    : params_(std::move(params)),
      names_(std::move(param_names)),
      comm_(std::move(comm)),
      opts_(opts),
      device_(params_.empty() ? at::Device(at::kCPU) : params_[0].device()) {
  TORCH_CHECK(!params_.empty(), "xddp Reducer: no parameters");
  for (auto& p : params_) {
    TORCH_CHECK(p.requires_grad(), "xddp Reducer: every parameter must require grad");
    TORCH_CHECK(p.device() == device_, "xddp Reducer: all parameters must live on one device (got ", p.device(),
                " and ", device_, ")");
    TORCH_CHECK(!p.is_sparse(), "xddp Reducer: sparse parameters are not supported (sparse GRADIENTS are: "
                                "pass expect_sparse)");
  }
  if (opts_.expect_sparse.size() != params_.size()) opts_.expect_sparse.assign(params_.size(), false);
  if (names_.size() != params_.size()) {
    names_.clear();
    for (size_t i = 0; i < params_.size(); ++i) names_.push_back("param_" + std::to_string(i));
  }
  const size_t n = params_.size();
  ready_.assign(n, 0);
  unused_mask_.assign(n, 0);
  local_used_ = at::zeros({static_cast<int64_t>(n)}, at::kInt);
  hook_count_.assign(n, 0);
  if (per_bucket_size_limits.size() != bucket_indices.size())
    per_bucket_size_limits.assign(bucket_indices.size(), opts_.bucket_bytes_cap);
  initialize_buckets(bucket_indices, per_bucket_size_limits);
  initial_bucket_bytes_ = bucket_sizes_bytes();
  if (on_gpu()) {
    c10::hip::HIPGuard g(device_.index());
    gpu_ev_.resize(5);
    for (auto& e : gpu_ev_) XDDP_HIP_CHECK(hipEventCreate(&e));
  }
  cpu_ts_.assign(5, 0);
  if (const char* f = std::getenv("XDDP_FAULT_CORRUPT")) {
    std::string spec(f);
    auto field = [&](const char* key) -> int64_t {
      const std::string k = std::string(key) + "=";
      const auto pos = spec.find(k);
      return pos == std::string::npos ? -1 : std::atoll(spec.c_str() + pos + k.size());
    };
    fault_rank_ = static_cast<int>(field("rank"));
    fault_iter_ = field("iter");
  }
  const char* c = std::getenv("XDDP_TSAN_CANARY");
  tsan_canary_ = c && std::string(c) == "1";
}

Reducer::~Reducer() {
  if (canary_thread_.joinable()) canary_thread_.join();
  remove_autograd_hooks();
  for (auto e : gpu_ev_) (void)hipEventDestroy(e);
}

void Reducer::install_hooks() {
  if (hooks_installed_) return;
  std::weak_ptr<Reducer> weak = shared_from_this();
  for (size_t i = 0; i < params_.size(); ++i) {
    auto acc = torch::autograd::impl::grad_accumulator(params_[i]);
    TORCH_CHECK(acc, "xddp Reducer: parameter ", names_[i], " has no grad accumulator");
    const int64_t idx = static_cast<int64_t>(i);
    auto key = acc->add_post_hook(std::make_unique<torch::autograd::utils::LambdaPostHook>(
        [weak, idx](const torch::autograd::variable_list& outputs, const torch::autograd::variable_list&) {
          if (auto r = weak.lock()) r->autograd_hook(idx);
          return outputs;
        }));
    grad_accs_.push_back(std::move(acc));
    hook_keys_.push_back(key);
  }
  hooks_installed_ = true;
}

void Reducer::remove_autograd_hooks() {
  if (!hooks_installed_) return;
  for (size_t i = 0; i < grad_accs_.size(); ++i) grad_accs_[i]->del_post_hook(hook_keys_[i]);
  grad_accs_.clear();
  hook_keys_.clear();
  hooks_installed_ = false;
}

void Reducer::initialize_buckets(const std::vector<std::vector<int64_t>>& indices,
                                 const std::vector<int64_t>& limits) {
  const size_t n = params_.size();
  std::vector<char> seen(n, 0);
  buckets_.clear();
  var_loc_.assign(n, {-1, -1});
  cur_limits_ = limits;
  for (size_t b = 0; b < indices.size(); ++b) {
    Bucket bk;
    bk.vars = indices[b];
    TORCH_CHECK(!bk.vars.empty(), "xddp Reducer: empty bucket");
    bool any_sparse = false;
    for (auto v : bk.vars) any_sparse = any_sparse || (v >= 0 && v < (int64_t)n && opts_.expect_sparse[v]);
    if (any_sparse) {
      TORCH_CHECK(bk.vars.size() == 1, "xddp Reducer: a sparse-gradient parameter needs a bucket of its own");
      const int64_t v = bk.vars[0];
      TORCH_CHECK(!seen[v], "xddp Reducer: param ", v, " assigned to two buckets");
      seen[v] = 1;
      bk.sparse = true;
      bk.offsets = {0};
      bk.lengths = {params_[v].numel()};
      bk.pending = 1;
      bk.size_limit = b < limits.size() ? limits[b] : opts_.bucket_bytes_cap;
      var_loc_[v] = {static_cast<int64_t>(b), 0};
      buckets_.push_back(std::move(bk));
      continue;
    }
    const auto dt = params_[bk.vars[0]].scalar_type();
    int64_t off = 0;
    for (size_t s = 0; s < bk.vars.size(); ++s) {
      const int64_t v = bk.vars[s];
      TORCH_CHECK(v >= 0 && v < static_cast<int64_t>(n), "xddp Reducer: bad param index ", v);
      TORCH_CHECK(!seen[v], "xddp Reducer: param ", v, " assigned to two buckets");
      seen[v] = 1;
      TORCH_CHECK(params_[v].scalar_type() == dt, "xddp Reducer: a bucket must hold one dtype");
      bk.offsets.push_back(off);
      bk.lengths.push_back(params_[v].numel());
      off = round_up(off + params_[v].numel(), kPad);
      var_loc_[v] = {static_cast<int64_t>(b), static_cast<int64_t>(s)};
    }
    const int64_t total = std::max<int64_t>(off, kPad);
    auto opt = params_[bk.vars[0]].options().dtype(dt).requires_grad(false);
    bk.flat = at::zeros({total}, opt);
    for (size_t s = 0; s < bk.vars.size(); ++s) bk.views.push_back(make_view(bk.flat, bk.offsets[s], params_[bk.vars[s]]));
    if (opts_.comm_dtype != at::ScalarType::Undefined && opts_.comm_dtype != dt) {
      bk.comm = at::zeros({total}, opt.dtype(opts_.comm_dtype));
      for (size_t s = 0; s < bk.vars.size(); ++s)
        bk.comm_views.push_back(make_view(bk.comm, bk.offsets[s], params_[bk.vars[s]]));
    } else {
      bk.comm = bk.flat;
    }
    bk.pending = static_cast<int64_t>(bk.vars.size());
    bk.size_limit = b < limits.size() ? limits[b] : opts_.bucket_bytes_cap;
    buckets_.push_back(std::move(bk));
  }
  for (size_t i = 0; i < n; ++i) TORCH_CHECK(seen[i], "xddp Reducer: param ", names_[i], " is in no bucket");
  if (opts_.gradient_as_bucket_view) {
    // existing grads move into the bucket so accumulation happens in place from now on
    for (size_t i = 0; i < n; ++i) {
      if (buckets_[var_loc_[i].first].sparse) continue;
      auto& g = params_[i].mutable_grad();
      const auto& view = buckets_[var_loc_[i].first].views[var_loc_[i].second];
      if (g.defined() && !g.is_alias_of(view)) {
        view.copy_(g);
        g = view;
      }
    }
  }
}

void Reducer::set_comm_hook(CommHookFn fn) {
  std::lock_guard<std::mutex> g(mu_);
  TORCH_CHECK(!hook_, "register_comm_hook can only be called once");
  hook_ = std::move(fn);
}

void Reducer::set_comm_dtype(at::ScalarType t) {
  std::lock_guard<std::mutex> g(mu_);
  opts_.comm_dtype = t;
  auto idx = bucket_indices();
  initialize_buckets(idx, cur_limits_);
}

void Reducer::set_static_graph() {
  std::lock_guard<std::mutex> g(mu_);
  TORCH_CHECK(num_iterations_ == 0, "set_static_graph() must be called before the first iteration");
  opts_.static_graph = true;
}

// =======================================================================================
// per-iteration flow
// =======================================================================================
hipStream_t Reducer::current_stream() const {
  return c10::hip::getCurrentHIPStream(device_.index()).stream();
}

void Reducer::timer_record(int slot) {
  if (!timing_this_iter_) return;
  if (on_gpu()) {
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    XDDP_HIP_CHECK(hipStreamIsCapturing(current_stream(), &cap));
    if (cap == hipStreamCaptureStatusActive) {  // no timing inside a HIP-graph capture
      timing_this_iter_ = false;
      return;
    }
    XDDP_HIP_CHECK(hipEventRecord(gpu_ev_[slot], current_stream()));
  } else {
    cpu_ts_[slot] = now_ns();
  }
}

void Reducer::harvest_timings() {
  if (!timing_pending_) return;
  // the collectives' own comm-stream intervals must be complete as well
  for (auto& bw : timed_works_)
    if (bw.second->timing_state() == Work::Timing::kPending) return;
  double fwd, bwd, tail;
  TimeRef bwd_end;
  if (on_gpu()) {
    for (auto e : gpu_ev_)
      if (hipEventQuery(e) != hipSuccess) return;  // not done yet; try next iteration
    float ms[3] = {0, 0, 0};
    (void)hipEventElapsedTime(&ms[0], gpu_ev_[0], gpu_ev_[1]);
    (void)hipEventElapsedTime(&ms[1], gpu_ev_[1], gpu_ev_[2]);
    (void)hipEventElapsedTime(&ms[2], gpu_ev_[2], gpu_ev_[4]);
    fwd = ms[0] * 1e6; bwd = ms[1] * 1e6; tail = std::max(0.f, ms[2]) * 1e6;
    bwd_end.ev = gpu_ev_[2];
  } else {
    fwd = double(cpu_ts_[1] - cpu_ts_[0]);
    bwd = double(cpu_ts_[2] - cpu_ts_[1]);
    tail = std::max<double>(0, double(cpu_ts_[4] - cpu_ts_[2]));
    bwd_end.ns = cpu_ts_[2];
  }
  sum_fwd_ += fwd; sum_bwd_ += bwd;
  n_timed_++;
  // Communication = what the collectives themselves took where they ran (comm-stream events /
  // the CPU backend's worker clock), not an interval on the compute stream. Iterations in which
  // nothing crossed a link (one rank) contribute no comm sample at all.
  int64_t launched = 0;
  double comm = 0, overlap = 0;
  for (auto& bw : timed_works_) {
    auto& w = bw.second;
    if (!w->collective) continue;
    launched++;
    if (w->timing_state() != Work::Timing::kReady) continue;
    const double c = w->comm_ms() * 1e6;
    comm += c;
    overlap += w->comm_ms_before(bwd_end) * 1e6;
    const size_t b = static_cast<size_t>(bw.first);
    if (bucket_comm_sum_.size() <= b) bucket_comm_sum_.resize(b + 1, 0.0);
    bucket_comm_sum_[b] += c;
  }
  timed_works_.clear();
  collectives_launched_ += launched;
  if (launched > 0) {
    sum_comm_ += comm; sum_overlap_ += overlap; sum_tail_ += tail;
    n_comm_timed_++;
  }
  timing_pending_ = false;
}

void Reducer::prepare_for_forward() {
  std::lock_guard<std::mutex> g(mu_);
  if (on_gpu()) {
    // event queries are illegal while the caller's stream is being captured into a HIP graph
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    XDDP_HIP_CHECK(hipStreamIsCapturing(current_stream(), &cap));
    if (cap == hipStreamCaptureStatusActive) {
      num_iterations_++;
      timing_this_iter_ = false;
      return;
    }
  }
  harvest_timings();
  if (!timing_pending_) timed_works_.clear();  // (a backward that raised may have left some)
  num_iterations_++;
  timing_this_iter_ = !timing_pending_ && (num_iterations_ <= 10 || num_iterations_ % sample_rate_ == 0);
  timer_record(0);
}

void Reducer::check_finalized() const {
  TORCH_CHECK(!require_finalize_,
              "Expected to have finished reduction in the prior iteration before starting a new one.");
}

void Reducer::prepare_for_backward(const std::vector<at::Tensor>& outputs) {
  std::lock_guard<std::mutex> g(mu_);
  if (tsan_canary_) canary_count_ += 1;  // races the canary thread's write (never joined before here)
  if (require_finalize_) {
    std::ostringstream os;
    os << "Expected to have finished reduction in the prior iteration before starting a new one. "
          "This error indicates that your module has parameters that were not used in producing loss. "
          "You can enable unused parameter detection by passing find_unused_parameters=True to "
          "DistributedDataParallel, and by making sure all forward outputs participate in calculating loss. "
          "Parameter indices which did not receive grad for rank "
       << comm_->rank() << ":";
    int shown = 0;
    for (size_t i = 0; i < ready_.size(); ++i)
      if (!ready_[i]) os << " " << i;
    os << "\nParameters which did not receive grad for rank " << comm_->rank() << ":";
    for (size_t i = 0; i < ready_.size() && shown < 32; ++i)
      if (!ready_[i]) { os << " " << names_[i]; shown++; }
    TORCH_CHECK(false, os.str());
  }
  timer_record(1);
  expect_hooks_ = true;
  require_finalize_ = true;
  finalize_queued_ = false;
  has_marked_unused_ = false;
  next_bucket_ = 0;
  std::fill(ready_.begin(), ready_.end(), 0);
  std::fill(hook_count_.begin(), hook_count_.end(), 0);
  for (auto& bk : buckets_) {
    bk.pending = static_cast<int64_t>(bk.vars.size());
    bk.work.reset();
    bk.hook_result.reset();
    bk.grad_bucket.reset();
    bk.launched = false;
    bk.skipped = false;
  }
  if (!has_rebuilt_) ready_order_.clear();
  local_used_.zero_();
  for (auto u : unused_) unused_mask_[u] = 0;
  unused_.clear();
  const bool static_first = opts_.static_graph && !static_first_iter_done_;
  if (opts_.find_unused_parameters && !static_first && !opts_.static_graph) search_unused_parameters(outputs);
  if (opts_.static_graph && static_first_iter_done_) {
    for (size_t i = 0; i < params_.size(); ++i)
      if (hook_count_expected_[i] == 0) unused_.push_back(static_cast<int64_t>(i));
  }
  for (auto u : unused_) unused_mask_[u] = 1;
}

void Reducer::search_unused_parameters(const std::vector<at::Tensor>& outputs) {
  std::unordered_set<torch::autograd::Node*> seen;
  std::deque<torch::autograd::Node*> q;
  for (auto& o : outputs) {
    if (!o.defined() || !o.requires_grad()) continue;
    auto fn = o.grad_fn();
    if (fn) {
      if (seen.insert(fn.get()).second) q.push_back(fn.get());
    } else {
      // output is itself a leaf parameter
      auto acc = torch::autograd::impl::try_get_grad_accumulator(o);
      if (acc) seen.insert(acc.get());
    }
  }
  while (!q.empty()) {
    auto* n = q.front();
    q.pop_front();
    for (const auto& e : n->next_edges()) {
      auto* nx = e.function.get();
      if (nx && seen.insert(nx).second) q.push_back(nx);
    }
  }
  for (size_t i = 0; i < grad_accs_.size(); ++i)
    if (!seen.count(grad_accs_[i].get())) unused_.push_back(static_cast<int64_t>(i));
}

void Reducer::autograd_hook(int64_t index) {
  std::lock_guard<std::mutex> g(mu_);
  if (!expect_hooks_) return;  // no_sync(), or a backward not prepared by the DDP forward
  if (tsan_canary_ && !canary_thread_.joinable())
    canary_thread_ = std::thread([this] { canary_count_ += 1; });  // hook-side write, no lock (canary)
  if (opts_.find_unused_parameters || opts_.static_graph) local_used_.data_ptr<int>()[index] = 1;
  const bool static_first = opts_.static_graph && !static_first_iter_done_;
  if (!has_rebuilt_ && (!opts_.find_unused_parameters || opts_.static_graph) &&
      std::find(ready_order_.begin(), ready_order_.end(), index) == ready_order_.end())
    ready_order_.push_back(index);
  if (static_first) {
    // first static-graph iteration: count hook firings, reduce everything at the end
    hook_count_[index]++;
    timer_record(2);
    if (!finalize_queued_) {
      finalize_queued_ = true;
      std::weak_ptr<Reducer> weak = shared_from_this();
      torch::autograd::Engine::get_default_engine().queue_callback([weak] {
        if (auto r = weak.lock()) r->finalize_backward();
      });
    }
    return;
  }
  if (opts_.static_graph) {
    if (++hook_count_[index] < hook_count_expected_[index]) return;
  }
  if (!has_marked_unused_) {
    has_marked_unused_ = true;
    for (auto u : unused_) mark_variable_ready(u);
  }
  mark_variable_ready(index);
}

void Reducer::mark_variable_ready(int64_t index) {
  if (ready_[index]) {
    TORCH_CHECK(false, "Expected to mark a variable ready only once. This error is caused by one of the following "
                       "reasons: 1) Use of a module parameter outside the `forward` function. 2) Reused parameters in "
                       "multiple reentrant backward passes (e.g. activation checkpointing); consider static_graph=True. "
                       "Parameter at index ",
                index, " with name ", names_[index], " has been marked as ready twice.");
  }
  ready_[index] = 1;
  auto loc = var_loc_[index];
  auto& bk = buckets_[loc.first];
  if (--bk.pending == 0) mark_bucket_ready(loc.first);
}

void Reducer::mark_bucket_ready(int64_t b) {
  if (b != next_bucket_) return;  // launch strictly in bucket order (cross-rank determinism)
  const int64_t nb = static_cast<int64_t>(buckets_.size());
  int64_t burst = 0;
  while (next_bucket_ + burst < nb && buckets_[next_bucket_ + burst].pending == 0) burst++;
  // Several buckets ready at once (the tail of backward, iteration 0, static-graph first
  // iteration): one RCCL group, so RCCL schedules the burst as one launch over the links.
  // Not with a Python comm hook (it may block or run non-RCCL work) or a PREMUL_SUM op (its
  // custom reduction op is created and destroyed per call).
  const bool group = burst > 1 && !hook_ && divide_factor_ <= 0.0;
  if (group) comm_->group_start();
  try {
    for (int64_t k = 0; k < burst; ++k) launch_bucket(next_bucket_++);
  } catch (...) {
    if (group) comm_->group_end();
    throw;
  }
  if (group) {
    comm_->group_end();
    grouped_launches_++;
  }
  if (next_bucket_ == static_cast<int64_t>(buckets_.size()) && !finalize_queued_) {
    timer_record(2);
    finalize_queued_ = true;
    std::weak_ptr<Reducer> weak = shared_from_this();
    torch::autograd::Engine::get_default_engine().queue_callback([weak] {
      if (auto r = weak.lock()) r->finalize_backward();
    });
  }
}

void Reducer::launch_bucket(int64_t b) {
  // Comm timing covers exactly the collectives issued for this bucket (the builtin all-reduce, or
  // whatever a comm hook launches for it), tagged with the bucket index: other users of the
  // process group during backward (SyncBN, another DDP model) are never counted, and timing is
  // off again even when the launch throws.
  if (!timing_this_iter_) return launch_bucket_impl(b);
  comm_->set_timing(true);
  try {
    launch_bucket_impl(b);
  } catch (...) {
    comm_->set_timing(false);
    comm_->drain_timed_works();
    throw;
  }
  comm_->set_timing(false);
  for (auto& w : comm_->drain_timed_works()) timed_works_.emplace_back(b, std::move(w));
}

void Reducer::launch_bucket_impl(int64_t b) {
  RECORD_FUNCTION("xddp::reducer::launch_bucket", std::vector<c10::IValue>());
  Range range("xddp::reducer::launch_bucket");
  auto& bk = buckets_[b];
  if (b == 0) timer_record(3);
  if (bk.sparse) {  // reduced at finalize (needs the peers' nnz first)
    bk.launched = true;
    return;
  }
  if (opts_.skip_all_reduce_unused_params && opts_.find_unused_parameters) {
    bool all_unused = true;
    for (auto v : bk.vars) all_unused = all_unused && unused_mask_[v];
    if (all_unused) {
      bk.skipped = true;
      bk.launched = true;
      return;
    }
  }
  const bool cast = !bk.comm.is_same(bk.flat);
  // In view mode grads live in `flat`; otherwise (cast) we pack straight into the comm buffer.
  const bool pack_to_comm = cast && !opts_.gradient_as_bucket_view;
  std::vector<at::Tensor> src, dst, slow_src, slow_dst, zero;
  for (size_t s = 0; s < bk.vars.size(); ++s) {
    auto& p = params_[bk.vars[s]];
    auto& g = p.mutable_grad();
    const auto& view = pack_to_comm ? bk.comm_views[s] : bk.views[s];
    if (!g.defined()) {
      zero.push_back(view);
      continue;
    }
    TORCH_CHECK(!g.is_sparse(), "xddp Reducer: parameter ", names_[bk.vars[s]],
                " produced a sparse gradient but was not declared sparse (expect_sparse)");
    if (!pack_to_comm && g.is_alias_of(bk.views[s])) continue;  // already accumulated in place
    if (same_layout(g, view) && g.scalar_type() == p.scalar_type()) {
      src.push_back(g);
      dst.push_back(view);
    } else {
      slow_src.push_back(g);
      slow_dst.push_back(view);
    }
  }
  for (auto& z : zero) z.zero_();
  if (!src.empty()) {
    if (on_gpu()) {
      kernels::mt_scale_copy(src, dst, 1.0, c10::nullopt, current_stream());
      native_launches_++;
    } else {
      for (size_t i = 0; i < src.size(); ++i) dst[i].copy_(src[i]);
    }
  }
  for (size_t i = 0; i < slow_src.size(); ++i) slow_dst[i].copy_(slow_src[i]);
  if (opts_.gradient_as_bucket_view) {
    for (size_t s = 0; s < bk.vars.size(); ++s) {
      auto& g = params_[bk.vars[s]].mutable_grad();
      if (g.defined() && !g.is_alias_of(bk.views[s])) g = bk.views[s];
    }
  }
  if (cast && !pack_to_comm) {
    if (on_gpu()) {
      kernels::mt_scale_copy({bk.flat}, {bk.comm}, 1.0, c10::nullopt, current_stream());
      native_launches_++;
    } else {
      bk.comm.copy_(bk.flat);
    }
  }
  if (hook_) {
    auto gb = std::make_shared<GradBucket>();
    gb->index = b;
    gb->bucket_count = static_cast<int64_t>(buckets_.size());
    gb->buffer = bk.comm;
    gb->offsets = bk.offsets;
    gb->lengths = bk.lengths;
    for (size_t s = 0; s < bk.vars.size(); ++s) {
      gb->sizes.push_back(params_[bk.vars[s]].sizes().vec());
      gb->gradients.push_back(cast ? bk.comm_views[s] : bk.views[s]);
      gb->parameters.push_back(params_[bk.vars[s]]);
    }
    bk.grad_bucket = gb;
    bk.hook_result = hook_(gb);
  } else if (divide_factor_ > 0.0) {
    bk.work = comm_->allreduce(bk.comm, RedOp::PREMUL_SUM, 1.0 / divide_factor_);
  } else {
    bk.work = comm_->allreduce(bk.comm, RedOp::AVG, 1.0);
  }
  bk.launched = true;
}

void Reducer::all_reduce_local_used_map() {
  // bitmap is tiny; the D2H read below is the one sync find_unused_parameters costs
  at::Tensor m = on_gpu() ? local_used_.to(device_, /*non_blocking=*/false) : local_used_.clone();
  comm_->allreduce(m, RedOp::SUM, 1.0)->wait();
  local_used_.copy_(m.cpu());
}

void Reducer::finalize_backward() {
  RECORD_FUNCTION("xddp::reducer::finalize_backward", std::vector<c10::IValue>());
  Range range("xddp::reducer::finalize_backward");
  std::lock_guard<std::mutex> g(mu_);
  if (!expect_hooks_) return;
  const bool static_first = opts_.static_graph && !static_first_iter_done_;
  if (static_first) {
    // delayed all-reduce of the first static-graph iteration: everything, in bucket order
    hook_count_expected_ = hook_count_;
    static_first_iter_done_ = true;
    for (size_t i = 0; i < params_.size(); ++i)
      if (!ready_[i]) {
        if (std::find(ready_order_.begin(), ready_order_.end(), (int64_t)i) == ready_order_.end())
          ready_order_.push_back(static_cast<int64_t>(i));
        mark_variable_ready(static_cast<int64_t>(i));
      }
  }
  TORCH_CHECK(next_bucket_ == static_cast<int64_t>(buckets_.size()), "xddp Reducer: finalize before all buckets ran");
  const bool use_map = opts_.find_unused_parameters || static_first;
  if (use_map) all_reduce_local_used_map();
  for (auto& bk : buckets_) {
    if (bk.sparse || bk.skipped) continue;
    at::Tensor result;
    if (bk.hook_result) {
      result = bk.hook_result->wait();
      bk.hook_result.reset();
      bk.grad_bucket.reset();
    } else {
      bk.work->wait();
      result = bk.comm;
      bk.work.reset();
    }
    if (result.defined() && !result.is_same(bk.comm)) bk.comm.view(-1).copy_(result.reshape(-1));
  }
  if (fault_rank_ >= 0 && comm_->rank() == fault_rank_ && num_iterations_ == fault_iter_) {
    for (auto& bk : buckets_) {
      if (bk.sparse || bk.skipped) continue;
      bk.comm.view(-1).narrow(0, 0, 1).add_(1.0);  // injected post-all-reduce corruption (one rank)
      break;
    }
  }
  // sparse gradients: all-gather (indices, values), sum, scale (same divide rule as dense)
  for (auto& bk : buckets_) {
    if (!bk.sparse) continue;
    const int64_t v = bk.vars[0];
    if (use_map && local_used_.data_ptr<int>()[v] == 0) continue;
    auto& gr = params_[v].mutable_grad();
    gr = sparse_allreduce(gr.defined() ? gr : at::zeros_like(params_[v]).to_sparse());
  }
  // copy-out
  for (auto& bk : buckets_) {
    if (bk.sparse || bk.skipped) continue;
    const bool cast = !bk.comm.is_same(bk.flat);
    if (cast && opts_.gradient_as_bucket_view) {
      if (on_gpu()) {
        kernels::mt_scale_copy({bk.comm}, {bk.flat}, 1.0, c10::nullopt, current_stream());
        native_launches_++;
      } else {
        bk.flat.copy_(bk.comm);
      }
    }
    std::vector<at::Tensor> src, dst;
    for (size_t s = 0; s < bk.vars.size(); ++s) {
      const int64_t v = bk.vars[s];
      if (use_map && local_used_.data_ptr<int>()[v] == 0) continue;  // globally unused: leave grad untouched
      auto& p = params_[v];
      auto& gr = p.mutable_grad();
      const auto& view = bk.views[s];
      if (opts_.gradient_as_bucket_view) {
        if (!gr.defined() || !gr.is_alias_of(view)) gr = view;
        continue;
      }
      const auto& from = cast ? bk.comm_views[s] : view;
      if (!gr.defined() || gr.is_alias_of(from)) {
        gr = at::empty_strided(p.sizes(), p.strides(), p.options());
      }
      if (same_layout(gr, from) && gr.scalar_type() == p.scalar_type()) {
        src.push_back(from);
        dst.push_back(gr);
      } else {
        gr.copy_(from);
      }
    }
    if (!src.empty()) {
      if (on_gpu()) {
        kernels::mt_scale_copy(src, dst, 1.0, c10::nullopt, current_stream());
        native_launches_++;
      } else {
        for (size_t i = 0; i < src.size(); ++i) dst[i].copy_(src[i]);
      }
    }
  }
  for (auto& f : post_bwd_futs_) f->wait();
  post_bwd_futs_.clear();
  timer_record(4);
  if (timing_this_iter_) timing_pending_ = true;
  timing_this_iter_ = false;
  if (!has_rebuilt_) prev_ready_order_ = ready_order_;
  expect_hooks_ = false;
  require_finalize_ = false;
  finalize_queued_ = false;
  divide_factor_ = 0.0;  // a join-time divide factor applies to one backward only
}

at::Tensor Reducer::sparse_allreduce(const at::Tensor& grad) {
  RECORD_FUNCTION("xddp::reducer::sparse_allreduce", std::vector<c10::IValue>());
  const int W = comm_->size();
  const double scale = 1.0 / (divide_factor_ > 0.0 ? divide_factor_ : static_cast<double>(W));
  auto g = grad.coalesce();
  if (W == 1) return g.mul(scale);
  auto idx = g._indices().contiguous();
  auto val = g._values().contiguous();
  const auto dev = val.device();
  auto lopt = at::TensorOptions().dtype(at::kLong).device(dev);
  auto nnz_all = at::zeros({W}, lopt);
  comm_->allgather(nnz_all, at::full({1}, g._nnz(), lopt))->wait();
  auto nnz_host = nnz_all.cpu();
  const int64_t* nn = nnz_host.data_ptr<int64_t>();
  int64_t maxn = 0;
  for (int r = 0; r < W; ++r) maxn = std::max(maxn, nn[r]);
  if (maxn == 0) return g.mul(scale);
  const int64_t sd = idx.size(0);
  auto dense_shape = val.sizes().vec();
  dense_shape[0] = maxn;
  auto idx_pad = at::zeros({sd, maxn}, idx.options());
  auto val_pad = at::zeros(dense_shape, val.options());
  idx_pad.narrow(1, 0, idx.size(1)).copy_(idx);
  val_pad.narrow(0, 0, val.size(0)).copy_(val);
  auto idx_all = at::empty({W * sd * maxn}, idx.options());
  auto val_all = at::empty({W * val_pad.numel()}, val.options());
  comm_->allgather(idx_all, idx_pad.reshape(-1))->wait();
  comm_->allgather(val_all, val_pad.reshape(-1))->wait();
  std::vector<at::Tensor> is, vs;
  auto idx3 = idx_all.view({W, sd, maxn});
  auto vshape = dense_shape;
  vshape.insert(vshape.begin(), W);
  auto val3 = val_all.view(vshape);
  for (int r = 0; r < W; ++r) {
    if (nn[r] == 0) continue;
    is.push_back(idx3[r].narrow(1, 0, nn[r]));
    vs.push_back(val3[r].narrow(0, 0, nn[r]));
  }
  auto out = at::sparse_coo_tensor(at::cat(is, 1), at::cat(vs, 0), g.sizes(), g.options()).coalesce();
  return out.mul(scale);
}

// =======================================================================================
// rebuild
// =======================================================================================
bool Reducer::should_rebuild_buckets() const {
  // iteration 0 never has a grad-ready order yet; rebuild_buckets() also requires one
  return !has_rebuilt_ && (opts_.static_graph || !opts_.find_unused_parameters);
}

void Reducer::push_all_rebuilt_params() {
  std::lock_guard<std::mutex> g(mu_);
  if (has_rebuilt_ || !prev_ready_order_.empty()) return;
  // no observed order: the reference's heuristic (reverse registration order ~ grad-ready order)
  for (int64_t i = static_cast<int64_t>(params_.size()) - 1; i >= 0; --i) prev_ready_order_.push_back(i);
}

std::pair<std::vector<std::vector<int64_t>>, std::vector<int64_t>> Reducer::assign_rebuilt(
    const std::vector<int64_t>& order) const {
  std::vector<at::Tensor> ordered;
  bool one_dtype = true, any_sparse = false;
  for (auto v : order) {
    ordered.push_back(params_[v]);
    one_dtype = one_dtype && params_[v].scalar_type() == params_[order[0]].scalar_type();
    any_sparse = any_sparse || opts_.expect_sparse[v];
  }
  const std::vector<int64_t> limits = {opts_.first_bucket_bytes_cap, opts_.bucket_bytes_cap};
  if (opts_.tail_bucket_bytes_cap <= 0 || !one_dtype || any_sparse || order.size() < 2)
    return compute_bucket_assignment_by_size(ordered, limits, opts_.expect_sparse, order);
  // tail: the trailing gradients (produced last in backward) up to tail cap form the final bucket
  size_t k = order.size();
  int64_t tail_bytes = 0;
  while (k > 1 && tail_bytes < opts_.tail_bucket_bytes_cap) {
    --k;
    tail_bytes += params_[order[k]].numel() * params_[order[k]].element_size();
  }
  std::vector<at::Tensor> head(ordered.begin(), ordered.begin() + k);
  std::vector<int64_t> head_idx(order.begin(), order.begin() + k);
  auto res = compute_bucket_assignment_by_size(head, limits, opts_.expect_sparse, head_idx);
  res.first.emplace_back(order.begin() + k, order.end());
  res.second.push_back(opts_.tail_bucket_bytes_cap);
  return res;
}

void Reducer::shadow_allreduce_buckets(bool premul_sum) {
  std::vector<at::Tensor> zs;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto& bk : buckets_) {
      TORCH_CHECK(!bk.sparse, "xddp Reducer: join() with sparse-gradient parameters is not supported");
      zs.push_back(at::zeros_like(bk.comm));
    }
  }
  std::vector<std::shared_ptr<Work>> ws;
  if (!premul_sum && zs.size() > 1) comm_->group_start();
  for (auto& z : zs) ws.push_back(comm_->allreduce(z, premul_sum ? RedOp::PREMUL_SUM : RedOp::AVG, 1.0));
  if (!premul_sum && zs.size() > 1) comm_->group_end();
  for (auto& w : ws) w->synchronize();
}

void Reducer::install_post_backward_futures(std::vector<std::shared_ptr<HookResult>> futs) {
  std::lock_guard<std::mutex> g(mu_);
  for (auto& f : futs) post_bwd_futs_.push_back(std::move(f));
}

void Reducer::reset_runtime_stats() {
  std::lock_guard<std::mutex> g(mu_);
  sum_fwd_ = sum_bwd_ = sum_comm_ = sum_overlap_ = sum_tail_ = 0;
  n_timed_ = n_comm_timed_ = collectives_launched_ = 0;
  bucket_comm_sum_.clear();
}

std::vector<double> Reducer::bucket_comm_times() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<double> r(bucket_comm_sum_.size());
  for (size_t b = 0; b < r.size(); ++b) r[b] = n_comm_timed_ ? bucket_comm_sum_[b] / n_comm_timed_ : 0.0;
  return r;
}

std::vector<std::vector<int64_t>> Reducer::sync_bucket_indices(std::vector<std::vector<int64_t>> indices,
                                                               std::vector<int64_t>& limits) {
  const int64_t P = static_cast<int64_t>(params_.size());
  // layout: [nbuckets, counts[P], limits[P], flat indices[P]]
  auto meta = at::zeros({1 + 3 * P}, at::kLong);
  auto* m = meta.data_ptr<int64_t>();
  m[0] = static_cast<int64_t>(indices.size());
  int64_t pos = 1 + 2 * P;
  for (size_t b = 0; b < indices.size(); ++b) {
    m[1 + b] = static_cast<int64_t>(indices[b].size());
    m[1 + P + b] = limits[b];
    for (auto v : indices[b]) m[pos++] = v;
  }
  at::Tensor t = on_gpu() ? meta.to(device_) : meta;
  comm_->broadcast(t, 0)->wait();
  meta = t.cpu();
  m = meta.data_ptr<int64_t>();
  const int64_t nb = m[0];
  std::vector<std::vector<int64_t>> out(nb);
  limits.assign(nb, 0);
  pos = 1 + 2 * P;
  for (int64_t b = 0; b < nb; ++b) {
    limits[b] = m[1 + P + b];
    for (int64_t k = 0; k < m[1 + b]; ++k) out[b].push_back(m[pos++]);
  }
  return out;
}

bool Reducer::rebuild_buckets() {
  RECORD_FUNCTION("xddp::reducer::rebuild_buckets", std::vector<c10::IValue>());
  std::lock_guard<std::mutex> g(mu_);
  if (!should_rebuild_buckets() || prev_ready_order_.empty()) return false;
  TORCH_CHECK(!require_finalize_, "xddp Reducer: cannot rebuild buckets while a reduction is in flight");
  has_rebuilt_ = true;
  if (prev_ready_order_.size() != params_.size()) {
    // some params never produced grads in iteration 0 (possible only with static graph); append them
    std::vector<char> in(params_.size(), 0);
    for (auto v : prev_ready_order_) in[v] = 1;
    for (size_t i = 0; i < params_.size(); ++i)
      if (!in[i]) prev_ready_order_.push_back(static_cast<int64_t>(i));
  }
  auto res = assign_rebuilt(prev_ready_order_);
  auto limits = res.second;
  auto idx = sync_bucket_indices(res.first, limits);
  initialize_buckets(idx, limits);
  bucket_comm_sum_.clear();  // per-bucket comm samples refer to the layout they were taken on
  return true;
}

// =======================================================================================
// introspection
// =======================================================================================
std::vector<at::Tensor> Reducer::zeros_like_buckets() const {
  std::vector<at::Tensor> out;
  for (auto& bk : buckets_)
    if (!bk.sparse) out.push_back(at::zeros_like(bk.comm));
  return out;
}

std::vector<std::vector<int64_t>> Reducer::bucket_indices() const {
  std::vector<std::vector<int64_t>> r;
  for (auto& bk : buckets_) r.push_back(bk.vars);
  return r;
}

std::vector<at::Tensor> Reducer::param_bucket_views() const {
  std::vector<at::Tensor> out(params_.size());
  for (size_t v = 0; v < params_.size() && v < var_loc_.size(); ++v) {
    const auto& loc = var_loc_[v];
    if (loc.first < 0 || loc.first >= static_cast<int64_t>(buckets_.size())) continue;
    const auto& bk = buckets_[loc.first];
    if (loc.second >= 0 && loc.second < static_cast<int64_t>(bk.views.size())) out[v] = bk.views[loc.second];
  }
  return out;
}

std::vector<int64_t> Reducer::bucket_sizes_bytes() const {
  std::vector<int64_t> r;
  for (auto& bk : buckets_) {
    int64_t s = 0;
    for (auto v : bk.vars) s += params_[v].numel() * params_[v].element_size();
    r.push_back(s);
  }
  return r;
}

std::map<std::string, double> Reducer::runtime_stats() const {
  std::map<std::string, double> m;
  const double n = std::max<int64_t>(1, n_timed_);
  m["avg_forward_compute_time"] = sum_fwd_ / n;
  m["avg_backward_compute_time"] = sum_bwd_ / n;
  // comm fields only from iterations that launched collectives (NaN = never measured; Python
  // reports it as null): at one rank every collective is a local identity
  const double nan = std::numeric_limits<double>::quiet_NaN();
  const double nc = static_cast<double>(n_comm_timed_);
  m["avg_backward_comm_time"] = n_comm_timed_ ? sum_comm_ / nc : nan;
  m["avg_backward_compute_comm_overlap_time"] = n_comm_timed_ ? sum_overlap_ / nc : nan;
  m["avg_backward_exposed_comm_time"] = n_comm_timed_ ? sum_tail_ / nc : nan;
  m["num_comm_timed_iterations"] = nc;
  m["num_collectives_launched"] = static_cast<double>(collectives_launched_);
  m["num_timed_iterations"] = static_cast<double>(n_timed_);
  m["iteration"] = static_cast<double>(num_iterations_);
  m["num_native_launches"] = static_cast<double>(native_launches_);
  m["num_grouped_launches"] = static_cast<double>(grouped_launches_);
  return m;
}

std::map<std::string, std::string> Reducer::construction_data() const {
  auto join = [](const std::vector<int64_t>& v) {
    std::ostringstream os;
    for (size_t i = 0; i < v.size(); ++i) os << (i ? ", " : "") << v[i];
    return os.str();
  };
  std::map<std::string, std::string> m;
  m["backend_name"] = comm_->backend();
  m["world_size"] = std::to_string(comm_->size());
  m["rank"] = std::to_string(comm_->rank());
  m["bucket_sizes"] = join(initial_bucket_bytes_);
  m["find_unused_parameters"] = opts_.find_unused_parameters ? "1" : "0";
  m["gradient_as_bucket_view"] = opts_.gradient_as_bucket_view ? "1" : "0";
  m["static_graph"] = opts_.static_graph ? "1" : "0";
  m["bucket_cap_bytes"] = std::to_string(opts_.bucket_bytes_cap);
  m["first_bucket_cap_bytes"] = std::to_string(opts_.first_bucket_bytes_cap);
  m["tail_bucket_cap_bytes"] = std::to_string(opts_.tail_bucket_bytes_cap);
  m["skip_all_reduce_unused_params"] = opts_.skip_all_reduce_unused_params ? "1" : "0";
  m["comm_dtype"] = opts_.comm_dtype == at::ScalarType::Undefined ? "" : c10::toString(opts_.comm_dtype);
  m["has_rebuilt_buckets"] = has_rebuilt_ ? "1" : "0";
  if (has_rebuilt_) {
    m["rebuilt_bucket_sizes"] = join(bucket_sizes_bytes());
    std::ostringstream os;
    auto bi = bucket_indices();
    for (size_t b = 0; b < bi.size(); ++b) os << (b ? " | " : "") << join(bi[b]);
    m["rebuilt_per_bucket_param_indices"] = os.str();
  }
  m["prev_iteration_grad_ready_order_indices"] = join(prev_ready_order_);
  return m;
}

// =======================================================================================
// free functions
// =======================================================================================
void verify_params_across_processes(const std::shared_ptr<Comm>& comm, const std::vector<at::Tensor>& params) {
  const auto dev = params.empty() ? at::Device(at::kCPU) : params[0].device();
  const int W = comm->size();
  auto cnt = at::full({1}, static_cast<int64_t>(params.size()), at::kLong);
  auto all = at::zeros({W}, at::kLong);
  if (dev.is_cuda()) {
    auto c = cnt.to(dev), a = all.to(dev);
    comm->allgather(a, c)->wait();
    all = a.cpu();
  } else {
    comm->allgather(all, cnt)->wait();
  }
  for (int r = 0; r < W; ++r) {
    TORCH_CHECK(all.data_ptr<int64_t>()[r] == static_cast<int64_t>(params.size()),
                "DDP expects the same number of parameters on every rank, but rank ", comm->rank(), " has ",
                params.size(), " while rank ", r, " has ", all.data_ptr<int64_t>()[r]);
  }
  std::vector<int64_t> meta;
  for (auto& p : params) {
    meta.push_back(p.dim());
    for (auto s : p.sizes()) meta.push_back(s);
    for (auto s : p.strides()) meta.push_back(s);
  }
  auto mine = at::tensor(meta, at::kLong);
  auto t = mine.clone();
  if (dev.is_cuda()) {
    auto d = t.to(dev);
    comm->broadcast(d, 0)->wait();
    t = d.cpu();
  } else {
    comm->broadcast(t, 0)->wait();
  }
  // agree on the verdict so every rank raises (not only the ones that differ from rank 0)
  const bool mismatch_local = !at::equal(t, mine);
  auto flag = at::full({1}, mismatch_local ? 1 : 0, at::kInt);
  if (dev.is_cuda()) {
    auto d = flag.to(dev);
    comm->allreduce(d, RedOp::MAX, 1.0)->wait();
    flag = d.cpu();
  } else {
    comm->allreduce(flag, RedOp::MAX, 1.0)->wait();
  }
  if (flag.item<int>() != 0 && !mismatch_local) {
    TORCH_CHECK(false, "DDP expects same model across all ranks, but another rank's parameter sizes/strides differ "
                       "from rank 0 (this rank, ", comm->rank(), ", matches rank 0)");
  }
  if (mismatch_local) {
    // locate first mismatch for a helpful message
    const int64_t* a = mine.data_ptr<int64_t>();
    const int64_t* b = t.data_ptr<int64_t>();
    size_t pos = 0;
    for (size_t i = 0; i < params.size(); ++i) {
      const int64_t d = params[i].dim();
      bool bad = false;
      for (int64_t k = 0; k < 1 + 2 * d; ++k) bad = bad || a[pos + k] != b[pos + k];
      if (bad)
        TORCH_CHECK(false, "DDP expects same model across all ranks, but rank ", comm->rank(), " has parameter ", i,
                    " with sizes/strides ", params[i].sizes(), "/", params[i].strides(),
                    " which differs from rank 0");
      pos += 1 + 2 * d;
    }
    TORCH_CHECK(false, "DDP expects same model across all ranks (parameter metadata mismatch)");
  }
}

void broadcast_coalesced(const std::shared_ptr<Comm>& comm, std::vector<at::Tensor> tensors, int64_t buffer_bytes,
                         int src) {
  // All dtypes travel in ONE byte buffer per <= buffer_bytes chunk (each tensor 16-B aligned
  // inside it): DDP's per-forward BN-buffer sync is one latency-bound broadcast instead of one
  // per dtype. Pack/unpack are single byte-exact multi-tensor kernels on the GPU.
  // one rank, or the fake backend (peers are hallucinated: local values stand for the root's)
  if (tensors.empty() || comm->size() == 1 || comm->backend() == "fake") return;
  size_t i = 0;
  while (i < tensors.size()) {
    std::vector<at::Tensor> chunk, staged;
    std::vector<int64_t> offs;
    int64_t bytes = 0;
    while (i < tensors.size() && (chunk.empty() || bytes + (int64_t)tensors[i].nbytes() <= buffer_bytes)) {
      const auto& t = tensors[i];
      TORCH_CHECK(t.device() == tensors[0].device(), "broadcast_coalesced: tensors on different devices");
      chunk.push_back(t);
      staged.push_back(t.is_non_overlapping_and_dense() ? t : t.contiguous());
      offs.push_back(bytes);
      bytes = round_up(bytes + (int64_t)t.nbytes(), 16);
      ++i;
    }
    const auto dev = chunk[0].device();
    auto flat = at::empty({std::max<int64_t>(bytes, 1)}, at::TensorOptions().dtype(at::kByte).device(dev));
    auto* base = static_cast<char*>(flat.data_ptr());
    const bool gpu = dev.is_cuda();
    std::vector<int64_t> nb;
    for (auto& t : staged) nb.push_back((int64_t)t.nbytes());
    if (comm->rank() == src) {
      if (gpu) {
        std::vector<const void*> s;
        std::vector<void*> d;
        for (size_t k = 0; k < staged.size(); ++k) {
          s.push_back(staged[k].data_ptr());
          d.push_back(base + offs[k]);
        }
        kernels::mt_copy_bytes(s, d, nb, c10::hip::getCurrentHIPStream(dev.index()).stream());
      } else {
        for (size_t k = 0; k < staged.size(); ++k) std::memcpy(base + offs[k], staged[k].data_ptr(), nb[k]);
      }
    }
    comm->broadcast(flat, src)->wait();
    if (comm->rank() != src) {
      if (gpu) {
        std::vector<const void*> s;
        std::vector<void*> d;
        for (size_t k = 0; k < staged.size(); ++k) {
          s.push_back(base + offs[k]);
          d.push_back(staged[k].data_ptr());
        }
        kernels::mt_copy_bytes(s, d, nb, c10::hip::getCurrentHIPStream(dev.index()).stream());
      } else {
        for (size_t k = 0; k < staged.size(); ++k) std::memcpy(staged[k].data_ptr(), base + offs[k], nb[k]);
      }
      at::NoGradGuard ng;
      for (size_t k = 0; k < chunk.size(); ++k)
        if (!staged[k].is_same(chunk[k])) chunk[k].copy_(staged[k]);
    }
  }
}

}  // namespace xddp
