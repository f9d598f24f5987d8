// Python bindings of the xddp native layer (module `distributeddataparallel_amd._C`).
#include <c10/hip/HIPStream.h>
#include <pybind11/chrono.h>
#include <pybind11/functional.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include "comm/comm.h"
#include "comm/peer.h"
#include "kernels/multi_tensor.h"
#include "kernels/norm.h"
#include "reducer/reducer.h"
#include "store/tcp_store.h"

namespace py = pybind11;
using namespace xddp;

namespace xddp {
bool install_crash_handler();
std::shared_ptr<Comm> make_fake_comm(int rank, int size);
std::shared_ptr<Store> make_file_store(const std::string& path, int world_size);
std::shared_ptr<Comm> make_py_comm(py::object impl, int rank, int size, const std::string& name);
}

namespace {

at::ScalarType dtype_from_str(const std::string& s) {
  if (s.empty() || s == "none") return at::ScalarType::Undefined;
  if (s == "float32" || s == "float") return at::kFloat;
  if (s == "bfloat16") return at::kBFloat16;
  if (s == "float16" || s == "half") return at::kHalf;
  if (s == "float64" || s == "double") return at::kDouble;
  TORCH_CHECK(false, "unsupported dtype string ", s);
}

hipStream_t stream_of(const at::Tensor& t) {
  return c10::hip::getCurrentHIPStream(t.device().index()).stream();
}

// GIL-safe owner of a Python object referenced from C++ threads.
std::shared_ptr<py::object> hold(py::object o) {
  return std::shared_ptr<py::object>(new py::object(std::move(o)), [](py::object* p) {
    if (Py_IsInitialized()) {
      py::gil_scoped_acquire g;
      delete p;
    }
  });
}

struct PyHookResult : HookResult {
  explicit PyHookResult(py::object f) : fut(hold(std::move(f))) {}
  at::Tensor wait() override {
    py::gil_scoped_acquire g;
    py::object r = fut->attr("wait")();
    if (py::isinstance<py::list>(r) || py::isinstance<py::tuple>(r)) r = r[py::int_(0)];
    return r.cast<at::Tensor>();
  }
  std::shared_ptr<py::object> fut;
};

// A future whose value is not a bucket (buffer comm hooks): only waited on.
struct PyFutureWait : HookResult {
  explicit PyFutureWait(py::object f) : fut(hold(std::move(f))) {}
  at::Tensor wait() override {
    py::gil_scoped_acquire g;
    fut->attr("wait")();
    return at::Tensor();
  }
  std::shared_ptr<py::object> fut;
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "xddp native layer for MI355X (gfx950): store, RCCL/CPU communicators, Reducer, HIP kernels";

  // ---------------------------------------------------------------- store
  py::class_<Store, std::shared_ptr<Store>>(m, "Store")
      .def("set", [](Store& s, const std::string& k, const py::bytes& v) { s.set(k, std::string(v)); },
           py::call_guard<py::gil_scoped_release>())
      .def("set", [](Store& s, const std::string& k, const std::string& v) { s.set(k, v); },
           py::call_guard<py::gil_scoped_release>())
      .def("get", [](Store& s, const std::string& k) {
             std::string v;
             {
               py::gil_scoped_release r;
               v = s.get(k);
             }
             return py::bytes(v);
           })
      .def("add", &Store::add, py::call_guard<py::gil_scoped_release>())
      .def("compare_set", [](Store& s, const std::string& k, const std::string& e, const std::string& d) {
             std::string v;
             {
               py::gil_scoped_release r;
               v = s.compare_set(k, e, d);
             }
             return py::bytes(v);
           })
      .def("check", &Store::check, py::call_guard<py::gil_scoped_release>())
      .def("wait", [](Store& s, const std::vector<std::string>& keys, double timeout_s) {
             s.wait(keys, std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000)));
           }, py::arg("keys"), py::arg("timeout_s") = 1800.0, py::call_guard<py::gil_scoped_release>())
      .def("delete_key", &Store::delete_key, py::call_guard<py::gil_scoped_release>())
      .def("num_keys", &Store::num_keys, py::call_guard<py::gil_scoped_release>())
      .def("append", [](Store& s, const std::string& k, const std::string& v) { s.append(k, v); },
           py::call_guard<py::gil_scoped_release>())
      .def_property("timeout_s", [](Store& s) { return s.timeout.count() / 1000.0; },
                    [](Store& s, double t) { s.timeout = std::chrono::milliseconds(static_cast<int64_t>(t * 1000)); });

  py::class_<TCPStore, Store, std::shared_ptr<TCPStore>>(m, "TCPStore")
      .def(py::init([](const std::string& host, int port, bool is_server, int world_size, double timeout_s,
                       bool wait_for_workers) {
             py::gil_scoped_release r;
             return std::make_shared<TCPStore>(host, port, is_server, world_size,
                                               std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000)),
                                               wait_for_workers);
           }),
           py::arg("host"), py::arg("port"), py::arg("is_server") = false, py::arg("world_size") = -1,
           py::arg("timeout_s") = 1800.0, py::arg("wait_for_workers") = false)
      .def_property_readonly("port", &TCPStore::port)
      .def_property_readonly("host", &TCPStore::host);

  py::class_<PrefixStore, Store, std::shared_ptr<PrefixStore>>(m, "PrefixStore")
      .def(py::init<std::string, std::shared_ptr<Store>>())
      .def_property_readonly("underlying_store", &PrefixStore::base);

  py::class_<HashStore, Store, std::shared_ptr<HashStore>>(m, "HashStore").def(py::init<>());

  m.def("FileStore", [](const std::string& path, int world_size, double timeout_s) {
        auto s = make_file_store(path, world_size);
        s->timeout = std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000));
        return s;
      }, py::arg("path"), py::arg("world_size") = -1, py::arg("timeout_s") = 1800.0,
      "File-backed store on a shared filesystem (file:// rendezvous)");

  py::register_exception<StoreTimeout>(m, "StoreTimeout", PyExc_TimeoutError);

  // ---------------------------------------------------------------- comm
  py::enum_<RedOp>(m, "RedOp")
      .value("SUM", RedOp::SUM)
      .value("AVG", RedOp::AVG)
      .value("PRODUCT", RedOp::PRODUCT)
      .value("MIN", RedOp::MIN)
      .value("MAX", RedOp::MAX)
      .value("BAND", RedOp::BAND)
      .value("BOR", RedOp::BOR)
      .value("BXOR", RedOp::BXOR)
      .value("PREMUL_SUM", RedOp::PREMUL_SUM);

  py::class_<Work, std::shared_ptr<Work>>(m, "Work")
      .def("wait", [](Work& w) { w.wait(); return true; }, py::call_guard<py::gil_scoped_release>())
      .def("is_completed", &Work::is_completed, py::call_guard<py::gil_scoped_release>())
      .def("synchronize", &Work::synchronize, py::call_guard<py::gil_scoped_release>())
      .def("result", &Work::result)
      .def_readonly("seq", &Work::seq)
      .def_readonly("collective", &Work::collective)
      .def("timing_state", [](Work& w) {
        auto s = w.timing_state();
        return s == Work::Timing::kNone ? "none" : (s == Work::Timing::kPending ? "pending" : "ready");
      })
      .def("comm_ms", &Work::comm_ms);

  py::class_<Comm, std::shared_ptr<Comm>>(m, "Comm")
      .def("rank", &Comm::rank)
      .def("size", &Comm::size)
      .def("backend", &Comm::backend)
      .def("allreduce", &Comm::allreduce, py::arg("tensor"), py::arg("op") = RedOp::SUM, py::arg("premul") = 1.0,
           py::call_guard<py::gil_scoped_release>())
      .def("broadcast", &Comm::broadcast, py::call_guard<py::gil_scoped_release>())
      .def("allgather", &Comm::allgather, py::call_guard<py::gil_scoped_release>())
      .def("reduce_scatter", &Comm::reduce_scatter, py::call_guard<py::gil_scoped_release>())
      .def("alltoall", &Comm::alltoall, py::call_guard<py::gil_scoped_release>())
      .def("send", &Comm::send, py::call_guard<py::gil_scoped_release>())
      .def("recv", &Comm::recv, py::call_guard<py::gil_scoped_release>())
      .def("barrier", &Comm::barrier, py::call_guard<py::gil_scoped_release>())
      .def("group_start", &Comm::group_start)
      .def("group_end", &Comm::group_end, py::call_guard<py::gil_scoped_release>())
      .def("abort", &Comm::abort, py::call_guard<py::gil_scoped_release>())
      .def("shutdown", &Comm::shutdown, py::call_guard<py::gil_scoped_release>())
      .def("set_timing", &Comm::set_timing)
      .def("timing", &Comm::timing)
      .def("allreduce_via", &Comm::allreduce_via, py::arg("tensor"), py::arg("op"), py::arg("route"),
           py::call_guard<py::gil_scoped_release>(),
           "All-reduce on a named route: 0 auto, 1 base (RCCL ring / peer one-shot chunks), 2 one-shot, 3 two-shot")
      .def("routes", &Comm::routes)
      .def("one_shot_capacity", &Comm::one_shot_capacity)
      .def("set_route_table", &Comm::set_route_table, py::arg("bounds"), py::arg("routes"))
      .def("route_table", &Comm::route_table)
      .def("peer_status", &Comm::peer_status)
      .def("set_peer_timeout_ms", &Comm::set_peer_timeout_ms)
      .def("finish_peer_probation", &Comm::finish_peer_probation, py::arg("keep"),
           py::call_guard<py::gil_scoped_release>())
      .def("info", &Comm::info)
      .def("flight_records", [](Comm& c) {
        py::list out;
        for (auto& e : c.flight().dump()) {
          py::dict d;
          d["seq"] = e.seq;
          d["op"] = e.op;
          d["numel"] = e.numel;
          d["dtype"] = e.dtype;
          d["t_enqueue_ns"] = e.t_enqueue_ns;
          d["t_done_ns"] = e.t_done_ns;
          d["state"] = e.state;
          out.append(d);
        }
        return out;
      })
      .def("num_collectives", [](Comm& c) { return c.flight().count(); })
      .def("flight_json", [](Comm& c, const std::string& reason) {
            return c.flight().to_json(c.rank(), c.backend(), reason);
          }, py::arg("reason") = "on demand")
      .def("dump_flight", &Comm::dump_flight, py::arg("reason") = "on demand", py::arg("force") = true,
           "Write the flight record JSON to $XDDP_FLIGHT_DUMP_PREFIX<rank>.json; returns the path");

  m.def("make_cpu_comm", [](std::shared_ptr<Store> store, int rank, int size, double timeout_s, const std::string& host) {
        return make_tcp_comm_host(std::move(store), rank, size,
                                  std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000)), host);
      }, py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("timeout_s") = 1800.0,
      py::arg("host") = "127.0.0.1", py::call_guard<py::gil_scoped_release>());
  m.def("make_rccl_comm", [](std::shared_ptr<Store> store, int rank, int size, int device, double timeout_s,
                             bool high_priority) {
        return make_rccl_comm(std::move(store), rank, size, device,
                              std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000)), high_priority);
      }, py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("device"), py::arg("timeout_s") = 600.0,
      py::arg("high_priority") = true, py::call_guard<py::gil_scoped_release>());
  py::class_<PeerAllReduce, std::shared_ptr<PeerAllReduce>>(m, "PeerAllReduce",
      "Peer-memory collectives over IPC-mapped staging buffers (xGMI): one-shot and two-shot all-reduce")
      .def(py::init([](std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity,
                       int64_t two_shot_capacity, double timeout_s) {
             return std::make_shared<PeerAllReduce>(std::move(store), rank, size, device, capacity, two_shot_capacity,
                                                    std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000)));
           }), py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("device"), py::arg("capacity") = 1 << 20,
           py::arg("two_shot_capacity") = 0, py::arg("timeout_s") = 600.0, py::call_guard<py::gil_scoped_release>())
      .def("supports", [](PeerAllReduce& p, const at::Tensor& t, int op, bool bcast) {
             return p.supports(t, static_cast<RedOp>(op), bcast);
           }, py::arg("t"), py::arg("op") = 0, py::arg("bcast") = false)
      .def("supports_two_shot", [](PeerAllReduce& p, const at::Tensor& t, int op) {
             return p.supports_two_shot(t, static_cast<RedOp>(op));
           }, py::arg("t"), py::arg("op") = 0)
      .def("allreduce", [](PeerAllReduce& p, at::Tensor t, int op) {
             p.allreduce(t, static_cast<RedOp>(op), c10::hip::getCurrentHIPStream(t.device().index()).stream());
           }, py::arg("t"), py::arg("op") = 0)
      .def("allreduce_two_shot", [](PeerAllReduce& p, at::Tensor t, int op) {
             p.allreduce_two_shot(t, static_cast<RedOp>(op),
                                  c10::hip::getCurrentHIPStream(t.device().index()).stream());
           }, py::arg("t"), py::arg("op") = 0)
      .def("broadcast", [](PeerAllReduce& p, at::Tensor t, int root) {
             p.broadcast(t, root, c10::hip::getCurrentHIPStream(t.device().index()).stream());
           }, py::arg("t"), py::arg("root") = 0)
      .def("allgather", [](PeerAllReduce& p, at::Tensor out, at::Tensor in) {
             p.allgather(out, in, c10::hip::getCurrentHIPStream(in.device().index()).stream());
           }, py::arg("out"), py::arg("in"))
      .def("status", &PeerAllReduce::status)
      .def("close", &PeerAllReduce::close)
      .def_property_readonly("capacity", &PeerAllReduce::capacity)
      .def_property_readonly("two_shot_capacity", &PeerAllReduce::two_shot_capacity)
      .def_property_readonly("timeout_ms", &PeerAllReduce::timeout_ms);
  m.def("make_peer_comm", [](std::shared_ptr<Store> store, int rank, int size, int device, int64_t capacity,
                             int64_t two_shot_capacity, double timeout_s) {
        return make_peer_comm(std::move(store), rank, size, device, capacity, two_shot_capacity,
                              std::chrono::milliseconds(static_cast<int64_t>(timeout_s * 1000)));
      }, py::arg("store"), py::arg("rank"), py::arg("size"), py::arg("device"), py::arg("capacity") = 16 << 20,
      py::arg("two_shot_capacity") = 64 << 20, py::arg("timeout_s") = 600.0, py::call_guard<py::gil_scoped_release>(),
      "RCCL-free single-node communicator over IPC-mapped peer memory (device tensors)");
  m.def("make_fake_comm", &make_fake_comm, py::arg("rank"), py::arg("size"),
        "Communicator whose collectives complete locally without peers (testing at any world size)");
  m.def("install_crash_handler", &install_crash_handler,
        "Print a native backtrace on fatal signals, then chain to the previous handler");
  m.def("make_py_comm", &make_py_comm, py::arg("impl"), py::arg("rank"), py::arg("size"),
        py::arg("name") = "torch");
  m.def("make_debug_comm", &make_debug_comm, py::arg("inner"), py::arg("fingerprint") = true,
        py::arg("nan_check") = false, py::arg("helper") = nullptr);
  m.def("rccl_version", &rccl_version);
  m.def("rccl_stream_handle", &rccl_stream_handle);

  // ---------------------------------------------------------------- reducer
  py::class_<GradBucket, std::shared_ptr<GradBucket>>(m, "GradBucket")
      .def("index", [](GradBucket& b) { return b.index; })
      .def("buffer", [](GradBucket& b) { return b.buffer; })
      .def("set_buffer", [](GradBucket& b, at::Tensor t) { b.buffer.copy_(t); })
      .def("gradients", [](GradBucket& b) { return b.gradients; })
      .def("parameters", [](GradBucket& b) { return b.parameters; })
      .def("is_last", &GradBucket::is_last)
      .def("offsets", [](GradBucket& b) { return b.offsets; })
      .def("lengths", [](GradBucket& b) { return b.lengths; })
      .def("sizes_list", [](GradBucket& b) { return b.sizes; });

  py::class_<Reducer, std::shared_ptr<Reducer>>(m, "Reducer")
      .def(py::init([](std::vector<at::Tensor> params, std::vector<std::vector<int64_t>> bucket_indices,
                       std::vector<int64_t> limits, std::shared_ptr<Comm> comm, bool find_unused,
                       bool grad_as_view, bool static_graph, int64_t bucket_cap, int64_t first_bucket_cap,
                       const std::string& comm_dtype, std::vector<std::string> names, bool skip_unused,
                       int64_t tail_cap, std::vector<bool> expect_sparse) {
             ReducerOptions o;
             o.skip_all_reduce_unused_params = skip_unused;
             o.tail_bucket_bytes_cap = tail_cap;
             o.expect_sparse = std::move(expect_sparse);
             o.find_unused_parameters = find_unused;
             o.gradient_as_bucket_view = grad_as_view;
             o.static_graph = static_graph;
             o.bucket_bytes_cap = bucket_cap;
             o.first_bucket_bytes_cap = first_bucket_cap;
             o.comm_dtype = dtype_from_str(comm_dtype);
             auto r = std::make_shared<Reducer>(std::move(params), std::move(bucket_indices), std::move(limits),
                                                std::move(comm), o, std::move(names));
             r->install_hooks();
             return r;
           }),
           py::arg("params"), py::arg("bucket_indices"), py::arg("per_bucket_size_limits"), py::arg("comm"),
           py::arg("find_unused_parameters") = false, py::arg("gradient_as_bucket_view") = false,
           py::arg("static_graph") = false, py::arg("bucket_bytes_cap") = 25 * 1024 * 1024,
           py::arg("first_bucket_bytes_cap") = 1024 * 1024, py::arg("comm_dtype") = "",
           py::arg("param_names") = std::vector<std::string>{}, py::arg("skip_all_reduce_unused_params") = false,
           py::arg("tail_bucket_bytes_cap") = 0, py::arg("expect_sparse") = std::vector<bool>{})
      .def("prepare_for_forward", &Reducer::prepare_for_forward, py::call_guard<py::gil_scoped_release>())
      .def("prepare_for_backward", &Reducer::prepare_for_backward, py::call_guard<py::gil_scoped_release>())
      .def("rebuild_buckets", &Reducer::rebuild_buckets, py::call_guard<py::gil_scoped_release>())
      .def("should_rebuild_buckets", &Reducer::should_rebuild_buckets)
      .def("register_comm_hook", [](Reducer& r, py::object state, py::object hook) {
        auto st = hold(std::move(state));
        auto fn = hold(std::move(hook));
        r.set_comm_hook([st, fn](std::shared_ptr<GradBucket> b) -> std::shared_ptr<HookResult> {
          py::gil_scoped_acquire g;
          py::object fut = (*fn)(*st, b);
          return std::make_shared<PyHookResult>(std::move(fut));
        });
      })
      .def("has_comm_hook", &Reducer::has_comm_hook)
      .def("set_comm_dtype", [](Reducer& r, const std::string& d) { r.set_comm_dtype(dtype_from_str(d)); })
      .def("set_static_graph", &Reducer::set_static_graph)
      .def("set_gradient_divide_factor", &Reducer::set_gradient_divide_factor)
      .def("set_comm", &Reducer::set_comm)
      .def("set_runtime_logging_sample_rate", &Reducer::set_runtime_logging_sample_rate)
      .def("zeros_like_buckets", &Reducer::zeros_like_buckets)
      .def("shadow_allreduce_buckets", &Reducer::shadow_allreduce_buckets, py::arg("premul_sum") = false,
           py::call_guard<py::gil_scoped_release>())
      .def("push_all_rebuilt_params", &Reducer::push_all_rebuilt_params)
      .def("install_post_backward_futures", [](Reducer& r, py::list futs) {
            std::vector<std::shared_ptr<HookResult>> v;
            for (auto f : futs) v.push_back(std::make_shared<PyFutureWait>(py::reinterpret_borrow<py::object>(f)));
            r.install_post_backward_futures(std::move(v));
          }, "Futures (e.g. from a buffer comm hook) awaited at the end of the next backward")
      .def("reset_runtime_stats", &Reducer::reset_runtime_stats)
      .def("local_used_map", &Reducer::local_used_map)
      .def("bucket_indices", &Reducer::bucket_indices)
      .def("bucket_sizes_bytes", &Reducer::bucket_sizes_bytes)
      .def("param_bucket_views", &Reducer::param_bucket_views)
      .def("grad_ready_order", &Reducer::grad_ready_order)
      .def("num_iterations", &Reducer::num_iterations)
      .def("finalized", &Reducer::finalized)
      .def("check_finalized", &Reducer::check_finalized)
      .def("static_graph", &Reducer::static_graph)
      .def("runtime_stats", &Reducer::runtime_stats)
      .def("bucket_comm_times", &Reducer::bucket_comm_times)
      .def("construction_data", &Reducer::construction_data)
      .def("native_launches", &Reducer::native_launches)
      .def("remove_autograd_hooks", &Reducer::remove_autograd_hooks)
      .def("reinstall_hooks", [](Reducer& r) {
            r.remove_autograd_hooks();
            r.install_hooks();
          },
          "Drop and re-acquire the parameters' AccumulateGrad nodes (recreated on the current stream "
          "once nothing else holds them) and re-register the hooks");

  m.def("compute_bucket_assignment_by_size", &compute_bucket_assignment_by_size, py::arg("tensors"),
        py::arg("limits"), py::arg("expect_sparse") = std::vector<bool>{},
        py::arg("tensor_indices") = std::vector<int64_t>{});
  m.def("verify_params_across_processes", &verify_params_across_processes, py::call_guard<py::gil_scoped_release>());
  m.def("broadcast_coalesced", &broadcast_coalesced, py::call_guard<py::gil_scoped_release>());

  // ---------------------------------------------------------------- kernels
  m.def("mt_scale_copy", [](const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst, double scale,
                            c10::optional<at::Tensor> scale_t) {
        if (src.empty()) return;
        kernels::mt_scale_copy(src, dst, scale, scale_t, stream_of(src[0]));
      }, py::arg("src"), py::arg("dst"), py::arg("scale") = 1.0, py::arg("scale_tensor") = py::none());
  m.def("mt_pack", [](const std::vector<at::Tensor>& src, at::Tensor flat, const std::vector<int64_t>& offs,
                      double scale) { kernels::mt_pack(src, flat, offs, scale, stream_of(flat)); },
        py::arg("src"), py::arg("flat"), py::arg("offsets"), py::arg("scale") = 1.0);
  m.def("mt_unpack", [](at::Tensor flat, const std::vector<int64_t>& offs, const std::vector<at::Tensor>& dst,
                        double scale) { kernels::mt_unpack(flat, offs, dst, scale, stream_of(flat)); },
        py::arg("flat"), py::arg("offsets"), py::arg("dst"), py::arg("scale") = 1.0);
  m.def("mt_copy_bytes", [](const std::vector<at::Tensor>& src, const std::vector<at::Tensor>& dst) {
        TORCH_CHECK(src.size() == dst.size(), "mt_copy_bytes: list length mismatch");
        if (src.empty()) return;
        std::vector<const void*> s;
        std::vector<void*> d;
        std::vector<int64_t> n;
        for (size_t i = 0; i < src.size(); ++i) {
          TORCH_CHECK(src[i].is_cuda() && dst[i].is_cuda(), "mt_copy_bytes expects device tensors");
          TORCH_CHECK(src[i].is_non_overlapping_and_dense() && dst[i].is_non_overlapping_and_dense() &&
                      src[i].nbytes() == dst[i].nbytes(), "mt_copy_bytes: dense tensors of equal byte size");
          s.push_back(src[i].data_ptr());
          d.push_back(dst[i].data_ptr());
          n.push_back((int64_t)src[i].nbytes());
        }
        kernels::mt_copy_bytes(s, d, n, stream_of(dst[0]));
      }, py::arg("src"), py::arg("dst"), "Bit-exact multi-tensor copy (any dtypes; byte sizes must match)");
  m.def("mt_l2norm", [](const std::vector<at::Tensor>& ts, at::Tensor out, double max_norm) {
        kernels::mt_l2norm(ts, out, max_norm, stream_of(out));
      }, py::arg("tensors"), py::arg("out"), py::arg("max_norm") = 0.0);
  m.def("mt_checksum", [](const std::vector<at::Tensor>& ts) {
        TORCH_CHECK(!ts.empty(), "mt_checksum: empty list");
        return kernels::mt_checksum(ts, stream_of(ts[0]));
      });
  m.def("mt_nonfinite", [](const std::vector<at::Tensor>& ts, at::Tensor out) {
        kernels::mt_nonfinite(ts, out, stream_of(out));
      });
  m.def("fused_sgd", [](const std::vector<at::Tensor>& p, const std::vector<at::Tensor>& g,
                        const std::vector<at::Tensor>& b, double lr, double momentum, double dampening, double wd,
                        bool nesterov, bool maximize, bool first, c10::optional<at::Tensor> gs) {
        if (p.empty()) return;
        kernels::fused_sgd(p, g, b, lr, momentum, dampening, wd, nesterov, maximize, first, gs, stream_of(p[0]));
      }, py::arg("params"), py::arg("grads"), py::arg("momentum_bufs"), py::arg("lr"), py::arg("momentum"),
      py::arg("dampening"), py::arg("weight_decay"), py::arg("nesterov"), py::arg("maximize"),
      py::arg("first_step"), py::arg("grad_scale") = py::none());
  m.def("fused_sgd_master", [](const std::vector<at::Tensor>& p, const std::vector<at::Tensor>& g,
                               const std::vector<at::Tensor>& b, const std::vector<at::Tensor>& q, double lr,
                               double momentum, double dampening, double wd, bool nesterov, bool maximize, bool first,
                               c10::optional<at::Tensor> gs) {
        if (p.empty()) return;
        kernels::fused_sgd_master(p, g, b, q, lr, momentum, dampening, wd, nesterov, maximize, first, gs,
                                  stream_of(p[0]));
      }, py::arg("masters"), py::arg("grads"), py::arg("momentum_bufs"), py::arg("model_params"), py::arg("lr"),
      py::arg("momentum"), py::arg("dampening"), py::arg("weight_decay"), py::arg("nesterov"), py::arg("maximize"),
      py::arg("first_step"), py::arg("grad_scale") = py::none());
  m.def("fused_adam", [](const std::vector<at::Tensor>& p, const std::vector<at::Tensor>& g,
                         const std::vector<at::Tensor>& m1, const std::vector<at::Tensor>& m2,
                         const std::vector<at::Tensor>& masters, double lr, double b1, double b2, double eps,
                         double wd, int64_t step, bool decoupled, bool maximize, c10::optional<at::Tensor> gs) {
        if (p.empty()) return;
        kernels::fused_adam(p, g, m1, m2, masters, lr, b1, b2, eps, wd, step, decoupled, maximize, gs,
                            stream_of(p[0]));
      }, py::arg("params"), py::arg("grads"), py::arg("exp_avgs"), py::arg("exp_avg_sqs"), py::arg("masters"),
      py::arg("lr"), py::arg("beta1"), py::arg("beta2"), py::arg("eps"), py::arg("weight_decay"), py::arg("step"),
      py::arg("decoupled"), py::arg("maximize"), py::arg("grad_scale") = py::none());

  kernels::bind_norm_kernels(m);
}
