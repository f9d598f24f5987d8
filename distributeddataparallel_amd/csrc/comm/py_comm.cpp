// Adapter Comm over a Python collective object — lets the native Reducer run on a
// torch.distributed ProcessGroup (interop: a script that keeps torch's
// init_process_group("nccl") and only swaps the DDP class still gets the xddp Reducer).
// Each call takes the GIL and dispatches to the Python adapter
// (distributeddataparallel_amd/distributed/torch_adapter.py), whose methods return an object
// with .wait() (torch's Work semantics: GPU work orders the caller's stream).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <tuple>

#include "comm/comm.h"

namespace py = pybind11;

namespace xddp {

namespace {

std::shared_ptr<py::object> hold_obj(py::object o) {
  return std::shared_ptr<py::object>(new py::object(std::move(o)), [](py::object* p) {
    if (Py_IsInitialized()) {
      py::gil_scoped_acquire g;
      delete p;
    }
  });
}

class PyWork : public Work {
 public:
  explicit PyWork(py::object w) : w_(hold_obj(std::move(w))) {}
  bool is_completed() override {
    py::gil_scoped_acquire g;
    return w_->attr("is_completed")().cast<bool>();
  }
  void wait() override {
    py::gil_scoped_acquire g;
    w_->attr("wait")();
  }

 private:
  std::shared_ptr<py::object> w_;
};

class PyComm : public Comm {
 public:
  PyComm(py::object impl, int rank, int size, std::string name)
      : Comm(rank, size), impl_(hold_obj(std::move(impl))), name_(std::move(name)) {}
  std::string backend() const override { return name_; }

  std::shared_ptr<Work> allreduce(at::Tensor t, RedOp op, double premul) override {
    return call("allreduce", t, std::make_tuple(t, static_cast<int>(op), premul));
  }
  std::shared_ptr<Work> broadcast(at::Tensor t, int root) override {
    return call("broadcast", t, std::make_tuple(t, root));
  }
  std::shared_ptr<Work> allgather(at::Tensor out, at::Tensor in) override {
    return call("allgather", in, std::make_tuple(out, in));
  }
  std::shared_ptr<Work> reduce_scatter(at::Tensor out, at::Tensor in, RedOp op) override {
    return call("reduce_scatter", in, std::make_tuple(out, in, static_cast<int>(op)));
  }
  std::shared_ptr<Work> alltoall(at::Tensor out, at::Tensor in) override {
    return call("alltoall", in, std::make_tuple(out, in));
  }
  std::shared_ptr<Work> send(at::Tensor t, int dst) override { return call("send", t, std::make_tuple(t, dst)); }
  std::shared_ptr<Work> recv(at::Tensor t, int src) override { return call("recv", t, std::make_tuple(t, src)); }
  std::shared_ptr<Work> barrier() override { return call("barrier", at::Tensor(), std::make_tuple()); }

 private:
  // Tensors -> Python objects need the GIL, so the argument tuple is built inside.
  template <typename... A>
  std::shared_ptr<Work> call(const char* fn, const at::Tensor& meta, std::tuple<A...> args) {
    int64_t seq = flight_.record(fn, meta.defined() ? meta.numel() : 0,
                                 meta.defined() ? meta.scalar_type() : at::kByte);
    py::gil_scoped_acquire g;
    py::object w = std::apply([&](auto&&... a) { return impl_->attr(fn)(a...); }, args);
    auto pw = std::make_shared<PyWork>(std::move(w));
    pw->seq = seq;
    pw->collective = size_ > 1;
    flight_.finish(seq, "scheduled");
    return pw;
  }
  std::shared_ptr<py::object> impl_;
  std::string name_;
};

}  // namespace

std::shared_ptr<Comm> make_py_comm(py::object impl, int rank, int size, const std::string& name) {
  return std::make_shared<PyComm>(std::move(impl), rank, size, name);
}

}  // namespace xddp
