"""Interop: run xddp (native Reducer, kernels) on a ``torch.distributed`` process group.

The reference initializes collectives with ``torch.distributed.init_process_group("nccl")``
(``ref:dpp.py:21``). ``from_torch_process_group()`` wraps such a group — RCCL underneath on
ROCm, or gloo on CPU — in an xddp ``ProcessGroup`` whose native communicator dispatches each
collective to torch (``csrc/comm/py_comm.cpp``). ``DistributedDataParallel`` uses it
automatically when only torch's default group exists, so swapping the DDP import is enough.
The native RCCL communicator (``init_process_group`` from this package) stays the fast path.
"""
from __future__ import annotations

from datetime import timedelta

import torch

from .._native import load

_OPS = {0: "SUM", 1: "AVG", 2: "PRODUCT", 3: "MIN", 4: "MAX", 5: "BAND", 6: "BOR", 7: "BXOR", 8: "PREMUL_SUM"}


class _TorchCollectives:
    """Python side of the native PyComm: every method returns an object with wait()."""

    def __init__(self, pg):
        import torch.distributed as tdist

        self.tdist, self.pg = tdist, pg
        self.size = tdist.get_world_size(pg)

    def _op(self, code):
        name = _OPS[code]
        if name == "AVG" and self.tdist.get_backend(self.pg) == "gloo":
            return None  # gloo has no AVG: SUM then divide (handled by the caller below)
        if name == "PREMUL_SUM":
            return None
        return getattr(self.tdist.ReduceOp, name)

    def allreduce(self, t, code, premul):
        op = self._op(code)
        if op is None:
            if _OPS[code] == "PREMUL_SUM":
                t.mul_(premul)
            w = self.tdist.all_reduce(t, op=self.tdist.ReduceOp.SUM, group=self.pg, async_op=True)
            if _OPS[code] == "AVG":
                return _Post(w, lambda: t.div_(self.size))
            return w
        return self.tdist.all_reduce(t, op=op, group=self.pg, async_op=True)

    def broadcast(self, t, root):
        return self.tdist.broadcast(t, self.tdist.get_global_rank(self.pg, root) if self.pg is not None else root,
                                    group=self.pg, async_op=True)

    def allgather(self, out, inp):
        return self.tdist.all_gather_into_tensor(out, inp, group=self.pg, async_op=True)

    def reduce_scatter(self, out, inp, code):
        return self.tdist.reduce_scatter_tensor(out, inp, op=self._op(code) or self.tdist.ReduceOp.SUM,
                                                group=self.pg, async_op=True)

    def alltoall(self, out, inp):
        return self.tdist.all_to_all_single(out, inp, group=self.pg, async_op=True)

    def send(self, t, dst):
        return self.tdist.isend(t, dst, group=self.pg)

    def recv(self, t, src):
        return self.tdist.irecv(t, src, group=self.pg)

    def barrier(self):
        return self.tdist.barrier(group=self.pg, async_op=True)


class _Post:
    def __init__(self, w, fn):
        self.w, self.fn, self.done = w, fn, False

    def wait(self):
        self.w.wait()
        if not self.done:
            self.done = True
            self.fn()
        return True

    def is_completed(self):
        return self.w.is_completed()


def from_torch_process_group(pg=None):
    """Wrap a torch.distributed process group (default: the default group) as an xddp ProcessGroup."""
    import torch.distributed as tdist

    from .c10d import ProcessGroup

    pg_obj = pg if pg is not None else tdist.group.WORLD
    rank, size = tdist.get_rank(pg), tdist.get_world_size(pg)
    backend = tdist.get_backend(pg)
    comm = load().make_py_comm(_TorchCollectives(pg), rank, size, f"torch:{backend}")
    dev = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    xbackend = "rccl" if backend == "nccl" else "cpu"
    return ProcessGroup(comm, None, rank, size, xbackend, list(range(size)), dev, f"torch:{id(pg_obj)}",
                        timedelta(minutes=30))
