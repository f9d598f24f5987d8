"""Collective front-end: process groups over the native xddp communicators.

API parity with the reference stack's ``torch.distributed`` surface that DDP users touch
(SURVEY.md §2.2 T4): ``init_process_group`` / ``destroy_process_group`` / ``get_rank`` /
``get_world_size`` / ``all_reduce`` / ``broadcast`` / ``all_gather`` / ``reduce_scatter`` /
``all_to_all`` / ``send`` / ``recv`` / ``barrier`` / ``new_group`` and ``ReduceOp``.

Backends (both native C++, see ``csrc/comm``):
  * ``"rccl"`` (alias ``"nccl"``) — RCCL over xGMI, one process per GPU;
  * ``"cpu"``  (alias ``"gloo"``) — TCP ring collectives, used for GPU-free multi-process runs;
  * ``"peer"`` — one-shot collectives over IPC-mapped peer memory (single node, device tensors, no
    RCCL): several ranks may share one GPU.
"""
from __future__ import annotations

import contextlib
import os
import time
import sys
from datetime import timedelta
from typing import List, Optional, Sequence

import torch

from .._native import load
from . import rccl_info
from .rendezvous import advertise_host, rendezvous

__all__ = [
    "ReduceOp", "Backend", "ProcessGroup", "Work", "GroupMember", "init_process_group", "destroy_process_group",
    "is_initialized", "get_rank", "get_world_size", "get_backend", "new_group", "all_reduce", "broadcast",
    "all_gather", "all_gather_into_tensor", "reduce_scatter_tensor", "all_to_all_single", "send", "recv",
    "barrier", "monitored_barrier", "broadcast_object_list", "all_gather_object", "get_default_group",
    "coalescing", "is_available", "get_local_rank",
]

DEFAULT_TIMEOUT = timedelta(minutes=30)
DEFAULT_RCCL_TIMEOUT = timedelta(minutes=10)


def is_available() -> bool:
    return True


class ReduceOp:
    """Reduction ops (values match the native ``RedOp`` enum)."""

    SUM = "SUM"
    AVG = "AVG"
    PRODUCT = "PRODUCT"
    MIN = "MIN"
    MAX = "MAX"
    BAND = "BAND"
    BOR = "BOR"
    BXOR = "BXOR"
    PREMUL_SUM = "PREMUL_SUM"


def _redop(op):
    C = load()
    if isinstance(op, C.RedOp):
        return op
    if op is None:
        return C.RedOp.SUM
    name = op if isinstance(op, str) else getattr(op, "name", str(op)).split(".")[-1]
    return getattr(C.RedOp, name.upper())


class Backend:
    RCCL = "rccl"
    NCCL = "rccl"  # on ROCm, "nccl" *is* RCCL
    CPU = "cpu"
    GLOO = "cpu"
    FAKE = "fake"  # hallucinated collectives (one process posing as rank r of W), for tests

    @staticmethod
    def normalize(name: Optional[str]) -> str:
        if name is None:
            return "rccl" if torch.cuda.is_available() else "cpu"
        n = name.lower()
        if n in ("nccl", "rccl", "cuda", "hip"):
            return "rccl"
        if n in ("gloo", "cpu", "tcp"):
            return "cpu"
        if n == "fake":
            return "fake"
        if n == "peer":
            return "peer"
        raise ValueError(f"unknown backend {name!r}")


class Work:
    """Async handle for one collective (wraps the native Work)."""

    def __init__(self, native, outputs=None, post=None):
        self._w = native
        self._outputs = outputs
        self._post = post
        self._fut = None
        self._done_post = False

    def wait(self, timeout=None):
        """GPU: order the caller's stream after the collective (no host block). CPU: block.
        With ``timeout`` (seconds or timedelta) raise RuntimeError if the collective has not
        completed by then; the collective itself keeps running (it can be waited on again)."""
        if self._w is not None and timeout is not None:
            secs = timeout.total_seconds() if hasattr(timeout, "total_seconds") else float(timeout)
            deadline = time.monotonic() + secs
            delay = 1e-5
            while not self._w.is_completed():
                if time.monotonic() > deadline:
                    raise RuntimeError(f"xddp: Work.wait timed out after {secs:.3f} s (collective seq {self._w.seq})")
                time.sleep(delay)
                delay = min(delay * 2, 5e-3)
        if self._w is not None:
            self._w.wait()
        if self._post is not None and not self._done_post:
            self._done_post = True
            self._post()
        return True

    def is_completed(self) -> bool:
        return self._w is None or self._w.is_completed()

    def is_success(self) -> bool:
        return self.is_completed()

    def synchronize(self):
        if self._w is not None:
            self._w.synchronize()
        if self._post is not None and not self._done_post:
            self._done_post = True
            self._post()

    def result(self):
        return self._outputs if self._outputs is not None else (self._w.result() if self._w is not None else [])

    def get_future(self) -> torch.futures.Future:
        """A future for the collective's result; never blocks the caller.

        GPU (RCCL): completed at once after the caller's current stream has been made to wait
        on the collective's event — consumers that run on that stream (a ``.then`` callback
        launching kernels) are ordered after it, exactly like the reference stack's NCCL
        futures. CPU backend: completed by a completion thread when the collective finishes
        (collectives complete in issue order, so one FIFO thread serves all of them).
        """
        if self._fut is None:
            self._fut = torch.futures.Future()
            gpu = self._w is not None and self._outputs_on_gpu()
            if self._w is None or gpu:
                self.wait()
                self._fut.set_result(self.result())
            else:
                _completer().submit(self)
        return self._fut

    def _outputs_on_gpu(self) -> bool:
        outs = self._outputs if self._outputs is not None else self._w.result()
        return any(isinstance(t, torch.Tensor) and t.is_cuda for t in outs)


class _FutureCompleter:
    """One daemon thread completing CPU-backend futures in issue order."""

    def __init__(self):
        import queue
        import threading

        self.q = queue.Queue()
        self.t = threading.Thread(target=self._run, name="xddp-future-completer", daemon=True)
        self.t.start()

    def submit(self, work: "Work"):
        self.q.put(work)

    def _run(self):
        while True:
            w = self.q.get()
            try:
                w.wait()
                w._fut.set_result(w.result())
            except Exception as e:  # noqa: BLE001 — surfaced through the future
                w._fut.set_exception(e)


_COMPLETER = None


def _completer() -> _FutureCompleter:
    global _COMPLETER
    if _COMPLETER is None:
        _COMPLETER = _FutureCompleter()
    return _COMPLETER


class _GroupMemberSentinel:
    def __repr__(self):
        return "NON_GROUP_MEMBER"


class GroupMember:
    WORLD = None
    NON_GROUP_MEMBER = _GroupMemberSentinel()


class ProcessGroup:
    """A set of ranks sharing one native communicator."""

    def __init__(self, comm, store, rank: int, size: int, backend: str, global_ranks: List[int], device,
                 name: str, timeout: timedelta):
        self.comm = comm
        self.store = store
        self._rank = rank
        self._size = size
        self._backend = backend
        self.global_ranks = list(global_ranks)
        self.device = device
        self.group_name = name
        self.timeout = timeout
        self._coalescing = 0
        self.comm_calibration = None  # distributed/calibrate.py report, once measured

    # torch.distributed.ProcessGroup-style accessors
    def rank(self) -> int:
        return self._rank

    def size(self) -> int:
        return self._size

    def name(self) -> str:
        return self._backend

    @property
    def backend(self) -> str:
        return self._backend

    def __repr__(self):
        return f"ProcessGroup({self._backend}, rank={self._rank}, size={self._size}, name={self.group_name})"

    # -------- collectives (return Work) --------
    def _prep(self, t: torch.Tensor) -> torch.Tensor:
        # the cpu backend stages device tensors through host memory (gloo-style CUDA support)
        if self._backend == "cpu" and t.device.type not in ("cpu", "cuda"):
            raise RuntimeError(f"the cpu backend cannot handle {t.device.type} tensors")
        return t

    def allreduce(self, tensor, op=ReduceOp.SUM, premul: float = 1.0) -> Work:
        t = self._prep(tensor)
        return Work(self.comm.allreduce(t, _redop(op), float(premul)), [tensor])

    def broadcast(self, tensor, src: int = 0) -> Work:
        return Work(self.comm.broadcast(self._prep(tensor), int(src)), [tensor])

    def allgather_into_tensor(self, output, input) -> Work:
        return Work(self.comm.allgather(output, input), [output])

    def reduce_scatter_tensor(self, output, input, op=ReduceOp.SUM) -> Work:
        return Work(self.comm.reduce_scatter(output, input, _redop(op)), [output])

    def alltoall_base(self, output, input) -> Work:
        return Work(self.comm.alltoall(output, input), [output])

    def send(self, tensor, dst: int) -> Work:
        return Work(self.comm.send(tensor, int(dst)), [tensor])

    def recv(self, tensor, src: int) -> Work:
        return Work(self.comm.recv(tensor, int(src)), [tensor])

    def barrier(self) -> Work:
        return Work(self.comm.barrier(), [])

    def flight_records(self):
        return self.comm.flight_records()

    def comm_info(self) -> dict:
        """What the communicator reports about itself: the native backend facts plus, for RCCL at
        W > 1, RCCL's own view parsed from its init log (version, ranks, channels, rings)."""
        out = dict(self.comm.info())
        extra = _comm_info.get(id(self.comm), {})
        out.update(extra)
        if extra.get("rccl_log"):
            out["rccl"] = rccl_info.parse(extra["rccl_log"])
        return out

    def shutdown(self):
        self.comm.shutdown()

    def abort(self):
        self.comm.abort()


class _World:
    def __init__(self):
        self.default_pg: Optional[ProcessGroup] = None
        self.groups: dict = {}
        self.group_count = 0
        self.store = None
        # init generation of this process: every store key of a process group's life is scoped
        # to it, so a second init_process_group over a persistent store (torchrun's agent store,
        # a caller-owned store) never reads the previous generation's RCCL unique id or finds its
        # init barrier already "done". All ranks run the same init/destroy sequence, so they agree.
        self.init_gen = 0


_world = _World()


def _scoped(name: str) -> str:
    return name if _world.init_gen <= 1 else f"gen{_world.init_gen}/{name}"


def _excepthook_prefix(rank: int):
    prev = sys.excepthook

    def hook(tp, val, tb):
        sys.stderr.write(f"[rank{rank}]: ")
        prev(tp, val, tb)

    sys.excepthook = hook


def _device_for(backend: str, device_id):
    if backend not in ("rccl", "peer"):
        return torch.device("cpu")
    if device_id is None:
        local = int(os.environ.get("LOCAL_RANK", "0"))
        n = torch.cuda.device_count()
        device_id = local % max(n, 1)
    if isinstance(device_id, torch.device):
        device_id = device_id.index if device_id.index is not None else 0
    torch.cuda.set_device(int(device_id))
    return torch.device("cuda", int(device_id))


def _make_comm(backend: str, store, rank: int, size: int, device, timeout: timedelta, master_addr: str):
    """Create the native communicator; XDDP_DEBUG=DETAIL / XDDP_NAN_CHECK=1 wrap it in the debug
    communicator (cross-rank collective fingerprints / NaN scan)."""
    C = load()
    info = {}
    if backend == "fake":
        return C.make_fake_comm(rank, size)
    if backend == "rccl":
        hp = os.environ.get("XDDP_COMM_HIGH_PRIORITY", "1") != "0"
        log = rccl_info.prepare(rank, size)  # RCCL's own view of the job (W > 1), parsed after init
        comm = C.make_rccl_comm(store, rank, size, device.index, timeout.total_seconds(), hp)
        info = rccl_info.collect(log)
    elif backend == "peer":  # IPC peer memory, one node, device tensors (csrc/comm/peer_comm.cpp)
        mb = lambda k, d: max(0, int(float(os.environ.get(k, d)) * (1 << 20)) // 4096 * 4096)  # noqa: E731
        # The device-side wait bound of the peer kernels: a rank that died leaves its peers' workgroups
        # spinning until it expires (the peer watchdog learns of the failure from the status word), so
        # it is capped at XDDP_PEER_DEVICE_TIMEOUT_S (default 120 s) rather than the group's 30-minute
        # timeout; XDDP_PEER_TIMEOUT_MS still overrides both.
        dev_to = min(timeout.total_seconds(), float(os.environ.get("XDDP_PEER_DEVICE_TIMEOUT_S", "120")))
        comm = C.make_peer_comm(store, rank, size, device.index, max(mb("XDDP_PEER_CAPACITY_MB", "16"), 4096),
                                mb("XDDP_PEER_TWO_SHOT_MB", "64"), dev_to)
    else:
        comm = C.make_cpu_comm(store, rank, size, timeout.total_seconds(), advertise_host(master_addr))
    detail = os.environ.get("XDDP_DEBUG", os.environ.get("TORCH_DISTRIBUTED_DEBUG", "OFF")).upper() == "DETAIL"
    nan = os.environ.get("XDDP_NAN_CHECK", "0") == "1"
    if detail or nan:
        helper = None
        if detail and backend in ("rccl", "peer"):
            # fingerprints go over a host-side ring on its own store prefix (ProcessGroupWrapper's
            # gloo helper): grouped RCCL launches only run at group_end, so the device
            # communicator cannot carry a check that must finish before the collective is issued
            helper = C.make_cpu_comm(C.PrefixStore("xddp_debug", store), rank, size, timeout.total_seconds(),
                                     advertise_host(master_addr))
        comm = C.make_debug_comm(comm, detail, nan, helper)
    _comm_info[id(comm)] = info
    return comm


_comm_info: dict = {}  # id(native comm) -> facts parsed at creation (RCCL debug log)


def init_process_group(backend: Optional[str] = None, init_method: Optional[str] = None,
                       timeout: Optional[timedelta] = None, world_size: int = -1, rank: int = -1,
                       store=None, group_name: str = "", device_id=None) -> ProcessGroup:
    """Create the default process group (reference: ``dist.init_process_group``).

    Unlike the reference stack the communicator is created eagerly and bound to
    ``device_id`` (default ``LOCAL_RANK``), fixing quirk Q2 (no ``set_device``).
    """
    if _world.default_pg is not None:
        raise RuntimeError("trying to initialize the default process group twice")
    C = load()
    be = Backend.normalize(backend)
    if timeout is None:
        timeout = DEFAULT_RCCL_TIMEOUT if be == "rccl" else DEFAULT_TIMEOUT
    master_addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    if store is None and be == "fake":
        if rank < 0 or world_size <= 0:
            raise ValueError("the fake backend needs explicit rank and world_size")
        store = C.HashStore()
    elif store is None:
        store, rank, world_size, master_addr = rendezvous(init_method, rank, world_size, timeout)
    else:
        if rank < 0 or world_size <= 0:
            raise ValueError("rank and world_size are required when passing a store")
    device = _device_for(be, device_id)
    _world.init_gen += 1
    pstore = C.PrefixStore(_scoped("default_pg"), store)
    comm = _make_comm(be, pstore, rank, world_size, device, timeout, master_addr)
    pg = ProcessGroup(comm, pstore, rank, world_size, be, list(range(world_size)), device,
                      group_name or "default_pg", timeout)
    _world.default_pg = pg
    _world.store = store
    _world.groups[pg.group_name] = pg
    GroupMember.WORLD = pg
    _excepthook_prefix(rank)
    if os.environ.get("XDDP_INIT_BARRIER", "1") == "1" and world_size > 1 and be != "fake":
        # store-based barrier: every rank's communicator is up before returning
        n = store.add(_scoped("xddp/init_barrier"), 1)
        if n == world_size:
            store.set(_scoped("xddp/init_done"), "1")
        store.wait([_scoped("xddp/init_done")], timeout.total_seconds())
    return pg


def is_initialized() -> bool:
    return _world.default_pg is not None


def get_default_group() -> ProcessGroup:
    if _world.default_pg is None:
        raise RuntimeError("Default process group has not been initialized, please call init_process_group")
    return _world.default_pg


def _resolve(group) -> ProcessGroup:
    if group is None or group is GroupMember.WORLD:
        return get_default_group()
    if group is GroupMember.NON_GROUP_MEMBER:
        raise RuntimeError("this rank is not part of the group")
    return group


def destroy_process_group(group=None):
    """Shut down communicators (sub-groups first, then the default group)."""
    if group is None or group is GroupMember.WORLD:
        for name in sorted(_world.groups.keys(), reverse=True):
            pg = _world.groups[name]
            if pg is not _world.default_pg:
                try:
                    pg.shutdown()
                except Exception:
                    pass
        if _world.default_pg is not None:
            try:
                _world.default_pg.shutdown()
            except Exception:
                pass
        _world.groups.clear()
        _world.default_pg = None
        _world.group_count = 0
        _world.store = None
        GroupMember.WORLD = None
    else:
        pg = _resolve(group)
        pg.shutdown()
        _world.groups.pop(pg.group_name, None)


def get_rank(group=None) -> int:
    if group is None and _world.default_pg is None:
        return 0
    if group is GroupMember.NON_GROUP_MEMBER:
        return -1
    return _resolve(group).rank()


def get_world_size(group=None) -> int:
    if group is None and _world.default_pg is None:
        return 1
    if group is GroupMember.NON_GROUP_MEMBER:
        return -1
    return _resolve(group).size()


def get_local_rank() -> int:
    return int(os.environ.get("LOCAL_RANK", "0"))


def get_backend(group=None) -> str:
    return _resolve(group).backend


def new_group(ranks: Optional[Sequence[int]] = None, timeout: Optional[timedelta] = None, backend=None):
    """Create a sub-group. Must be called by every rank of the default group (same order)."""
    C = load()
    world = get_default_group()
    ranks = sorted(range(world.size()) if ranks is None else ranks)
    _world.group_count += 1
    name = f"group_{_world.group_count}"
    be = Backend.normalize(backend) if backend is not None else world.backend
    if world.rank() not in ranks:
        return GroupMember.NON_GROUP_MEMBER
    timeout = timeout or world.timeout
    sub_rank = ranks.index(world.rank())
    store = C.PrefixStore(_scoped(name), _world.store)
    comm = _make_comm(be, store, sub_rank, len(ranks), world.device if be in ("rccl", "peer") else torch.device("cpu"),
                      timeout, os.environ.get("MASTER_ADDR", "127.0.0.1"))
    pg = ProcessGroup(comm, store, sub_rank, len(ranks), be, ranks, world.device, name, timeout)
    _world.groups[name] = pg
    return pg


def get_process_group_ranks(group) -> List[int]:
    return list(_resolve(group).global_ranks)


def _group_rank(pg: ProcessGroup, global_rank: int) -> int:
    if pg is _world.default_pg:
        return global_rank
    return pg.global_ranks.index(global_rank)


# ---------------------------------------------------------------------------------------
# functional collectives
# ---------------------------------------------------------------------------------------
_coalesce_pending: List[tuple] = []  # per open coalescing() block: (its group, blocking works issued inside)


def _ret(work: Work, async_op: bool, pg=None):
    if async_op:
        return work
    for opg, works in reversed(_coalesce_pending):
        if opg is pg:
            # inside coalescing() on this group the collective is only launched when the outermost
            # block closes (one RCCL group launch): the blocking call's wait happens there.
            # Collectives on other groups are not part of that launch and wait as usual.
            works.append(work)
            return None
    if pg is not None and pg.backend == "rccl" and any(opg.backend == "rccl" for opg, _ in _coalesce_pending):
        # ncclGroupStart is per thread, not per communicator: this collective is held back until the
        # open block closes too, but that block's launch does not track it, so it cannot be waited on
        raise RuntimeError("a blocking collective on another RCCL group inside an open coalescing() block "
                           "cannot complete before the block closes; issue it with async_op=True and wait "
                           "after the block, or outside the block")
    work.wait()
    return None


def all_reduce(tensor, op=ReduceOp.SUM, group=None, async_op=False):
    pg = _resolve(group)
    return _ret(pg.allreduce(tensor, op), async_op, pg)


def broadcast(tensor, src=0, group=None, async_op=False):
    pg = _resolve(group)
    return _ret(pg.broadcast(tensor, _group_rank(pg, src)), async_op, pg)


def all_gather_into_tensor(output_tensor, input_tensor, group=None, async_op=False):
    pg = _resolve(group)
    return _ret(pg.allgather_into_tensor(output_tensor, input_tensor), async_op, pg)


def all_gather(tensor_list, tensor, group=None, async_op=False):
    pg = _resolve(group)
    flat = torch.empty((pg.size(),) + tuple(tensor.shape), dtype=tensor.dtype, device=tensor.device)
    src = tensor.contiguous()

    def post():
        for i, t in enumerate(tensor_list):
            t.copy_(flat[i])

    w = pg.allgather_into_tensor(flat, src)
    w._post = post
    w._outputs = tensor_list
    return _ret(w, async_op, pg)


def reduce_scatter_tensor(output, input, op=ReduceOp.SUM, group=None, async_op=False):
    pg = _resolve(group)
    return _ret(pg.reduce_scatter_tensor(output, input, op), async_op, pg)


def all_to_all_single(output, input, output_split_sizes=None, input_split_sizes=None, group=None, async_op=False):
    """All-to-all along dim 0; uneven splits supported.

    Uneven splits ride the equal-split collective (one ``ncclAllToAll`` on RCCL): every chunk
    is padded to the largest split in the group (agreed with one tiny MAX all-reduce), then the
    received chunks are compacted with one gather. Padding costs bandwidth only in proportion to
    the imbalance, and the launch count stays at two collectives whatever W is."""
    pg = _resolve(group)
    if output_split_sizes is None and input_split_sizes is None:
        return _ret(pg.alltoall_base(output, input), async_op, pg)
    W = pg.size()
    n_in, n_out = input.shape[0], output.shape[0]
    ins = list(input_split_sizes) if input_split_sizes is not None else [n_in // W] * W
    outs = list(output_split_sizes) if output_split_sizes is not None else [n_out // W] * W
    if len(ins) != W or len(outs) != W or sum(ins) != n_in or sum(outs) != n_out:
        raise ValueError("split sizes must have one entry per rank and sum to dim 0 of the tensors")
    m = torch.tensor([max(ins + outs)], dtype=torch.int64, device=input.device if pg.backend in ("rccl", "peer") else "cpu")
    pg.allreduce(m, ReduceOp.MAX).wait()
    M = int(m.item())
    row = tuple(input.shape[1:])
    send = torch.zeros((W * M,) + row, dtype=input.dtype, device=input.device)
    src_idx = torch.cat([torch.arange(M * d, M * d + n, device=input.device) for d, n in enumerate(ins)])
    send.index_copy_(0, src_idx, input.contiguous())
    recv = torch.empty_like(send)
    w = pg.alltoall_base(recv, send)
    dst_idx = torch.cat([torch.arange(M * s, M * s + n, device=output.device) for s, n in enumerate(outs)])

    def post():
        output.copy_(recv.index_select(0, dst_idx))

    w._post = post
    w._outputs = [output]
    return _ret(w, async_op, pg)


def send(tensor, dst, group=None):
    pg = _resolve(group)
    pg.send(tensor, _group_rank(pg, dst)).wait()


def recv(tensor, src, group=None):
    pg = _resolve(group)
    pg.recv(tensor, _group_rank(pg, src)).wait()
    return src


def isend(tensor, dst, group=None) -> Work:
    pg = _resolve(group)
    return pg.send(tensor, _group_rank(pg, dst))


def irecv(tensor, src, group=None) -> Work:
    pg = _resolve(group)
    return pg.recv(tensor, _group_rank(pg, src))


def barrier(group=None, async_op=False, device_ids=None):
    pg = _resolve(group)
    return _ret(pg.barrier(), async_op, pg)


def monitored_barrier(group=None, timeout=None, wait_all_ranks=False):
    """Store-based barrier that names the ranks that failed to arrive (CPU-side).

    Every rank keeps its own per-group generation count (all ranks call barriers in the same
    order, so the counts agree): a rank that leaves barrier k early can never rejoin barrier k's
    key. Each rank also marks its own arrival key, so a timeout names the missing ranks (all of
    them with ``wait_all_ranks``, else the first)."""
    import time

    pg = _resolve(group)
    timeout = timeout or pg.timeout
    store = pg.store
    gen = getattr(pg, "_monitored_barrier_gen", 0)
    pg._monitored_barrier_gen = gen + 1
    key = f"monitored_barrier/{gen}"
    store.set(f"{key}/{pg.rank()}", "1")
    store.add(key, 1)
    deadline = time.time() + timeout.total_seconds()
    while store.add(key, 0) < pg.size():
        if time.time() > deadline:
            missing = [r for r in range(pg.size()) if not store.check([f"{key}/{r}"])]
            named = missing if wait_all_ranks else missing[:1]
            raise RuntimeError(f"monitored_barrier timed out after {timeout.total_seconds():.1f} s: "
                               f"{store.add(key, 0)}/{pg.size()} ranks arrived; missing ranks {named}")
        time.sleep(0.005)


@contextlib.contextmanager
def coalescing(group=None):
    """Coalesce the collectives issued inside into one RCCL group launch. Blocking collectives
    issued inside return at once and are waited for when the outermost block closes (the works of
    ``async_op=True`` calls may only be waited on after that)."""
    pg = _resolve(group)
    pg.comm.group_start()
    _coalesce_pending.append((pg, []))
    ok = False
    try:
        yield
        ok = True
    finally:
        _, works = _coalesce_pending.pop()
        pg.comm.group_end()
        outer = next((w for opg, w in reversed(_coalesce_pending) if opg is pg), None)
        if outer is not None:
            outer.extend(works)
        elif ok:
            for w in works:
                w.wait()


def broadcast_object_list(object_list, src=0, group=None, device=None):
    import pickle

    pg = _resolve(group)
    dev = pg.device if pg.backend in ("rccl", "peer") else torch.device("cpu")
    if pg.rank() == _group_rank(pg, src):
        payload = pickle.dumps(list(object_list))
        n = torch.tensor([len(payload)], dtype=torch.long, device=dev)
    else:
        payload = b""
        n = torch.zeros(1, dtype=torch.long, device=dev)
    broadcast(n, src, group)
    size = int(n.item())
    buf = (torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev) if payload
           else torch.zeros(size, dtype=torch.uint8, device=dev))
    broadcast(buf, src, group)
    if pg.rank() != _group_rank(pg, src):
        # our own pickles, produced by the src rank of this job
        objs = pickle.loads(bytes(buf.cpu().numpy()))
        for i, o in enumerate(objs):
            object_list[i] = o


def all_gather_object(object_list, obj, group=None):
    import pickle

    pg = _resolve(group)
    dev = pg.device if pg.backend in ("rccl", "peer") else torch.device("cpu")
    payload = pickle.dumps(obj)
    n = torch.tensor([len(payload)], dtype=torch.long, device=dev)
    sizes = torch.zeros(pg.size(), dtype=torch.long, device=dev)
    all_gather_into_tensor(sizes, n, group)
    mx = int(sizes.max().item())
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    buf[: len(payload)] = torch.frombuffer(bytearray(payload), dtype=torch.uint8).to(dev)
    out = torch.zeros(pg.size() * mx, dtype=torch.uint8, device=dev)
    all_gather_into_tensor(out, buf, group)
    out = out.cpu().view(pg.size(), mx)
    for i in range(pg.size()):
        object_list[i] = pickle.loads(bytes(out[i, : int(sizes[i])].numpy()))
