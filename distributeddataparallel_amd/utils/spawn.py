"""Process launcher: one process per rank (reference: ``torch.multiprocessing.spawn``,
SURVEY.md §2.2 T1 / §3.1, used by ``ref:dpp.py:62``).

* children run ``fn(rank, *args)`` in a ``spawn`` context, die with their parent
  (``PR_SET_PDEATHSIG``), and report exceptions (formatted traceback text, no pickles of
  foreign objects) through a temp file;
* ``join()`` waits on all sentinels; at the first failure it SIGTERMs the rest, then
  SIGKILLs after a grace period, and raises ``ProcessRaisedException`` /
  ``ProcessExitedException`` naming the failing rank;
* unlike the reference, MASTER_ADDR / MASTER_PORT get defaults (127.0.0.1 + a free port),
  fixing quirk Q1, and each child sees RANK / LOCAL_RANK / WORLD_SIZE.
"""
from __future__ import annotations

import ctypes
import multiprocessing as mp
import multiprocessing.connection
import os
import signal
import socket
import tempfile
import time
import traceback
from typing import Callable, Optional


class ProcessException(Exception):
    def __init__(self, msg: str, error_index: int, pid: int):
        super().__init__(msg)
        self.msg = msg
        self.error_index = error_index
        self.pid = pid


class ProcessRaisedException(ProcessException):
    pass


class ProcessExitedException(ProcessException):
    def __init__(self, msg, error_index, pid, exit_code, signal_name=None):
        super().__init__(msg, error_index, pid)
        self.exit_code = exit_code
        self.signal_name = signal_name


def free_port() -> int:
    return free_ports(1)[0]


def free_ports(n: int) -> list:
    """n distinct free loopback ports: every socket stays bound until all are chosen (consecutive
    single picks can return the same ephemeral port, and two stores then collide on it)."""
    socks = []
    try:
        for _ in range(n):
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            socks.append(s)
            s.bind(("127.0.0.1", 0))
        return [s.getsockname()[1] for s in socks]
    finally:
        for s in socks:
            s.close()


def _set_pdeathsig():
    try:
        libc = ctypes.CDLL("libc.so.6")
        libc.prctl(1, signal.SIGINT)  # PR_SET_PDEATHSIG
    except OSError:
        pass


def _wrap(fn, i, args, error_file, env):
    _set_pdeathsig()
    os.environ.update(env)
    os.environ["RANK"] = str(i)
    os.environ["LOCAL_RANK"] = str(i)
    try:
        fn(i, *args)
    except KeyboardInterrupt:
        pass
    except Exception:
        with open(error_file, "w") as f:
            f.write(traceback.format_exc())
        raise SystemExit(1)


class ProcessContext:
    def __init__(self, processes, error_files):
        self.processes = processes
        self.error_files = error_files
        self.sentinels = {p.sentinel: i for i, p in enumerate(processes)}

    def pids(self):
        return [p.pid for p in self.processes]

    def join(self, timeout: Optional[float] = None, grace_period: float = 5.0) -> bool:
        if not self.sentinels:
            return True
        ready = multiprocessing.connection.wait(list(self.sentinels.keys()), timeout=timeout)
        failed = None
        for s in ready:
            i = self.sentinels.pop(s)
            p = self.processes[i]
            p.join()
            if p.exitcode != 0:
                failed = i
                break
        if failed is None:
            return len(self.sentinels) == 0
        # terminate the rest
        for p in self.processes:
            if p.is_alive():
                p.terminate()
        deadline = time.time() + grace_period
        for p in self.processes:
            p.join(max(0.0, deadline - time.time()))
        for p in self.processes:
            if p.is_alive():
                p.kill()
                p.join()
        p = self.processes[failed]
        ef = self.error_files[failed]
        if os.path.exists(ef) and os.path.getsize(ef) > 0:
            with open(ef) as f:
                tb = f.read()
            raise ProcessRaisedException(f"\n\n-- Process {failed} terminated with the following error:\n{tb}",
                                         failed, p.pid)
        code = p.exitcode
        if code is not None and code < 0:
            name = signal.Signals(-code).name
            raise ProcessExitedException(f"process {failed} terminated with signal {name}", failed, p.pid, code, name)
        raise ProcessExitedException(f"process {failed} terminated with exit code {code}", failed, p.pid, code)


def start_processes(fn: Callable, args=(), nprocs: int = 1, join: bool = True, daemon: bool = False,
                    start_method: str = "spawn", env: Optional[dict] = None):
    ctx = mp.get_context(start_method)
    env = dict(env or {})
    env.setdefault("MASTER_ADDR", os.environ.get("MASTER_ADDR", "127.0.0.1"))
    env.setdefault("MASTER_PORT", os.environ.get("MASTER_PORT", str(free_port())))
    env.setdefault("WORLD_SIZE", str(nprocs))
    env.setdefault("LOCAL_WORLD_SIZE", str(nprocs))
    procs, files = [], []
    for i in range(nprocs):
        fd, path = tempfile.mkstemp(prefix="xddp_err_")
        os.close(fd)
        os.unlink(path)
        p = ctx.Process(target=_wrap, args=(fn, i, args, path, env), daemon=daemon)
        p.start()
        procs.append(p)
        files.append(path)
    pc = ProcessContext(procs, files)
    if not join:
        return pc
    try:
        while not pc.join():
            pass
    finally:
        for f in files:
            if os.path.exists(f):
                os.unlink(f)
    return None


def spawn(fn: Callable, args=(), nprocs: int = 1, join: bool = True, daemon: bool = False,
          start_method: str = "spawn", env: Optional[dict] = None):
    """Run ``fn(rank, *args)`` in ``nprocs`` processes (torch.multiprocessing.spawn parity)."""
    return start_processes(fn, args, nprocs, join, daemon, start_method, env)
