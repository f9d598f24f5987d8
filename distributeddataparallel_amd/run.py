"""``python -m distributeddataparallel_amd.run`` — one-process-per-GPU launcher.

Replaces the reference's ``mp.spawn(train, nprocs=torch.cuda.device_count())``
(``ref:dpp.py:60-65``) with a torchrun-style CLI:

    python -m distributeddataparallel_amd.run --nproc-per-node 8 train.py --epochs 5

* sets RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT
  (defaults 127.0.0.1 and a free port — fixes quirk Q1) and HSA_ENABLE_IPC_MODE_LEGACY=0;
* multi-node: ``--nnodes``/``--node-rank`` with a shared ``--master-addr``;
* kills the whole group on the first failing rank (SIGTERM, then SIGKILL after a grace
  period) and exits with that rank's code;
* ``--max-restarts k`` re-launches the whole group after a failure (simple elastic
  recovery; workers resume from their own checkpoints), exporting XDDP_RESTART_COUNT.
"""
from __future__ import annotations

import argparse
import os
import signal
import subprocess
import sys
import time

from .utils.spawn import free_port


def _parse(argv):
    ap = argparse.ArgumentParser(prog="python -m distributeddataparallel_amd.run")
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=None)
    ap.add_argument("--nnodes", type=int, default=1)
    ap.add_argument("--node-rank", "--node_rank", type=int, default=0)
    ap.add_argument("--master-addr", "--master_addr", default="127.0.0.1")
    ap.add_argument("--master-port", "--master_port", type=int, default=None)
    ap.add_argument("--max-restarts", "--max_restarts", type=int, default=0)
    ap.add_argument("--grace-period", type=float, default=5.0)
    ap.add_argument("-m", "--module", action="store_true", help="run the target as a python module")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def _default_nproc() -> int:
    try:
        import torch

        n = torch.cuda.device_count()
        return n if n > 0 else 1
    except Exception:
        return 1


def _launch_group(a, nproc: int, port: int, restart: int):
    world = nproc * a.nnodes
    procs = []
    for local in range(nproc):
        rank = a.node_rank * nproc + local
        env = dict(os.environ)
        env.update({
            "RANK": str(rank), "LOCAL_RANK": str(local), "WORLD_SIZE": str(world),
            "LOCAL_WORLD_SIZE": str(nproc), "GROUP_RANK": str(a.node_rank),
            "MASTER_ADDR": a.master_addr, "MASTER_PORT": str(port),
            "XDDP_RESTART_COUNT": str(restart), "HSA_ENABLE_IPC_MODE_LEGACY": "0",
        })
        env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        cmd = [sys.executable, "-u"] + (["-m", a.script] if a.module else [a.script]) + list(a.args)
        procs.append(subprocess.Popen(cmd, env=env, start_new_session=True))
    return procs


def _kill(procs, grace: float):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace
    for p in procs:
        try:
            p.wait(max(0.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            pass
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def _monitor(procs, grace: float) -> int:
    """Wait for all ranks; on the first failure kill the rest. Returns the group exit code."""
    try:
        while True:
            alive = False
            for i, p in enumerate(procs):
                rc = p.poll()
                if rc is None:
                    alive = True
                elif rc != 0:
                    sys.stderr.write(f"[xddp.run] local rank {i} (pid {p.pid}) failed with exit code {rc}; "
                                     f"terminating the group\n")
                    _kill(procs, grace)
                    return rc
            if not alive:
                return 0
            time.sleep(0.05)
    except KeyboardInterrupt:
        _kill(procs, grace)
        return 130


def main(argv=None) -> int:
    a = _parse(sys.argv[1:] if argv is None else argv)
    nproc = a.nproc_per_node or _default_nproc()
    port = a.master_port or (free_port() if a.nnodes == 1 else 29500)
    restart = 0
    while True:
        procs = _launch_group(a, nproc, port, restart)
        rc = _monitor(procs, a.grace_period)
        if rc == 0 or restart >= a.max_restarts:
            return rc
        restart += 1
        sys.stderr.write(f"[xddp.run] restarting the group ({restart}/{a.max_restarts})\n")
        if a.nnodes == 1 and a.master_port is None:
            port = free_port()


if __name__ == "__main__":
    sys.exit(main())
