"""Rendezvous: turn an init URL / environment into a native xddp store.

Reference behaviour: ``env://`` reads RANK/WORLD_SIZE and the
*required* MASTER_ADDR/MASTER_PORT; rank 0 hosts the TCP store. Quirk Q1 of the reference
(crash when MASTER_ADDR/PORT are unset) is fixed here: they default to 127.0.0.1 and a port
chosen by the launcher (or 29500).

Under ``torchrun`` the elastic agent already owns a store on MASTER_PORT. Then rank 0 starts
the xddp store on an ephemeral port and publishes its address through the agent's store, so
the two never fight over the port.

``file:///path`` uses the native FileStore (an flock-guarded append-only log on a shared
filesystem); rank/world_size come from the query string or the arguments.
"""
from __future__ import annotations

import os
import socket
from datetime import timedelta
from urllib.parse import urlparse, parse_qs

from .._native import load

DEFAULT_MASTER_PORT = 29500

_bootstrap_gen = 0  # agent-store bootstraps by this process (the address key is scoped to it)


def _is_loopback(host: str) -> bool:
    try:
        return socket.gethostbyname(host).startswith("127.")
    except OSError:
        return False


def advertise_host(master_addr: str) -> str:
    """Address other ranks should use to reach this host (for the CPU backend mesh)."""
    env = os.environ.get("XDDP_SOCKET_HOST")
    if env:
        return env
    if _is_loopback(master_addr):
        return "127.0.0.1"
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect((master_addr, 9))
            return s.getsockname()[0]
    except OSError:
        return "127.0.0.1"


def _agent_store_bootstrap(rank: int, world_size: int, timeout: timedelta):
    """Create the xddp store when running under torchrun (agent owns MASTER_PORT)."""
    import torch.distributed as tdist

    global _bootstrap_gen
    C = load()
    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ["MASTER_PORT"])
    agent = tdist.TCPStore(host, port, is_master=False, timeout=timeout, wait_for_workers=False)
    _bootstrap_gen += 1  # a second init in the same worker must not read the first store's address
    key = (f"xddp/store_addr/{os.environ.get('TORCHELASTIC_RUN_ID', 'run')}/"
           f"{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}/{_bootstrap_gen}")
    if rank == 0:
        store = C.TCPStore("0.0.0.0", 0, True, world_size, timeout.total_seconds(), False)
        agent.set(key, f"{advertise_host(host)}:{store.port}")
    else:
        addr = agent.get(key).decode()
        h, p = addr.rsplit(":", 1)
        store = C.TCPStore(h, int(p), False, world_size, timeout.total_seconds(), False)
    return store


def rendezvous(init_method: str | None, rank: int, world_size: int, timeout: timedelta):
    """Return ``(store, rank, world_size, master_addr)``."""
    C = load()
    url = urlparse(init_method or "env://")
    if url.scheme == "env":
        rank = int(os.environ.get("RANK", rank if rank >= 0 else 0)) if rank < 0 else rank
        world_size = int(os.environ.get("WORLD_SIZE", world_size if world_size > 0 else 1)) if world_size <= 0 else world_size
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True" and "MASTER_PORT" in os.environ:
            return _agent_store_bootstrap(rank, world_size, timeout), rank, world_size, host
        port = int(os.environ.get("MASTER_PORT", DEFAULT_MASTER_PORT))
    elif url.scheme == "tcp":
        q = parse_qs(url.query)
        if rank < 0:
            rank = int(q.get("rank", [0])[0])
        if world_size <= 0:
            world_size = int(q.get("world_size", [1])[0])
        host, port = url.hostname or "127.0.0.1", int(url.port or DEFAULT_MASTER_PORT)
    elif url.scheme == "file":
        q = parse_qs(url.query)
        if rank < 0:
            rank = int(q.get("rank", [os.environ.get("RANK", 0)])[0])
        if world_size <= 0:
            world_size = int(q.get("world_size", [os.environ.get("WORLD_SIZE", 1)])[0])
        if rank < 0 or world_size <= 0 or rank >= world_size:
            raise ValueError(f"invalid rank/world_size: {rank}/{world_size}")
        store = C.FileStore(url.path, world_size, timeout.total_seconds())
        return store, rank, world_size, os.environ.get("MASTER_ADDR", "127.0.0.1")
    else:
        raise ValueError(f"unsupported init_method {init_method!r} (use env://, tcp://host:port or file:///path)")
    if rank < 0 or world_size <= 0 or rank >= world_size:
        raise ValueError(f"invalid rank/world_size: {rank}/{world_size}")
    store = C.TCPStore(host, port, rank == 0, world_size, timeout.total_seconds(), False)
    return store, rank, world_size, host
