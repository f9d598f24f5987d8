"""RCCL's own view of a job, for benchmarks and triage (VERDICT r2 "Next round" #1c).

RCCL has no API for the channel / ring layout it picked, but it logs it at init with
``NCCL_DEBUG=INFO``. For a W > 1 RCCL communicator :func:`prepare` points that log at a private
file (only when the user has not configured ``NCCL_DEBUG`` themselves; ``XDDP_RCCL_INFO=0`` turns
it off), and :func:`collect` / :func:`parse` read back the facts that decide xGMI bandwidth: ranks
and nodes, collective / p2p channel counts, the topology graphs (pattern, channels, bandwidth,
link type) and the ring channel count. The log is re-read on every :func:`parse`, because RCCL
connects its rings lazily at the first collective.
"""
from __future__ import annotations

import os
import re
import tempfile
from typing import Optional

_SET = ("NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE")


def prepare(rank: int, size: int) -> Optional[str]:
    """Route RCCL's INFO log to a file for this process; returns the path (None: not captured).
    RCCL reads these variables once, at its first call in the process; the caller's environment is
    restored by :func:`collect` right after the communicator exists."""
    if size <= 1 or os.environ.get("XDDP_RCCL_INFO", "1") == "0":
        return None
    if os.environ.get("NCCL_DEBUG"):
        path = os.environ.get("NCCL_DEBUG_FILE")
        return path.replace("%p", str(os.getpid())).replace("%h", os.uname().nodename) if path else None
    path = os.path.join(tempfile.gettempdir(), f"xddp_rccl_r{rank}_{os.getpid()}.log")
    prepare.saved = {k: os.environ.get(k) for k in _SET}
    os.environ["NCCL_DEBUG"] = "INFO"
    os.environ["NCCL_DEBUG_SUBSYS"] = "INIT,GRAPH,ENV"
    os.environ["NCCL_DEBUG_FILE"] = path
    return path


prepare.saved = None


def collect(path: Optional[str]) -> dict:
    """Restore the environment :func:`prepare` changed; returns ``{"rccl_log": path}`` (parsed later)."""
    saved, prepare.saved = prepare.saved, None
    if saved:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return {"rccl_log": path} if path else {}


_PATTERNS = {
    "version": re.compile(r"(?:NCCL|RCCL) version[ :]+([0-9][\w.+\-]*)"),
    "comm": re.compile(r"rank (\d+) nRanks (\d+) nNodes (\d+) localRanks (\d+) localRank (\d+)"),
    "channels": re.compile(r"(\d+) coll channels, (?:(\d+) collnet channels, )?(?:(\d+) nvls channels, )?"
                           r"(\d+) p2p channels, (\d+) p2p channels per peer"),
    "graph": re.compile(r"Pattern (\d+), crossNic (\d+), nChannels (\d+), bw ([\d.]+)/([\d.]+), type (\S+)"),
    "ring": re.compile(r"Channel (\d+)/(\d+) :"),
    "env": re.compile(r"(\w+) set by environment to (\S+)"),
    "busid": re.compile(r"busId ([0-9a-fA-F:.]+)"),
}


def parse(path: Optional[str], max_lines: int = 200_000) -> dict:
    """Facts from one RCCL INFO log (missing fields are simply absent)."""
    out: dict = {}
    if not path or not os.path.isfile(path):
        return out
    graphs, env, rings = [], {}, 0
    with open(path, errors="replace") as f:
        for i, line in enumerate(f):
            if i >= max_lines:
                break
            m = _PATTERNS["version"].search(line)
            if m and "version" not in out:
                out["version"] = m.group(1)
            m = _PATTERNS["comm"].search(line)
            if m:
                out.update(rank=int(m.group(1)), nranks=int(m.group(2)), nnodes=int(m.group(3)),
                           local_ranks=int(m.group(4)))
            m = _PATTERNS["channels"].search(line)
            if m:
                out.update(coll_channels=int(m.group(1)), p2p_channels=int(m.group(4)),
                           p2p_channels_per_peer=int(m.group(5)))
            m = _PATTERNS["graph"].search(line)
            if m and len(graphs) < 8:
                graphs.append({"pattern": int(m.group(1)), "n_channels": int(m.group(3)),
                               "bw_intra": float(m.group(4)), "bw_inter": float(m.group(5)), "type": m.group(6)})
            m = _PATTERNS["ring"].search(line)
            if m:
                rings = max(rings, int(m.group(2)))
            m = _PATTERNS["env"].search(line)
            if m and len(env) < 32:
                env[m.group(1)] = m.group(2)
            m = _PATTERNS["busid"].search(line)
            if m and "bus_id" not in out:
                out["bus_id"] = m.group(1)
    if graphs:
        out["graphs"] = graphs
    if rings:
        out["ring_channels"] = rings
    if env:
        out["env"] = env
    return out
