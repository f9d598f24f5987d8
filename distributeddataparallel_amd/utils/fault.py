"""Fault injection for failure-detection tests.

``XDDP_FAULT_INJECT="rank=1,step=3[,mode=exit|raise|hang][,code=13]"`` makes the named rank
fail when its DDP forward counter reaches ``step``: ``exit`` terminates the process with
``code``, ``raise`` raises RuntimeError, ``hang`` sleeps forever (exercises timeouts /
watchdogs / the launcher's kill-all).
"""
from __future__ import annotations

import os
import time

_spec = None
_parsed = False


def _parse():
    global _spec, _parsed
    _parsed = True
    raw = os.environ.get("XDDP_FAULT_INJECT")
    if not raw:
        return
    kv = dict(p.split("=", 1) for p in raw.split(",") if "=" in p)
    _spec = {"rank": int(kv.get("rank", 0)), "step": int(kv.get("step", 0)), "mode": kv.get("mode", "exit"),
             "code": int(kv.get("code", 13))}


def maybe_fail(rank: int, step: int) -> None:
    if not _parsed:
        _parse()
    if _spec is None or _spec["rank"] != rank or _spec["step"] != step:
        return
    if int(os.environ.get("XDDP_RESTART_COUNT", "0")) > 0 and os.environ.get("XDDP_FAULT_ONCE", "1") == "1":
        return  # only fail in the first incarnation, so a restarted group can finish
    mode = _spec["mode"]
    if mode == "raise":
        raise RuntimeError(f"xddp injected fault on rank {rank} at step {step}")
    if mode == "hang":
        while True:
            time.sleep(3600)
    os._exit(_spec["code"])
