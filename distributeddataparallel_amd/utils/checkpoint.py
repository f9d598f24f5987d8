"""Checkpoint / resume helpers.

* ``save_checkpoint`` — rank 0 writes ``{model, optimizer, step, extra}`` atomically
  (tmp file + rename); other ranks wait at a barrier.
* ``load_checkpoint`` — loads with ``torch.load(weights_only=True)`` (no pickled code), strips
  or adds the DDP ``module.`` prefix as needed, and re-broadcasts parameters/buffers from
  rank 0 so every replica resumes bit-identical (the DDP init-sync contract).
"""
from __future__ import annotations

import os
from typing import Any, Optional

import torch

from .. import distributed as xdist


def _unwrap(model):
    return getattr(model, "module", model)


def save_checkpoint(path: str, model, optimizer=None, step: Optional[int] = None, extra: Any = None,
                    rank0_only: bool = True) -> None:
    rank = xdist.get_rank() if xdist.is_initialized() else 0
    if not rank0_only or rank == 0:
        state = {"model": _unwrap(model).state_dict(), "step": step, "extra": extra,
                 "optimizer": optimizer.state_dict() if optimizer is not None else None}
        d = os.path.dirname(os.path.abspath(path))
        os.makedirs(d, exist_ok=True)
        tmp = f"{path}.tmp.{os.getpid()}"
        torch.save(state, tmp)
        os.replace(tmp, path)
    if xdist.is_initialized():
        xdist.barrier()


def load_checkpoint(path: str, model, optimizer=None, map_location="cpu", strict: bool = True) -> dict:
    state = torch.load(path, map_location=map_location, weights_only=True)
    sd = state["model"]
    if any(k.startswith("module.") for k in sd):
        sd = {k[len("module."):] if k.startswith("module.") else k: v for k, v in sd.items()}
    _unwrap(model).load_state_dict(sd, strict=strict)
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if xdist.is_initialized() and hasattr(model, "_sync_module_states"):
        model._sync_module_states(src=0)
    return state
