"""Uneven-input support: ``Join`` context manager, ``Joinable`` and ``JoinHook``.

Behaviour follows the reference stack (``torch/distributed/algorithms/
join.py:14-350``): every iteration each non-joined rank all-reduces a ``1``; once a rank
runs out of data it loops, all-reducing ``0`` to count the ranks still training and
running each Joinable's ``main_hook`` to shadow their per-iteration collectives, then
``post_hook(is_last_joiner)``.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, List, NamedTuple, Optional

import torch

from .. import distributed as xdist


class JoinHook:
    def main_hook(self) -> None:  # shadow one iteration of collectives
        ...

    def post_hook(self, is_last_joiner: bool) -> None:
        ...


class _JoinConfig(NamedTuple):
    enable: bool
    throw_on_early_termination: bool
    is_first_joinable: bool

    @staticmethod
    def construct_disabled_join_config():
        return _JoinConfig(enable=False, throw_on_early_termination=False, is_first_joinable=False)


class Joinable(ABC):
    @abstractmethod
    def __init__(self):
        super().__init__()
        self._join_config = _JoinConfig.construct_disabled_join_config()

    @abstractmethod
    def join_hook(self, **kwargs) -> JoinHook:
        ...

    @property
    @abstractmethod
    def join_device(self) -> torch.device:
        ...

    @property
    @abstractmethod
    def join_process_group(self) -> Any:
        ...


class Join:
    def __init__(self, joinables: List[Joinable], enable: bool = True, throw_on_early_termination: bool = False,
                 **kwargs):
        if len(joinables) == 0:
            raise ValueError("The join context manager requires at least one joinable")
        self._joinables = joinables
        self._join_hooks = [j.join_hook(**kwargs) for j in joinables]
        self._enable = enable
        self._throw_on_early_termination = throw_on_early_termination
        self._set_joinable_configs()
        self._extract_dist_info()

    def _set_joinable_configs(self):
        for i, j in enumerate(self._joinables):
            j._join_config = _JoinConfig(self._enable, self._throw_on_early_termination, i == 0)

    def _extract_dist_info(self):
        pgs = {id(j.join_process_group) for j in self._joinables}
        if len(pgs) > 1:
            raise ValueError("Using join context manager with multiple process groups")
        self._process_group = self._joinables[0].join_process_group
        self._device = self._joinables[0].join_device
        self._rank = xdist.get_rank(self._process_group)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc_value, tb):
        if not self._enable or exc_type:
            return
        all_procs_joined = False
        is_last_joiner = True
        i = 0
        while not all_procs_joined:
            num_nonjoined = self._get_num_nonjoined_procs()
            if num_nonjoined == 0:
                all_procs_joined = True
            else:
                if self._throw_on_early_termination:
                    self._notify_procs_to_terminate()
                is_last_joiner = False
                for h in self._join_hooks:
                    h.main_hook()
            i += 1
        for h in self._join_hooks:
            h.post_hook(is_last_joiner)
        for j in self._joinables:
            j._join_config = _JoinConfig.construct_disabled_join_config()

    def _get_num_nonjoined_procs(self) -> int:
        t = torch.zeros(1, device=self._device)
        xdist.all_reduce(t, group=self._process_group)
        return int(t.item())

    def _notify_procs_to_terminate(self):
        ones = torch.ones(1, device=self._device)
        xdist.all_reduce(ones, group=self._process_group)
        raise RuntimeError(f"Rank {self._rank} exhausted all inputs.")

    @staticmethod
    def notify_join_context(joinable: Joinable) -> Optional[xdist.Work]:
        """Called once per iteration by every non-joined rank; returns the async all-reduce."""
        cfg = joinable._join_config
        if not cfg.is_first_joinable or not cfg.enable:
            return None
        device = joinable.join_device
        pg = joinable.join_process_group
        ones = torch.ones(1, device=device)
        work = xdist.all_reduce(ones, group=pg, async_op=True)
        if cfg.throw_on_early_termination:
            zeros = torch.zeros(1, device=device)
            xdist.all_reduce(zeros, group=pg)
            if int(zeros.item()) > 0:
                raise RuntimeError("Detected at least one rank that exhausted inputs. Throwing across all ranks.")
        work._ones = ones
        return work
