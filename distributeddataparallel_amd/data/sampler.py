"""DistributedSampler (reference: ``torch.utils.data.distributed.DistributedSampler``,
SURVEY.md §2.2 T15, used by ``ref:dpp.py:34``).

Same index stream as the reference for identical arguments: an epoch-seeded ``randperm``
(seed + epoch), padding by repeating the head (or dropping the tail with ``drop_last``),
then the strided subsample ``indices[rank:total:num_replicas]``.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch
from torch.utils.data import Sampler

from .. import distributed as xdist


class DistributedSampler(Sampler):
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas is None:
            num_replicas = xdist.get_world_size() if xdist.is_initialized() else 1
        if rank is None:
            rank = xdist.get_rank() if xdist.is_initialized() else 0
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def __iter__(self) -> Iterator[int]:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        if not self.drop_last:
            pad = self.total_size - len(indices)
            if pad <= len(indices):
                indices += indices[:pad]
            else:
                indices += (indices * math.ceil(pad / len(indices)))[:pad]
        else:
            indices = indices[: self.total_size]
        assert len(indices) == self.total_size
        indices = indices[self.rank: self.total_size: self.num_replicas]
        assert len(indices) == self.num_samples
        return iter(indices)

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
