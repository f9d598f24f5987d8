"""Datasets for the reference workload without a network.

* ``SyntheticImages`` — random tensors of an image-classification shape (ImageNet-like
  3x224x224 for the headline bench, CIFAR-like 3x32x32 for the reference config), drawn
  deterministically per index so every rank sees a stable dataset.
* ``CIFAR10Binary`` — reader for the official CIFAR-10 *binary* distribution
  (``data_batch_{1..5}.bin`` / ``test_batch.bin``: 1 label byte + 3072 pixel bytes per
  record) read with numpy only — no pickles. Applies the reference's
  ``ToTensor`` + ``Normalize((0.5,), (0.5,))`` (``ref:dpp.py:32``).
"""
from __future__ import annotations

import os
from typing import Tuple

import numpy as np
import torch
from torch.utils.data import Dataset


class SyntheticImages(Dataset):
    def __init__(self, length: int = 50000, shape: Tuple[int, int, int] = (3, 32, 32), num_classes: int = 10,
                 seed: int = 0):
        self.length, self.shape, self.num_classes, self.seed = length, tuple(shape), num_classes, seed

    def __len__(self):
        return self.length

    def __getitem__(self, i):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + i)
        x = torch.randn(self.shape, generator=g)
        y = int(torch.randint(0, self.num_classes, (1,), generator=g))
        return x, y


class CIFAR10Binary(Dataset):
    RECORD = 1 + 3 * 32 * 32

    def __init__(self, root: str, train: bool = True):
        d = root if os.path.exists(os.path.join(root, "data_batch_1.bin")) else os.path.join(root, "cifar-10-batches-bin")
        files = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        chunks = []
        for f in files:
            raw = np.fromfile(os.path.join(d, f), dtype=np.uint8)
            chunks.append(raw.reshape(-1, self.RECORD))
        data = np.concatenate(chunks)
        self.labels = torch.from_numpy(data[:, 0].astype(np.int64))
        self.images = torch.from_numpy(data[:, 1:].reshape(-1, 3, 32, 32).copy())

    def __len__(self):
        return self.labels.numel()

    def __getitem__(self, i):
        x = self.images[i].float().div_(255.0).sub_(0.5).div_(0.5)
        return x, int(self.labels[i])

    @staticmethod
    def available(root: str) -> bool:
        return os.path.exists(os.path.join(root, "data_batch_1.bin")) or os.path.exists(
            os.path.join(root, "cifar-10-batches-bin", "data_batch_1.bin"))
