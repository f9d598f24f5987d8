"""Bucket assignment parity with the reference stack."""
import sys

import pytest
import torch
import torch.distributed as tdist

from distributeddataparallel_amd._native import load
from distributeddataparallel_amd.models import SimpleCNN, resnet50


def _torch_assign(params, limits, indices=None):
    if indices is None:
        r = tdist._compute_bucket_assignment_by_size(params, limits, [False] * len(params))
    else:
        r = tdist._compute_bucket_assignment_by_size(params, limits, [False] * len(params), indices)
    return [list(b) for b in r[0]], list(r[1])


@pytest.mark.parametrize("limits", [[sys.maxsize], [1 << 20, 25 << 20], [1 << 20, 4 << 20], [10 << 20]])
def test_matches_reference_resnet18(limits):
    C = load()
    params = list(SimpleCNN().parameters())
    ours = C.compute_bucket_assignment_by_size(params, limits)
    ref = _torch_assign(params, limits)
    assert [list(b) for b in ours[0]] == ref[0]
    assert list(ours[1]) == ref[1]


def test_reference_rebuilt_layout_resnet18():
    """Reversed (grad-ready) order with [1 MiB, 25 MiB] gives the 3 buckets of SURVEY §2.2 T8."""
    C = load()
    params = list(SimpleCNN().parameters())
    order = list(reversed(range(len(params))))
    ordered = [params[i] for i in order]
    idx, lim = C.compute_bucket_assignment_by_size(ordered, [1 << 20, 25 << 20], [], order)
    sizes = [sum(params[i].numel() * 4 for i in b) for b in idx]
    assert sizes == [9461800, 26494976, 8769792]
    assert [list(b) for b in idx] == _torch_assign(ordered, [1 << 20, 25 << 20], order)[0]


def test_mixed_dtypes_separate_buckets():
    C = load()
    ts = [torch.zeros(1000), torch.zeros(1000, dtype=torch.bfloat16), torch.zeros(10)]
    idx, _ = C.compute_bucket_assignment_by_size(ts, [1 << 30])
    assert sorted(map(sorted, idx)) == [[0, 2], [1]]


def test_resnet50_param_count():
    assert sum(p.numel() for p in resnet50().parameters()) == 25_557_032
    assert sum(p.numel() for p in SimpleCNN().parameters()) == 11_181_642
