"""Interop: xddp DDP on a torch.distributed process group (the reference's own
``dist.init_process_group`` call, ref:dpp.py:21), via the native PyComm adapter."""
import os
import sys

import torch
import torch.nn.functional as F

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port):
    sys.path.insert(0, REPO)
    import torch.distributed as tdist

    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd.models import MLP

    tdist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    assert not xdist.is_initialized()
    torch.manual_seed(0)
    m1 = MLP(784, 64, 10)
    torch.manual_seed(0)
    m2 = MLP(784, 64, 10)
    ddp = xddp.DDP(m1, bucket_cap_mb=0.05)  # several buckets
    assert ddp.process_group.comm.backend() == "torch:gloo"
    tddp = torch.nn.parallel.DistributedDataParallel(m2)
    o1 = torch.optim.SGD(m1.parameters(), lr=0.05, momentum=0.9)
    o2 = torch.optim.SGD(m2.parameters(), lr=0.05, momentum=0.9)
    g = torch.Generator().manual_seed(rank + 1)
    for it in range(4):
        x, y = torch.randn(8, 1, 28, 28, generator=g), torch.randint(0, 10, (8,), generator=g)
        o1.zero_grad()
        o2.zero_grad()
        if it == 1:
            with ddp.no_sync():
                F.cross_entropy(ddp(x), y).backward()
            with tddp.no_sync():
                F.cross_entropy(tddp(x), y).backward()
        F.cross_entropy(ddp(x), y).backward()
        F.cross_entropy(tddp(x), y).backward()
        for a, b in zip(m1.parameters(), m2.parameters()):
            torch.testing.assert_close(a.grad, b.grad, rtol=1e-5, atol=1e-6)
        o1.step()
        o2.step()
    # explicit group argument works too
    ddp2 = xddp.DDP(MLP(784, 16, 10), process_group=tdist.group.WORLD)
    F.cross_entropy(ddp2(x), y).backward()
    tdist.destroy_process_group()


def test_ddp_on_torch_process_group():
    from distributeddataparallel_amd.utils.spawn import free_port, spawn

    spawn(_worker, args=(2, free_port()), nprocs=2, env={"OMP_NUM_THREADS": "1"})
