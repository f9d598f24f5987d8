"""The "fake" backend (SURVEY.md §4.2 FakeProcessGroup): one process poses as rank r of a large
world; DDP bookkeeping (bucketing, rebuild, hooks, logging) runs without peers."""
import torch
import torch.nn.functional as F


def test_fake_backend_ddp_world_64():
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd import distributed as xdist
    from distributeddataparallel_amd.models import MLP

    xdist.init_process_group("fake", rank=5, world_size=64)
    try:
        assert xdist.get_world_size() == 64 and xdist.get_rank() == 5
        torch.manual_seed(0)
        m, ref = MLP(784, 64, 10), MLP(784, 64, 10)
        ref.load_state_dict(m.state_dict())
        ddp = xddp.DDP(m, bucket_cap_mb=0.05)
        for _ in range(3):
            x, y = torch.randn(8, 1, 28, 28), torch.randint(0, 10, (8,))
            ddp.zero_grad()
            ref.zero_grad()
            F.cross_entropy(ddp(x), y).backward()
            F.cross_entropy(ref(x), y).backward()
            for a, b in zip(m.parameters(), ref.parameters()):  # AVG of 64 identical replicas
                torch.testing.assert_close(a.grad, b.grad)
        d = ddp._get_ddp_logging_data()
        assert d["world_size"] == "64" and d["has_rebuilt_buckets"] == "1"
        t = torch.arange(4.0)
        out = torch.empty(64 * 4)
        xdist.all_gather_into_tensor(out, t)
        assert torch.equal(out.view(64, 4), t.expand(64, 4))
        xdist.barrier()
    finally:
        xdist.destroy_process_group()
