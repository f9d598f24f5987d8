"""Run by tests/test_reference_workload_gpu.py in a fresh process: the reference workload's training
loop (``ref:dpp.py:44-53``: SyntheticImages CIFAR-shaped data -> DistributedSampler -> DataLoader,
ResNet-18 10-class, fp32, SGD(lr=0.01), CrossEntropy) on xddp DDP over RCCL with one rank, checked
step by step against an fp64 CPU model that is re-loaded with xddp's parameters before every step
(teacher forcing: the training itself is chaotic — a 1e-7 relative weight perturbation moves the
step-1 loss by 2e-4 on the CPU — so free-running trajectories cannot be compared past a few steps).
Prints one line per step: 'step i loss_rel grad_rel worst_param own_grad_rel' where own_grad_rel covers
the parameters whose gradients xddp's own kernels produce (BatchNorm weights / biases, the fc layer);
the conv weight gradients come from MIOpen (utils/precision.py)."""
import os
import sys

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import distributeddataparallel_amd as xddp  # noqa: E402
from distributeddataparallel_amd import distributed as dist  # noqa: E402
from distributeddataparallel_amd.data import DistributedSampler, SyntheticImages  # noqa: E402
from distributeddataparallel_amd.models import SimpleCNN  # noqa: E402
from distributeddataparallel_amd.ops import FusedBatchNorm2d  # noqa: E402
from distributeddataparallel_amd.utils.precision import accurate_fp32_convs  # noqa: E402


def main(steps):
    if os.environ.get("XDDP_TEST_ACCURATE_CONVS") == "1":
        accurate_fp32_convs()
    if os.environ.get("XDDP_TEST_NO_MIOPEN") == "1":  # (diagnosis: PyTorch's native convolutions)
        torch.backends.cudnn.enabled = False
    dist.init_process_group("rccl", device_id=0)
    torch.manual_seed(0)
    ds = SyntheticImages(length=4096, shape=(3, 32, 32))
    sampler = DistributedSampler(ds, num_replicas=1, rank=0, shuffle=True)
    loader = DataLoader(ds, batch_size=32, sampler=sampler)
    dev = torch.device("cuda", 0)
    model = SimpleCNN(norm_layer=FusedBatchNorm2d).to(dev).to(memory_format=torch.channels_last)
    ddp = xddp.DDP(model, device_ids=[0])
    opt = torch.optim.SGD(ddp.parameters(), lr=0.01)
    oracle = SimpleCNN().double()
    for i, (x, y) in enumerate(loader):
        if i >= steps:
            break
        oracle.load_state_dict({k: v.detach().double().cpu() for k, v in model.state_dict().items()})
        oracle.zero_grad()
        lo = F.cross_entropy(oracle(x.double()), y)
        lo.backward()
        opt.zero_grad()
        loss = F.cross_entropy(ddp(x.to(dev).contiguous(memory_format=torch.channels_last)), y.to(dev))
        loss.backward()
        g, worst, own = 0.0, "", 0.0
        for (n, p), q in zip(model.named_parameters(), oracle.parameters()):
            e = (p.grad.double().cpu() - q.grad).abs().max().item() / (q.grad.abs().max().item() + 1e-30)
            if e > g:
                g, worst = e, n
            if ".bn" in n or n.startswith("model.bn") or ".fc." in n or n.startswith("model.fc"):
                own = max(own, e)
        print(f"step {i} {abs(loss.item() - lo.item()) / abs(lo.item()):.3e} {g:.3e} {worst} {own:.3e}", flush=True)
        opt.step()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 50)
