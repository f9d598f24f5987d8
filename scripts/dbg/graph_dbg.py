import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.nn.functional as F
import distributeddataparallel_amd as xddp
from distributeddataparallel_amd import distributed as dist
from distributeddataparallel_amd.models import SimpleCNN
from distributeddataparallel_amd.ops import FusedBatchNorm2d
from distributeddataparallel_amd.optim import FusedSGD
from distributeddataparallel_amd.utils.graphs import GraphedTrainStep
from distributeddataparallel_amd.utils.spawn import free_port
os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(free_port())
dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
g = torch.Generator(device="cuda").manual_seed(3)
xs = [torch.randn(32, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last) for _ in range(6)]
ys = [torch.randint(0, 10, (32,), device="cuda", generator=g) for _ in range(6)]
import torch.nn as nn
from distributeddataparallel_amd.models.resnet import ResNet, BasicBlock
def mk(variant):
    if variant.startswith("torch"):
        return SimpleCNN()
    if variant == "fused":
        return SimpleCNN(norm_layer=FusedBatchNorm2d)
    if variant == "fusedbn_torchpool":
        m = SimpleCNN(); m.model = ResNet(BasicBlock, [2, 2, 2, 2], num_classes=10, norm_layer=FusedBatchNorm2d, pool_layer=nn.MaxPool2d); return m
    return SimpleCNN()
for trial, variant in enumerate(["torch-noddp"]):
    torch.manual_seed(0)
    m = mk(variant).cuda().to(memory_format=torch.channels_last)
    print("variant", variant, flush=True)
    d = m if "noddp" in variant else xddp.DDP(m, device_ids=[0], gradient_as_bucket_view=True)
    o = torch.optim.SGD(d.parameters(), lr=0.05, momentum=0.9) if "torchsgd" in variant else FusedSGD(d.parameters(), lr=0.05, momentum=0.9)
    step = GraphedTrainStep(d, o, F.cross_entropy, xs[0], ys[0], warmup_steps=3)
    for i, (x, y) in enumerate(zip(xs[:3], ys[:3])):
        p0 = [p.detach().clone() for p in m.parameters()]
        loss = step(x, y); torch.cuda.synchronize()
        bad = []
        for (n, p), q in zip(m.named_parameters(), p0):
            gr = p.grad
            st = o.state[p]["momentum_buffer"]
            u = (p - q).abs().max().item()
            if not torch.isfinite(p).all() or (gr is not None and not torch.isfinite(gr).all()) or not torch.isfinite(st).all() or u > 1.0:
                bad.append((n, u, None if gr is None else gr.abs().max().item(), st.abs().max().item(), gr is not None and gr.data_ptr() == 0))
        print(f"trial {trial} step {i} loss {loss.item():.4f} bad={bad[:3]}", flush=True)
dist.destroy_process_group()
