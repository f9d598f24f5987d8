"""Probe: W=1 DDP grads vs a plain model, per iteration (prints max |diff| per config)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn.functional as F
import distributeddataparallel_amd as xddp
from distributeddataparallel_amd import distributed as dist
from distributeddataparallel_amd.models import SimpleCNN
from distributeddataparallel_amd.utils.spawn import free_port

os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(free_port())
dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)
torch.backends.cudnn.deterministic = bool(int(os.environ.get("DET", "0")))

def run(kind, gav=False, cd=None):
    torch.manual_seed(0)
    model = SimpleCNN().cuda(); ref = SimpleCNN().cuda(); ref.load_state_dict(model.state_dict())
    net = xddp.DDP(model, device_ids=[0], gradient_as_bucket_view=gav, comm_dtype=cd) if kind == "ddp" else model
    o1 = torch.optim.SGD(net.parameters(), lr=0.01); o2 = torch.optim.SGD(ref.parameters(), lr=0.01)
    out = []
    for it in range(4):
        x = torch.randn(16, 3, 32, 32, device="cuda"); y = torch.randint(0, 10, (16,), device="cuda")
        o1.zero_grad(); o2.zero_grad()
        F.cross_entropy(net(x), y).backward(); F.cross_entropy(ref(x), y).backward()
        d = max((p.grad - q.grad).abs().max().item() for p, q in zip(model.parameters(), ref.parameters()))
        pd = max((p - q).abs().max().item() for p, q in zip(model.parameters(), ref.parameters()))
        worst = max(((p.grad - q.grad).abs().max().item(), n) for (n, p), q in zip(model.named_parameters(), ref.parameters()))
        out.append((it, f"{d:.3e}", f"param {pd:.3e}", worst[1]))
        o1.step(); o2.step()
    print(kind, gav, cd, out, flush=True)

run("plain")
run("ddp", False, None); run("ddp", True, None); run("ddp", False, torch.bfloat16); run("ddp", True, torch.bfloat16)
dist.destroy_process_group()
