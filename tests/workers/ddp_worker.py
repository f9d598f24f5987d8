"""Worker launched by tests/test_launch.py (torchrun or xddp.run): a few DDP steps on CPU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import distributeddataparallel_amd as xddp  # noqa: E402
from distributeddataparallel_amd import distributed as dist  # noqa: E402
from distributeddataparallel_amd.models import MLP  # noqa: E402

dist.init_process_group("cpu")
rank, world = dist.get_rank(), dist.get_world_size()
torch.manual_seed(0)
ddp = xddp.DDP(MLP(784, 32, 10))
opt = torch.optim.SGD(ddp.parameters(), lr=0.1)
steps = int(os.environ.get("WORKER_STEPS", "4"))
for i in range(steps):
    x = torch.randn(8, 784)
    y = torch.randint(0, 10, (8,))
    opt.zero_grad()
    F.cross_entropy(ddp(x), y).backward()
    opt.step()
t = torch.ones(1)
dist.all_reduce(t)
assert t.item() == world
w = next(ddp.parameters()).detach().clone()
dist.broadcast(w, 0)
assert torch.equal(w, next(ddp.parameters()).detach())
print(f"RANK {rank}/{world} OK restart={os.environ.get('XDDP_RESTART_COUNT', '-')}", flush=True)
dist.destroy_process_group()
