"""Which component breaks HIP-graph capture? Capture fwd+bwd for increasingly complete stacks."""
import os, sys, traceback
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, torch.nn as nn, torch.nn.functional as F
import distributeddataparallel_amd as xddp
from distributeddataparallel_amd import distributed as dist
from distributeddataparallel_amd.ops import FusedBatchNorm2d
from distributeddataparallel_amd.models import SimpleCNN, llama_tiny
from distributeddataparallel_amd.utils.spawn import free_port

os.environ["MASTER_ADDR"] = "127.0.0.1"; os.environ["MASTER_PORT"] = str(free_port())
dist.init_process_group("rccl", rank=0, world_size=1, device_id=0)

def try_capture(name, make, bench):
    torch.backends.cudnn.benchmark = bench
    try:
        model, x, lossf = make()
        s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
        if hasattr(model, "_rebind_grad_accumulators"):
            model._rebind_grad_accumulators(s)
        with torch.cuda.stream(s):
            for _ in range(3):
                model.zero_grad(set_to_none=True)
                lossf(model(x)).backward()
        torch.cuda.current_stream().wait_stream(s); torch.cuda.synchronize()
        model.zero_grad(set_to_none=True)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            l = lossf(model(x)); l.backward()
        g.replay(); torch.cuda.synchronize()
        print(f"OK   {name} bench={bench}", flush=True)
    except Exception as e:
        print(f"FAIL {name} bench={bench}: {str(e).splitlines()[0][:150]}", flush=True)
    torch.cuda.synchronize()

def conv_plain():
    m = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.ReLU(), nn.Conv2d(16, 16, 3, padding=1)).cuda()
    return m, torch.randn(8, 3, 16, 16, device="cuda"), lambda o: o.float().pow(2).mean()
def conv_cl():
    m = nn.Sequential(nn.Conv2d(3, 16, 3, padding=1), nn.ReLU(), nn.Conv2d(16, 16, 3, padding=1)).cuda().to(memory_format=torch.channels_last)
    return m, torch.randn(8, 3, 16, 16, device="cuda").contiguous(memory_format=torch.channels_last), lambda o: o.float().pow(2).mean()
def linear_only():
    m = nn.Sequential(nn.Linear(64, 64), nn.ReLU(), nn.Linear(64, 10)).cuda()
    return m, torch.randn(8, 64, device="cuda"), lambda o: o.float().pow(2).mean()
def our_bn():
    m = nn.Sequential(FusedBatchNorm2d(16)).cuda()
    return m, torch.randn(8, 16, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last).requires_grad_(), lambda o: o.float().pow(2).mean()
def ddp_linear():
    m = xddp.DDP(nn.Sequential(nn.Linear(64, 64), nn.ReLU(), nn.Linear(64, 10)).cuda(), device_ids=[0], gradient_as_bucket_view=True)
    return m, torch.randn(8, 64, device="cuda"), lambda o: o.float().pow(2).mean()
def llama():
    m = xddp.DDP(llama_tiny().cuda(), device_ids=[0], gradient_as_bucket_view=True)
    return m, torch.randint(0, 512, (2, 32), device="cuda"), lambda o: o.float().pow(2).mean()
def simplecnn():
    m = xddp.DDP(SimpleCNN(norm_layer=FusedBatchNorm2d).cuda().to(memory_format=torch.channels_last), device_ids=[0])
    return m, torch.randn(8, 3, 32, 32, device="cuda").contiguous(memory_format=torch.channels_last), lambda o: o.float().pow(2).mean()

def mt_copy():
    C = xddp.native()
    a = torch.randn(1000, device="cuda"); b = torch.empty_like(a)
    class M(nn.Module):
        def __init__(self):
            super().__init__(); self.w = nn.Parameter(torch.ones(1, device="cuda"))
        def forward(self, x):
            C.mt_scale_copy([a], [b], 2.0); return x * self.w + b.sum()
    return M(), torch.randn(4, device="cuda"), lambda o: o.float().pow(2).mean()
def ln_fwd():
    from distributeddataparallel_amd.ops import FusedLayerNorm
    m = FusedLayerNorm(64).cuda()
    return m, torch.randn(8, 64, device="cuda"), lambda o: o.float().pow(2).mean()
def bn_fwd_only():
    C = xddp.native()
    x = torch.randn(8, 16, 8, 8, device="cuda").contiguous(memory_format=torch.channels_last)
    class M(nn.Module):
        def __init__(self):
            super().__init__(); self.w = nn.Parameter(torch.ones(1, device="cuda"))
        def forward(self, inp):
            y = C.bn_forward(x, None, None, None, None, None, True, 0.1, False, 1e-5, None, False)[0]
            return inp * self.w + y.sum()
    return M(), torch.randn(4, device="cuda"), lambda o: o.float().pow(2).mean()
cases = {"mt_copy": mt_copy, "ln_fwd": ln_fwd, "bn_fwd_only": bn_fwd_only, "linear_only": linear_only, "our_bn": our_bn, "ddp_linear": ddp_linear, "llama": llama,
         "conv_plain": conv_plain, "conv_cl": conv_cl, "simplecnn": simplecnn}
for name in sys.argv[1:] or list(cases):
    for bench in (False, True):
        try_capture(name, cases[name], bench)
dist.destroy_process_group()
