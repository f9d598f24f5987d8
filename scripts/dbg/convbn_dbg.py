import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch, torch.nn.functional as F
from distributeddataparallel_amd.models import resnet50
from distributeddataparallel_amd.models.resnet import Bottleneck
from distributeddataparallel_amd.ops import FusedBatchNorm2d

def run(m, x, y, fwd):
    res = {}
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    for flag in ("1", "0"):
        os.environ["XDDP_CONV_BN_FUSION"] = flag
        m.load_state_dict(sd); m.zero_grad()
        out = fwd(m, x)
        loss = F.cross_entropy(out.float(), y) if y is not None else (out.float() ** 2).mean()
        loss.backward()
        res[flag] = (loss.item(), {n: p.grad.float().clone() for n, p in m.named_parameters()}, out.detach().float())
    print("loss", res["1"][0], res["0"][0], "out rel", ((res["1"][2]-res["0"][2]).norm()/res["0"][2].norm()).item())
    errs = sorted((((res["1"][1][n] - res["0"][1][n]).norm() / (res["0"][1][n].norm() + 1e-6)).item(), n, res["0"][1][n].norm().item()) for n in res["0"][1])
    for e in errs[-8:]:
        print(f"  {e[0]:.3e} {e[1]} |g|={e[2]:.3e}")

torch.manual_seed(3)
for dtype in (torch.float32, torch.bfloat16):
    print("== single bottleneck (with downsample)", dtype)
    from torch import nn
    ds = nn.Sequential(nn.Conv2d(256, 512, 1, stride=2, bias=False), FusedBatchNorm2d(512))
    blk = Bottleneck(256, 128, stride=2, downsample=ds, norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(8, 256, 28, 28, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
    run(blk, x, None, lambda m, x: m(x)[0] if isinstance(m(x), tuple) else m(x))
    break
print("== resnet50")
m = resnet50(norm_layer=FusedBatchNorm2d).cuda().to(torch.bfloat16).to(memory_format=torch.channels_last)
x = torch.randn(8, 3, 96, 96, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
y = torch.randint(0, 1000, (8,), device="cuda")
run(m, x, y, lambda m, x: m(x))
