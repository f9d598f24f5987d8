"""Debug: 2 ranks on cuda:0 (staged cpu backend) — per-iteration worst relative grad error vs the
shard-mean oracle, plus the oracle's own run-to-run noise, for BN impl x determinism."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch, torch.nn.functional as F
from _dist_utils import run_ranks


def _w(rank, world, fused, det, cl):
    import distributeddataparallel_amd as xddp
    from distributeddataparallel_amd.models import SimpleCNN
    from distributeddataparallel_amd.ops import FusedBatchNorm2d
    torch.backends.cudnn.deterministic = det
    torch.cuda.set_device(0)
    kw = dict(norm_layer=FusedBatchNorm2d) if fused else {}
    mf = torch.channels_last if cl else torch.contiguous_format
    torch.manual_seed(0); model = SimpleCNN(**kw).cuda().to(memory_format=mf)
    torch.manual_seed(0); ref = SimpleCNN(**kw).cuda().to(memory_format=mf)
    torch.manual_seed(0); ref2 = SimpleCNN(**kw).cuda().to(memory_format=mf)
    ddp = xddp.DDP(model, device_ids=[0], bucket_cap_mb=4)
    opt = torch.optim.SGD(ddp.parameters(), lr=0.05)
    g = torch.Generator(device="cuda").manual_seed(7)
    per = 8
    for it in range(4):
        ref.load_state_dict(model.state_dict()); ref2.load_state_dict(model.state_dict())
        x = torch.randn(per * world, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=mf)
        y = torch.randint(0, 10, (per * world,), device="cuda", generator=g)
        opt.zero_grad(); ref.zero_grad(); ref2.zero_grad()
        F.cross_entropy(ddp(x[rank * per:(rank + 1) * per]), y[rank * per:(rank + 1) * per]).backward()
        for m in (ref, ref2):
            for r in range(world):
                F.cross_entropy(m(x[r * per:(r + 1) * per]), y[r * per:(r + 1) * per]).div(world).backward()
        torch.cuda.synchronize()
        rel = lambda a, b: (a - b).abs().max().item() / (b.abs().max().item() + 1e-6)
        worst = max((rel(p.grad, q.grad), n) for (n, p), q in zip(model.named_parameters(), ref.parameters()))
        noise = max((rel(q2.grad, q.grad), n) for (n, q), q2 in zip(ref.named_parameters(), ref2.parameters()))
        print(f"fused={fused} det={det} cl={cl} rank{rank} it{it}: ddp-vs-oracle {worst[0]:.2e} ({worst[1]})  "
              f"oracle-noise {noise[0]:.2e} ({noise[1]})", flush=True)
        opt.step()


if __name__ == "__main__":
    for fused in (True, False):
        for det in (False, True):
            for cl in (True, False):
                run_ranks(_w, world=2, backend="cpu", args=(fused, det, cl))
