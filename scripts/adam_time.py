"""Fused AdamW step (bf16 params + grads, fp32 master weights and moments: 28 B per parameter) on
1.07 B parameters in 8 tensors: ms per step and effective HBM bandwidth; also checks one step
against torch.optim.AdamW on a small copy. Run with PYTHONPATH=. from the repo root."""
import torch

from distributeddataparallel_amd.optim import FusedAdamW

torch.manual_seed(0)
ps = [torch.randn(1 << 27, device="cuda").bfloat16().requires_grad_() for _ in range(8)]
for p in ps:
    p.grad = torch.randn_like(p)
opt = FusedAdamW(ps, lr=1e-3, weight_decay=0.1, master_weights=True)
for _ in range(3):
    opt.step()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    opt.step()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
n = sum(p.numel() for p in ps)
print(f"fused AdamW: {ms:.3f} ms per step for {n / 1e9:.2f} B params, {28 * n / ms / 1e9:.2f} TB/s", flush=True)
# correctness vs torch.optim.AdamW (fp32 reference on the same master values, 3 steps)
q = torch.randn(3 * 8192 + 77, device="cuda")
g = [torch.randn_like(q) for _ in range(3)]
a = q.clone().requires_grad_()
b = q.clone().requires_grad_()
oa = FusedAdamW([a], lr=1e-3, weight_decay=0.1)
ob = torch.optim.AdamW([b], lr=1e-3, weight_decay=0.1)
for gg in g:
    a.grad, b.grad = gg.clone(), gg.clone()
    oa.step()
    ob.step()
print("max |fused - torch| =", (a - b).abs().max().item(), flush=True)
assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)
