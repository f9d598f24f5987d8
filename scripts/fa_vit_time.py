"""Time the flash attention forward at the ViT-L/16 bs256 head shape (B256, S197, H16, D64).

usage: python scripts/fa_vit_time.py
Prints one JSON line: us per forward call, per forward + backward through autograd (q / k / v
views of one qkv tensor), and per call of the backward kernels alone.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd.ops.attention import flash_attention  # noqa: E402

B, S, H, D = 256, 197, 16, 64
torch.manual_seed(0)
qkv = torch.randn(B, S, 3, H, D, device="cuda", dtype=torch.bfloat16)
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
for _ in range(3):
    flash_attention(q, k, v)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
iters = 30
e0.record()
for _ in range(iters):
    flash_attention(q, k, v)
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) * 1e3 / iters
tf = 4.0 * B * H * S * S * D / us / 1e6
qkv.requires_grad_(True)
q, k, v = qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2]
g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)


def step():
    flash_attention(q, k, v).backward(g)
    qkv.grad = None


for _ in range(3):
    step()
torch.cuda.synchronize()
e0.record()
for _ in range(iters):
    step()
e1.record()
torch.cuda.synchronize()
fb = e0.elapsed_time(e1) * 1e3 / iters
# the backward kernels alone (delta pre-pass + dK/dV/dQ), as the encoder block calls them
from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
qd, kd, vd = (t.detach() for t in (q, k, v))
o, lse = C.flash_attn_forward(qd, kd, vd, False, D ** -0.5)[:2]
for _ in range(3):
    C.flash_attn_backward(g, qd, kd, vd, o, lse, False, D ** -0.5, None, None, None)
torch.cuda.synchronize()
e0.record()
for _ in range(iters):
    C.flash_attn_backward(g, qd, kd, vd, o, lse, False, D ** -0.5, None, None, None)
e1.record()
torch.cuda.synchronize()
bw = e0.elapsed_time(e1) * 1e3 / iters
print(json.dumps({"shape": [B, S, H, D], "fwd_us": round(us, 1),
                  "tflops": round(tf, 1), "fwd_bwd_us": round(fb, 1), "bwd_kernels_us": round(bw, 1)}))
