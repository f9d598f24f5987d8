"""Flash attention: xddp HIP kernels vs torch SDPA (AOTriton on ROCm), forward and forward+backward,
at the Llama-3-8B (B1, S4096, H32/8, D128, causal) and ViT-L/16 (B64, S197, H16, D64) shapes."""
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributeddataparallel_amd.ops.attention import flash_attention  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


for name, B, S, H, Hkv, D, causal in (("llama3-8b", 1, 4096, 32, 8, 128, True), ("vit-l16", 64, 197, 16, 16, 64, False)):
    q = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    k = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    v = torch.randn(B, S, Hkv, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(B, S, H, D, device="cuda", dtype=torch.bfloat16)
    fl_f = 4.0 * B * H * S * S * D * (0.5 if causal else 1.0)

    def ours():
        return flash_attention(q, k, v, causal=causal)

    def sdpa():
        return F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                              is_causal=causal, enable_gqa=Hkv != H).transpose(1, 2)

    for lab, fn in (("xddp", ours), ("sdpa", sdpa)):
        tf = timeit(lambda: fn())
        tb = timeit(lambda: fn().backward(g))
        print(f"{name} {lab}: fwd {tf:.3f} ms ({fl_f / tf / 1e9:.0f} TF/s) | fwd+bwd {tb:.3f} ms "
              f"({3.5 * fl_f / tb / 1e9:.0f} TF/s)", flush=True)
