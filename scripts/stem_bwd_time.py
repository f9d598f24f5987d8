"""Time the stem's fused maxpool + ReLU + BN backward passes at ResNet-50 bs256 shapes.

usage: python scripts/stem_bwd_time.py [batch]
Prints one JSON line: us per call of the partial-sums pass and of the dX pass.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
C = load()
dev = torch.device("cuda")
torch.manual_seed(0)
cl = torch.channels_last
y = torch.randn(B, 64, 112, 112, device=dev, dtype=torch.bfloat16).to(memory_format=cl)
ss = torch.cat([torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev) * 0.1]).contiguous()
pooled, idx = C.stem_pool_forward(y, ss)
d1 = torch.randn_like(pooled)
d2 = torch.randn_like(pooled)
mean = y.float().mean(dim=(0, 2, 3)).contiguous()
coef = torch.randn(3, 64, device=dev).contiguous()


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


red = timeit(lambda: C.stem_pool_bn_backward(d1, d2, idx, y, ss, mean))
elem = timeit(lambda: C.stem_pool_bn_backward(d1, d2, idx, y, ss, mean, coef))
print(json.dumps({"batch": B, "reduce_us": round(red, 1),
                  "elem_us": round(elem, 1)}))
