"""Time the LayerNorm backward with the residual-gradient form at ViT-L/16 bs256 (50,432 x 1,024).

usage: python scripts/ln_bwd_time.py   (XDDP_LN_RESPF=0: res loaded in pass 2, not prefetched)
Prints one JSON line: us per call with and without the residual input.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
rows, D = 256 * 197, 1024
torch.manual_seed(0)
x = torch.randn(rows, D, device="cuda", dtype=torch.bfloat16)
w = torch.rand(D, device="cuda", dtype=torch.bfloat16) + 0.5
b = torch.randn(D, device="cuda", dtype=torch.bfloat16)
y, mean, rstd = C.ln_forward(x, w, b, 1e-6, False)[:3]
dy = torch.randn_like(x)
res = torch.randn_like(x)


def timeit(fn, iters=30):
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


t_res = timeit(lambda: C.ln_backward(dy, x, w, mean, rstd, False, True, True, res))
t_plain = timeit(lambda: C.ln_backward(dy, x, w, mean, rstd, False, True, True))
print(json.dumps({"rows": rows, "D": D, "respf": os.environ.get("XDDP_LN_RESPF", "1"), "res_us": round(t_res, 1),
                  "plain_us": round(t_plain, 1)}))
