"""Time the LayerNorm / RMSNorm backward: ViT-L/16 bs256 LayerNorm rows (50,432 x 1,024, with and
without the residual-gradient input) and Llama-3-8B RMSNorm rows (4,096 x 4,096).

usage: python scripts/ln_bwd_time.py
Prints one JSON line per shape: us per call and the effective HBM rate.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()


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


torch.manual_seed(0)
for name, rows, D, rms in (("vit_ln", 256 * 197, 1024, False), ("llama_rms", 4096, 4096, True)):
    x = torch.randn(rows, D, device="cuda", dtype=torch.bfloat16)
    w = torch.rand(D, device="cuda", dtype=torch.bfloat16) + 0.5
    b = None if rms else torch.randn(D, device="cuda", dtype=torch.bfloat16)
    y, mean, rstd = C.ln_forward(x, w, b, 1e-6, rms)[:3]
    dy = torch.randn_like(x)
    mb = rows * D * 2 * 3 / 1e6  # x, dy read, dx written
    t_plain = timeit(lambda: C.ln_backward(dy, x, w, None if rms else mean, rstd, rms, True, not rms))
    out = {"shape": name, "rows": rows, "D": D, "plain_us": round(t_plain, 1), "TBps": round(mb / t_plain, 2)}
    if not rms:
        res = torch.randn_like(x)
        out["res_us"] = round(timeit(lambda: C.ln_backward(dy, x, w, mean, rstd, False, True, True, res)), 1)
    print(json.dumps(out), flush=True)
