"""Time the BN-backward reduce with the folded finalize (XDDP_BN_TAIL) against the separate
finalize, and the folded form's stages (XDDP_BN_TAIL_DBG: 1 = partial stores only, 3 = + arrival
atomic and the reducers' poll, 0 = + the reduction): 50 back-to-back calls per shape and mode
(bn_backward coefficient form of a 3x3 BN + ReLU). Run with PYTHONPATH=. from the repo root."""
import os

import torch

from distributeddataparallel_amd._native import load

C_ = load()
cl = torch.channels_last
for shape in [(256, 64, 56, 56), (256, 128, 28, 28), (256, 256, 14, 14), (256, 512, 7, 7)]:
    C = shape[1]
    x = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=cl)
    g1 = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=cl)
    w = torch.rand(C, device="cuda").bfloat16() + 0.5
    b = torch.zeros(C, device="cuda").bfloat16()
    y, mean, inv, ss, _ = C_.bn_forward(x, w, b, None, None, None, True, 0.1, False, 1e-5, None, True, False)
    row = []
    for tail, dbg in [(0, 0), (1, 1), (1, 3), (1, 0), (0, 0)]:  # (2 never resets the counters: not timed)
        os.environ["XDDP_BN_TAIL"] = str(tail)
        os.environ["XDDP_BN_TAIL_DBG"] = str(dbg)
        f = lambda: C_.bn_backward(g1, x, None, w, mean, inv, ss, True, False, True, None, None, True)  # noqa
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(50):
            f()
        e1.record()
        torch.cuda.synchronize()
        row.append(f"{'tail' if tail else 'sep'}{dbg if tail else ''} {e0.elapsed_time(e1) / 50 * 1e3:6.1f}")
    print(shape, " | ".join(row), flush=True)
