"""1x1-conv input gradient: MIOpen (aten::convolution_backward, dgrad only) vs the MFMA GEMM of
conv_gemm.hip run on (dY, W^T); also MIOpen wgrad-only and dgrad+wgrad for reference."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: F401,E402  (installs the shipped MIOpen tuning db)
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
SHAPES = [(64, 56, 256), (64, 56, 64), (256, 56, 64), (256, 56, 128), (128, 28, 512), (512, 28, 128), (512, 28, 256),
          (256, 14, 1024), (1024, 14, 256), (1024, 14, 512), (512, 7, 2048), (2048, 7, 512)]
COUNT = [4, 1, 2, 1, 4, 3, 1, 6, 5, 1, 3, 2]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


tot = [0.0] * 5
for (cin, hw, cout), cnt in zip(SHAPES, COUNT):
    x = torch.randn(256, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    dy = torch.randn(256, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    cb = torch.ops.aten.convolution_backward

    def miopen(mask):
        return lambda: cb(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, mask)

    def ours():
        wt = w.view(cout, cin).t().contiguous().view(cin, cout, 1, 1)
        return C.conv1x1_gemm(dy, wt, 1, None, False)[0]

    refw = cb(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [False, True, False])[1]
    gotw = C.conv1x1_wgrad(dy, x, 1, w)
    errw = (gotw.float() - refw.float()).norm().item() / refw.float().norm().item()
    ref = cb(dy, x, w, None, [1, 1], [0, 0], [1, 1], False, [0, 0], 1, [True, False, False])[0]
    got = ours()
    err = (got.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
    t = [timeit(miopen([True, False, False])), timeit(ours), timeit(miopen([False, True, False])),
         timeit(miopen([True, True, False])), timeit(lambda: C.conv1x1_wgrad(dy, x, 1, w))]
    for i in range(5):
        tot[i] += t[i] * cnt
    print(f"C{cin} {hw}x{hw} -> {cout} x{cnt}: err {err:.1e} | dgrad miopen {t[0]:6.1f} us  ours {t[1]:6.1f} | "
          f"wgrad miopen {t[2]:6.1f} ours {t[4]:6.1f} (rel err {errw:.1e}) | both {t[3]:6.1f}", flush=True)
print(f"TOTAL (x count) ms: dgrad miopen {tot[0]/1e3:.3f} ours {tot[1]/1e3:.3f} | wgrad {tot[2]/1e3:.3f} "
      f"ours {tot[4]/1e3:.3f} | "
      f"both {tot[3]/1e3:.3f}")
