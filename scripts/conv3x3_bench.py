"""MIOpen time per ResNet-50 3x3 conv shape (bs256, bf16, channels_last): forward, dgrad, wgrad,
with achieved TFLOP/s — sizing data for a hand-written 3x3 implicit GEMM."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: F401,E402  (installs the shipped MIOpen tuning db)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()

# (cin, input hw, cout, stride, count per step)
SHAPES = [(64, 56, 64, 1, 3), (128, 56, 128, 2, 1), (128, 28, 128, 1, 3), (256, 28, 256, 2, 1),
          (256, 14, 256, 1, 5), (512, 14, 512, 2, 1), (512, 7, 512, 1, 2)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


tot = [0.0] * 6
for cin, hw, cout, s, cnt in SHAPES:
    B = 256
    x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, 3, 3, device="cuda") / (9 * cin) ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    oh = (hw + 2 - 3) // s + 1
    dy = torch.randn(B, cout, oh, oh, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    cb = torch.ops.aten.convolution_backward
    fl = 2.0 * B * oh * oh * cout * cin * 9
    t = [timeit(lambda: F.conv2d(x, w, None, s, 1)),
         timeit(lambda: cb(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])),
         timeit(lambda: cb(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))]
    ref = F.conv2d(x, w, None, s, 1)
    got = C.conv3x3_forward(x, w, s, False)[0]
    err = (got.float() - ref.float()).abs().max().item() / ref.float().abs().max().item()
    t.append(timeit(lambda: C.conv3x3_forward(x, w, s, False)))
    derr, td = float("nan"), float("nan")
    if s == 1:
        wt = w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)
        dref = cb(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])[0]
        dgot = C.conv3x3_forward(dy, wt, 1, False)[0]
        derr = (dgot.float() - dref.float()).abs().max().item() / dref.float().abs().max().item()
        td = timeit(lambda: C.conv3x3_forward(dy, wt, 1, False))
    t.append(td)
    wref = cb(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]
    wgot = C.conv3x3_wgrad_patch(dy, x, s, w)
    werr = (wgot.float() - wref.float()).norm().item() / wref.float().norm().item()
    t.append(timeit(lambda: C.conv3x3_wgrad_patch(dy, x, s, w)))
    for i in range(5):
        tot[i] += (t[i] if t[i] == t[i] else t[1]) * cnt
    tot[5] += t[5] * cnt
    print(f"C{cin}->{cout} {hw}x{hw} s{s} x{cnt}: GFLOP {fl/1e9:6.1f} | fwd {t[0]:6.1f} us {fl/t[0]/1e6:5.0f} TF/s | "
          f"dgrad {t[1]:6.1f} us {fl/t[1]/1e6:5.0f} TF/s | wgrad {t[2]:6.1f} us {fl/t[2]/1e6:5.0f} TF/s || "
          f"ours fwd {t[3]:6.1f} us {fl/t[3]/1e6:5.0f} TF/s (err {err:.1e}) dgrad {t[4]:6.1f} us (err {derr:.1e}) "
          f"wgrad {t[5]:6.1f} us {fl/t[5]/1e6:5.0f} TF/s (rel {werr:.1e})",
          flush=True)
print(f"TOTAL (x count) ms: fwd {tot[0]/1e3:.3f} dgrad {tot[1]/1e3:.3f} wgrad {tot[2]/1e3:.3f} | "
      f"ours fwd {tot[3]/1e3:.3f} dgrad (s2 on MIOpen) {tot[4]/1e3:.3f} wgrad {tot[5]/1e3:.3f}")
