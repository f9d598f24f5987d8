"""Per-shape time of the 3x3 weight gradient (ResNet-50 bs256 shapes): MIOpen vs the 8x8-patch
kernel (csrc/kernels/conv3x3_wgrad.hip) at several split counts (slab traffic vs parallelism)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: F401,E402
import torch  # noqa: E402

bench._install_miopen_tuning()
from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
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


tot_m, tot_o = 0.0, 0.0
for cin, hw, cout, s, cnt in SHAPES:
    B = 256
    x = torch.randn(B, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(cout, cin, 3, 3, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    oh = (hw - 1) // s + 1
    dy = torch.randn(B, cout, oh, oh, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    cb = torch.ops.aten.convolution_backward
    fl = 2.0 * B * oh * oh * cout * cin * 9
    tm = timeit(lambda: cb(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False]))
    ref = cb(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1].float()
    res = []
    for sp in (-1, 64, 128, 256, 512):
        got = C.conv3x3_wgrad_patch(dy, x, s, w, sp).float()
        rel = ((got - ref).norm() / ref.norm()).item()
        res.append((sp, timeit(lambda: C.conv3x3_wgrad_patch(dy, x, s, w, sp)), rel))
    best = min(r[1] for r in res)
    tot_m += tm * cnt
    tot_o += res[0][1] * cnt
    print(f"C{cin}->{cout} {hw} s{s} x{cnt}: MIOpen {tm:6.1f} us ({fl / tm / 1e6:4.0f} TF/s) | ours " +
          " ".join(f"S{sp}:{t:6.1f}us(rel {r:.1e})" for sp, t, r in res) + f" | best {fl / best / 1e6:4.0f} TF/s",
          flush=True)
print(f"TOTAL x count: MIOpen {tot_m / 1e3:.3f} ms, ours (auto splits) {tot_o / 1e3:.3f} ms")
