"""1x1-conv MFMA GEMM (csrc/kernels/conv_gemm.hip) vs MIOpen conv2d forward on every ResNet-50
1x1 shape at batch 256 (bf16, NHWC): correctness vs fp32 torch, and time per call."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: F401,E402  (installs the shipped MIOpen tuning db)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()

SHAPES = [  # (Cin, H, W, Cout, stride) at batch 256
    (64, 56, 56, 256, 1), (64, 56, 56, 64, 1), (256, 56, 56, 64, 1), (256, 56, 56, 512, 2), (256, 56, 56, 128, 1),
    (128, 28, 28, 512, 1), (512, 28, 28, 128, 1), (512, 28, 28, 1024, 2), (512, 28, 28, 256, 1),
    (256, 14, 14, 1024, 1), (1024, 14, 14, 256, 1), (1024, 14, 14, 2048, 2), (1024, 14, 14, 512, 1),
    (512, 7, 7, 2048, 1), (2048, 7, 7, 512, 1),
]
COUNT = [4, 1, 2, 1, 1, 4, 3, 1, 1, 6, 5, 1, 1, 3, 2]  # occurrences in ResNet-50


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    B = int(os.environ.get("B", "256"))
    tot = [0.0] * 4
    for (cin, h, w, cout, s), cnt in zip(SHAPES, COUNT):
        x = torch.randn(B, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, 1, 1, device="cuda") / cin ** 0.5).to(torch.bfloat16)
        ss = torch.stack([torch.rand(cin, device="cuda") + 0.5, torch.randn(cin, device="cuda")]).contiguous()
        ref = F.conv2d(x.float(), wt.float(), stride=s)
        y, part = C.conv1x1_gemm(x, wt, s, None, True)
        err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
        xp = torch.relu(x.float() * ss[0].view(1, -1, 1, 1) + ss[1].view(1, -1, 1, 1)).to(torch.bfloat16)
        refp = F.conv2d(xp.float(), wt.float(), stride=s)
        yp, partp = C.conv1x1_gemm(x, wt, s, ss, True)
        errp = (yp.float() - refp).abs().max().item() / refp.abs().max().item()
        M = y.numel() // cout
        mean, invstd, _ = C.bn_stats_from_partials(partp, M, None, None, None, None, None, 0.1, False, 1e-5)
        yf = yp.float().permute(0, 2, 3, 1).reshape(-1, cout)
        merr = (mean - yf.mean(0)).abs().max().item() / (yf.std(0).max().item())
        verr = ((1 / invstd ** 2 - 1e-5) / yf.var(0, unbiased=False) - 1).abs().max().item()
        wcl = wt.contiguous(memory_format=torch.channels_last)
        t0 = timeit(lambda: F.conv2d(x, wcl, stride=s))
        t1 = timeit(lambda: C.conv1x1_gemm(x, wt, s, None, False))
        t2 = timeit(lambda: C.conv1x1_gemm(x, wt, s, None, True))
        t3 = timeit(lambda: C.conv1x1_gemm(x, wt, s, ss, True))
        for i, t in enumerate((t0, t1, t2, t3)):
            tot[i] += t * cnt
        gb = (x.numel() / (s * s) + y.numel()) * 2 / 1e9
        print(f"C{cin} {h}x{w} -> {cout} s{s} x{cnt}: err {err:.1e} pro {errp:.1e} mean {merr:.1e} var {verr:.1e} | "
              f"miopen {t0*1e3:7.1f} us  gemm {t1*1e3:7.1f}  +stats {t2*1e3:7.1f}  +pro {t3*1e3:7.1f} us "
              f"({gb / (t2 * 1e-3):.0f} GB/s)", flush=True)
        assert err < 2e-2 and errp < 2e-2 and merr < 1e-3 and verr < 1e-2, "numerics"
    print(f"TOTAL per ResNet-50 fwd (x count): miopen {tot[0]:.3f} ms, gemm {tot[1]:.3f}, +stats {tot[2]:.3f}, "
          f"+pro+stats {tot[3]:.3f}")


if __name__ == "__main__":
    main()
