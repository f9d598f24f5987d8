"""EPI input-gradient GEMM (conv1 dgrad + previous block's identity gradient, ReLU mask and BN
reduce in the epilogue) on the four ResNet-50 bs256 stage shapes: per-shape time and effective
HBM bandwidth (also the workload for rocprofv3 --pmc passes)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
cl = torch.channels_last
for hw, n, k in ((56, 256, 64), (28, 512, 128), (14, 1024, 256), (7, 2048, 512)):
    b = 256
    dy = torch.randn(b, k, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    w = (torch.randn(k, n, 1, 1, device="cuda") / k ** 0.5).to(torch.bfloat16)  # conv1 weight [width, Cin]
    add = torch.randn(b, n, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    y = torch.randn(b, n, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
    bits = torch.randint(0, 256, (y.numel() // 8,), device="cuda", dtype=torch.uint8)
    mean = torch.zeros(n, device="cuda")
    f = lambda: C.conv1x1_gemm(dy, w, 1, None, False, None, True, add, y, bits, mean)  # noqa: E731
    for _ in range(3):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(10):
        f()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / 10 * 1e3
    byts = dy.numel() * 2 + 3 * y.numel() * 2 + bits.numel()
    print(f"{hw}x{hw} N={n} K={k}: {t:7.1f} us, {byts / t / 1e6:5.2f} TB/s of unique bytes "
          f"({2 * y.numel() * k / t / 1e6:5.0f} TF/s)", flush=True)
