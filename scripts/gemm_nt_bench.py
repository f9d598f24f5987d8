"""Own transformer GEMM (gemm_nt: csrc/kernels/gemm.hip) vs torch.mm (hipBLASLt) on random bf16
operands at the linear-layer shapes of BASELINE.json (ViT-L/16 bs64, Llama-3-8B s4096) and the
ResNet-50 deep-K 1x1 shapes; A/B interleaved in one process (median of rounds). Fused epilogues
(bias, bias+GELU) are timed against hipBLASLt addmm (+ torch GELU).

usage: python scripts/gemm_nt_bench.py [--out FILE]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()


def timed(fn, iters=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


SHAPES = [("vit qkv", 12608, 1024, 3072), ("vit proj", 12608, 1024, 1024), ("vit fc1", 12608, 1024, 4096),
          ("vit fc2", 12608, 4096, 1024), ("llama qkv", 4096, 4096, 6144), ("llama o", 4096, 4096, 4096),
          ("llama gate+up", 4096, 4096, 28672), ("llama down", 4096, 14336, 4096),
          ("r50 l3 1024>256", 50176, 1024, 256), ("r50 l4 2048>512", 12544, 2048, 512),
          ("4096^3", 4096, 4096, 4096), ("8192^3", 8192, 8192, 8192)]
lines = []
for name, M, K, N in SHAPES:
    g = torch.Generator(device="cuda").manual_seed(0)
    a = (torch.rand(M, K, device="cuda", generator=g) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda", generator=g) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g).to(torch.bfloat16)
    ref = torch.mm(a, w.t())
    err = ((C.gemm_nt(a, w)[0].float() - ref.float()).norm() / ref.float().norm()).item()
    fl = 2.0 * M * N * K
    arms = {"blas": lambda: torch.mm(a, w.t()), "own": lambda: C.gemm_nt(a, w)}
    if name.startswith("vit fc1"):
        arms["blas_bias_gelu"] = lambda: F.gelu(torch.addmm(b, a, w.t()))
        arms["own_bias_gelu"] = lambda: C.gemm_nt(a, w, b, 2)
    for f in arms.values():
        f()
    torch.cuda.synchronize()
    t = {k: [] for k in arms}
    for _ in range(5):
        for k, f in arms.items():
            t[k].append(timed(f))
    med = {k: statistics.median(v) for k, v in t.items()}
    line = (f"{name:16s} M{M} K{K} N{N}: hipBLASLt {med['blas']:.3f} ms ({fl / med['blas'] / 1e9:.0f} TF/s) | "
            f"own {med['own']:.3f} ms ({fl / med['own'] / 1e9:.0f} TF/s) = {med['blas'] / med['own']:.2f}x "
            f"(rel err {err:.1e})")
    if "own_bias_gelu" in med:
        line += (f" | +bias+GELU: hipBLASLt addmm + gelu {med['blas_bias_gelu']:.3f} ms, own fused "
                 f"{med['own_bias_gelu']:.3f} ms")
    print(line, flush=True)
    lines.append(line)
    del a, w, ref
    torch.cuda.empty_cache()
if len(sys.argv) > 2 and sys.argv[1] == "--out":
    with open(sys.argv[2], "w") as f:
        f.write("# own gemm_nt vs hipBLASLt (torch.mm), random uniform bf16 operands, 1x MI355X, median of 5 "
                "interleaved rounds x 20 calls\n" + "\n".join(lines) + "\n")
