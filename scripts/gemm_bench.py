"""Own MFMA GEMM (conv1x1_gemm: y[M, N] = x[M, K] · w[N, K]^T) vs torch.mm (hipBLASLt) at the
transformer linear-layer shapes of BASELINE.json (ViT-L/16 bs64, Llama-3-8B s4096)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


resnet = [("r50 l1 64>256", 802816, 64, 256), ("r50 l1 256>64", 802816, 256, 64), ("r50 l2 128>512", 200704, 128, 512),
          ("r50 l2 512>128", 200704, 512, 128), ("r50 l3 256>1024", 50176, 256, 1024),
          ("r50 l3 1024>256", 50176, 1024, 256), ("r50 l4 512>2048", 12544, 512, 2048),
          ("r50 l4 2048>512", 12544, 2048, 512), ("r50 l2.0 256>128", 802816, 256, 128)]
vit256 = [("vit256 qkv", 50432, 1024, 3072), ("vit256 proj", 50432, 1024, 1024), ("vit256 fc1", 50432, 1024, 4096),
          ("vit256 fc2", 50432, 4096, 1024)]
shapes = resnet if os.environ.get("GEMM_SET") == "resnet" else vit256 if os.environ.get("GEMM_SET") == "vit256" else [("vit qkv", 12608, 1024, 3072), ("vit proj", 12608, 1024, 1024), ("vit fc1", 12608, 1024, 4096),
          ("vit fc2", 12608, 4096, 1024), ("llama qkv", 4096, 4096, 6144), ("llama o", 4096, 4096, 4096),
          ("llama gate+up", 4096, 4096, 28672), ("llama down", 4096, 14336, 4096)]
for name, M, K, N in shapes:
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
    fl = 2.0 * M * N * K
    t_mm = timeit(lambda: torch.mm(x, w.t()))
    x4 = x.view(M, K, 1, 1)
    w4 = w.view(N, K, 1, 1)
    t_own = 1.0
    try:
        y = C.conv1x1_gemm(x4, w4, 1, None, False, None, False, None, None, None, None, None)[0]
        err = (y.view(M, N).float() - torch.mm(x, w.t()).float()).abs().max().item()
        t_own = timeit(lambda: C.conv1x1_gemm(x4, w4, 1, None, False, None, False, None, None, None, None, None))
        own = f"own {t_own:.3f} ms ({fl / t_own / 1e9:.0f} TF/s, maxerr {err:.3f})"
    except Exception as e:  # noqa: BLE001
        own = f"own: {str(e)[:80]}"
    gb = 2.0 * (M * K + N * K + M * N) / 1e9
    print(f"{name:14s} M{M} K{K} N{N}: hipBLASLt {t_mm:.3f} ms ({fl / t_mm / 1e9:.0f} TF/s, {gb / t_mm:.1f} TB/s) | "
          f"{own} [{gb / t_own if 'own ' in own else 0:.1f} TB/s]", flush=True)
