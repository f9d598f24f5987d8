"""How far the 3x3 implicit GEMM (conv3x3.hip) is from a plain GEMM of the same size: per stride-1
ResNet-50 3x3 shape (bs256), the forward conv vs the explicit GEMM Y[M, N] = A[M, 9C] · W[N, 9C]ᵀ
on the own LDS-DMA GEMM (gemm_nt, N % 128 == 0) and on hipBLASLt (torch.mm), same FLOPs; plus the
3x3 weight-gradient kernel. Median of interleaved rounds.

usage: python scripts/conv3x3_ceiling.py [--out FILE]"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
SHAPES = [(64, 56, 64), (128, 28, 128), (256, 14, 256), (512, 7, 512)]  # (C, HW, N), stride 1


def timed(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    lines = [f"{'shape':22s} {'conv3x3 fwd':>14s} {'conv dgrad':>14s} {'wgrad':>14s} {'gemm_nt':>14s} {'hipBLASLt':>14s}"]
    for c, hw, n in SHAPES:
        B = 256
        M, K = B * hw * hw, 9 * c
        fl = 2.0 * M * n * K
        x = torch.randn(B, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(n, c, 3, 3, device="cuda") / K ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        dy = torch.randn(B, n, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wr = C.conv3x3_rot_weight(w)
        a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        wm = torch.randn(n, K, device="cuda").to(torch.bfloat16)
        fns = {"fwd": lambda: C.conv3x3_forward(x, w, 1, True),
               "dgrad": lambda: C.conv3x3_forward(dy, wr, 1, False),
               "wgrad": lambda: C.conv3x3_wgrad_patch(dy, x, 1, w),
               "gemm_nt": (lambda: C.gemm_nt(a, wm)) if n % 128 == 0 else None,
               "blas": lambda: torch.mm(a, wm.t())}
        res = {k: [] for k, f in fns.items() if f is not None}
        for _ in range(5):
            for k in res:
                res[k].append(timed(fns[k]))
        med = {k: statistics.median(v) for k, v in res.items()}
        cell = lambda k: f"{med[k]:7.1f}us {fl / med[k] / 1e6:5.0f}" if k in med else f"{'-':>14s}"  # noqa: E731
        lines.append(f"C{c:<4d}{hw:3d}x{hw:<3d} N{n:<4d}    {cell('fwd')} {cell('dgrad')} {cell('wgrad')} "
                     f"{cell('gemm_nt')} {cell('blas')}")
    lines.append("(us per call, TF/s; bf16, batch 256; gemm_nt/hipBLASLt: the explicit [M, 9C] x [9C, N] GEMM)")
    text = "\n".join(lines)
    print(text)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
