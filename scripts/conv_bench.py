"""Per-layer conv timing for ResNet-50 (batch 256, bf16, NHWC): MIOpen conv2d vs GEMM forms.

For every conv shape in ResNet-50, times forward + dgrad + wgrad through (a) torch conv2d
(MIOpen, with the shipped find-db if present) and, for 1x1 convs, (b) the equivalent GEMMs
through torch.mm (hipBLASLt): y = x[M,Cin] @ W[Cout,Cin]^T, dx = dy @ W, dW = dy^T @ x.
Prints per-shape ms and the total, to decide which convs to route where.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: F401,E402  (installs the shipped MIOpen tuning db)
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from distributeddataparallel_amd.models import resnet50  # noqa: E402


def shapes(batch=256):
    m = resnet50()
    out = []

    def hook(mod, inp, outp):
        x = inp[0]
        out.append((x.shape[1], x.shape[2], x.shape[3], mod.out_channels, mod.kernel_size[0], mod.stride[0],
                    mod.padding[0]))

    hs = [mod.register_forward_hook(hook) for mod in m.modules() if isinstance(mod, torch.nn.Conv2d)]
    with torch.no_grad():
        m(torch.zeros(1, 3, 224, 224))
    for h in hs:
        h.remove()
    return [(batch,) + s for s in out]


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def main():
    dev = "cuda"
    tot_conv, tot_mm1 = 0.0, 0.0
    rows = []
    for (n, cin, h, w, cout, k, s, p) in shapes():
        x = torch.randn(n, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = torch.randn(cout, cin, k, k, device=dev, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        x.requires_grad_()
        wt.requires_grad_()
        y = F.conv2d(x, wt, stride=s, padding=p)
        gy = torch.randn_like(y)

        def conv_step():
            yy = F.conv2d(x, wt, stride=s, padding=p)
            torch.autograd.grad(yy, (x, wt), gy)

        tc = timeit(conv_step)
        tm = float("nan")
        if k == 1:
            xs = x.detach()[:, :, ::s, ::s] if s > 1 else x.detach()
            M = xs.shape[0] * xs.shape[2] * xs.shape[3]
            x2 = xs.permute(0, 2, 3, 1).reshape(M, cin).contiguous()
            w2 = wt.detach().view(cout, cin)
            g2 = gy.permute(0, 2, 3, 1).reshape(M, cout).contiguous()

            def mm_step():
                torch.mm(x2, w2.t())
                torch.mm(g2, w2)
                torch.mm(g2.t(), x2)

            tm = timeit(mm_step)
            tot_mm1 += tm
            tot_conv_1x1 = tc
        tot_conv += tc
        rows.append((n, cin, h, w, cout, k, s, tc, tm))
        print(f"N{n} C{cin} {h}x{w} -> {cout} k{k} s{s}: conv {tc:.3f} ms   mm {tm:.3f} ms", flush=True)
    c1 = sum(r[7] for r in rows if r[5] == 1)
    c3 = sum(r[7] for r in rows if r[5] != 1)
    print(f"TOTAL conv fwd+bwd: {tot_conv:.2f} ms  (1x1: {c1:.2f} ms, other: {c3:.2f} ms); 1x1 via mm: {tot_mm1:.2f} ms")


if __name__ == "__main__":
    main()
