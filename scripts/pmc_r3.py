"""Workload for rocprofv3 --pmc passes over the hand-written kernels (VERDICT r2 "Next round" #7; r3 adds
the halo 3x3, the conv-on-gemm_nt path, the pending-apply prologues and the deep-K statistics GEMM):
3x3 implicit-GEMM forward / stride-1 dgrad, 3x3 patch weight gradient, stem conv forward / weight
gradient, flash attention forward / backward (dK/dV with fused dQ), and the conv1 input-gradient
GEMM with the BN-reduce epilogue (EPI), and the transformer GEMM (gemm_nt) beside hipBLASLt.
ResNet-50 / ViT-L/16 / Llama-3-8B shapes at the bench batch.

Each op runs CALLS times back to back between two marker kernels (an int16 add, a name nothing else
in the workload launches); ``gpurun_out/pmc_r3_plan.json`` records, in launch order, the kernel-name
pattern, the call count and the analytic FLOPs / unique HBM bytes of one call, so
``scripts/pmc_summary.py`` can put each op's dispatches on the roofline.

usage: python scripts/pmc_r3.py [--plan-out PATH] [--only-gemm]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from distributeddataparallel_amd._native import load  # noqa: E402

C = load()
CALLS = 3
cl = torch.channels_last
plan = []
_marker = torch.zeros(7, dtype=torch.int16, device="cuda")


def bf(*shape, scale=1.0, fmt=cl):
    t = (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)
    return t.contiguous(memory_format=fmt) if len(shape) == 4 else t.contiguous()


def run(label, pattern, flops, nbytes, fn):
    if ONLY_GEMM and "gemm_nt" not in label and "hipBLASLt" not in label:
        return
    if ONLY and not any(o in label for o in ONLY):
        return
    fn()  # warm (first-call allocations, tuning) — not part of the plan
    torch.cuda.synchronize()
    plan.append({"label": label, "pattern": pattern, "calls": CALLS, "flops": float(flops), "bytes": float(nbytes)})
    _marker.add_(1)
    for _ in range(CALLS):
        fn()
    _marker.add_(1)
    torch.cuda.synchronize()


ONLY_GEMM = "--only-gemm" in sys.argv  # stall-counter passes over the transformer GEMMs alone
# --only A,B,...: ops whose label contains one of the substrings (stall passes over a subset)
ONLY = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
B = 256
# 3x3 forward (+ BN statistics epilogue) and the stride-1 input gradient (same kernel, rotated W)
# (r3 routing: 64/128 channels on the halo kernel, 256/512 on gemm_nt's im2col pipeline)
for cin, hw in ((64, 56), (128, 28), (256, 14), (512, 7)):
    x, w = bf(B, cin, hw, hw), bf(cin, cin, 3, 3, scale=(9 * cin) ** -0.5)
    m = B * hw * hw
    fl, by = 2.0 * m * cin * 9 * cin, 2.0 * (2 * x.numel() + w.numel())
    pat = "conv3x3_band_kernel" if cin <= 256 else "gemm_nt_kernel"
    run(f"conv3x3 fwd C{cin} {hw}x{hw}", pat, fl, by, lambda: C.conv3x3_forward(x, w, 1, True))
    wr = C.conv3x3_rot_weight(w)
    run(f"conv3x3 dgrad C{cin} {hw}x{hw}", pat, fl, by, lambda: C.conv3x3_forward(x, wr, 1, False))
    if cin == 512:
        continue
    run(f"conv3x3 wgrad(patch) C{cin} {hw}x{hw}", "conv3x3_wgrad_kernel", fl, 2.0 * 2 * x.numel() + 4 * w.numel(),
        lambda: C.conv3x3_wgrad_patch(x, x, 1, w))
# stem 7x7/s2 (3 -> 64, 224 -> 112): forward with BN statistics, weight gradient
xs = bf(B, 3, 224, 224)
ws = bf(64, 3, 7, 7, scale=147 ** -0.5)
ys, _ = C.stem_conv_forward(xs, ws)
m = B * 112 * 112
run("stem conv fwd", "stem_conv_fwd_kernel", 2.0 * m * 64 * 147, 2.0 * (xs.numel() + ys.numel()),
    lambda: C.stem_conv_forward(xs, ws))
run("stem conv wgrad", "stem_conv_wgrad_kernel", 2.0 * m * 64 * 147, 2.0 * (xs.numel() + ys.numel()),
    lambda: C.stem_conv_wgrad(ys, xs, ws))
# EPI: conv1 input gradient + identity gradient + ReLU mask + BN-backward reduce in the epilogue
for hw, n, k in ((56, 256, 64), (28, 512, 128), (14, 1024, 256)):
    dy = bf(B, k, hw, hw)
    w = bf(k, n, 1, 1, scale=k ** -0.5)
    add, y = bf(B, n, hw, hw), bf(B, n, hw, hw)
    bits = torch.randint(0, 256, (y.numel() // 8,), device="cuda", dtype=torch.uint8)
    mean = torch.zeros(n, device="cuda")
    run(f"EPI dgrad N{n} K{k} {hw}x{hw}", "conv1x1_gemm_kernel", 2.0 * y.numel() * k,
        2.0 * (dy.numel() + 3 * y.numel()) + bits.numel(),
        lambda: C.conv1x1_gemm(dy, w, 1, None, False, None, True, add, y, bits, mean))
# r3: pending block-output apply in conv1's GEMM prologue (relu(y3·s + t + identity), side output +
# mask bits) and BN2's apply in conv3's (side output), layer-1 shapes; the deep-K conv1 forward on
# gemm_nt with the statistics epilogue (layer 3)
for label, (k, n, res) in (("pending block->conv1 K256 N64 56x56", (256, 64, True)),
                          ("pending BN2->conv3 K64 N256 56x56", (64, 256, False))):
    y3, wt = bf(B, k, 56, 56), bf(n, k, 1, 1, scale=k ** -0.5)
    ss = torch.stack([torch.rand(k, device="cuda") + 0.5, torch.randn(k, device="cuda") * 0.2]).contiguous()
    ident = bf(B, k, 56, 56) if res else None
    side = torch.empty_like(y3)
    bits = torch.empty(y3.numel() // 8, dtype=torch.uint8, device="cuda") if res else None
    m = B * 56 * 56
    by = 2.0 * (y3.numel() * (3 if res else 2) + m * n) + (y3.numel() / 8 if res else 0)
    run(label, "conv1x1_gemm_kernel", 2.0 * m * n * k, by,
        lambda: C.conv1x1_gemm(y3, wt, 1, ss, True, pro_out=side, pro_bits=bits, pro_res=ident))
xd, wd = bf(B, 1024, 14, 14), bf(256, 1024, 1, 1, scale=1024 ** -0.5)
md = B * 14 * 14
run("deep-K conv1 fwd K1024 N256 14x14 (gemm_nt stats)", "gemm_nt_kernel", 2.0 * md * 256 * 1024,
    2.0 * (xd.numel() + md * 256 + 256 * 1024), lambda: C.gemm_nt(xd.permute(0, 2, 3, 1).reshape(-1, 1024),
                                                                  wd.view(256, 1024), None, 5))
# flash attention, ViT-L/16 (197 tokens, 16 heads x 64) at 64 images, and a Llama-like causal shape
for (b, s, h, d, causal) in ((64, 197, 16, 64, False), (2, 4096, 32, 128, True)):
    nc = torch.contiguous_format  # [B, S, H, D] row-major (channels_last would move D)
    q, k, v = bf(b, s, h, d, fmt=nc), bf(b, s, h, d, fmt=nc), bf(b, s, h, d, fmt=nc)
    o, lse = C.flash_attn_forward(q, k, v, causal, d ** -0.5)
    do = bf(b, s, h, d, fmt=nc)
    f = 0.5 if causal else 1.0
    fl = 4.0 * b * h * s * s * d * f
    run(f"flash fwd B{b} S{s} H{h} D{d}{' causal' if causal else ''}", "fa_fwd_kernel", fl, 2.0 * 4 * q.numel(),
        lambda: C.flash_attn_forward(q, k, v, causal, d ** -0.5))
    run(f"flash bwd B{b} S{s} H{h} D{d}{' causal' if causal else ''}", "fa_bwd_(dkdv|dq)_kernel", 2.5 * fl,
        2.0 * 8 * q.numel(), lambda: C.flash_attn_backward(do, q, k, v, o, lse, causal, d ** -0.5))

# the transformer GEMM (own LDS-DMA MFMA kernel) next to hipBLASLt on the same operands
for name, M, K, N in (("8192^3", 8192, 8192, 8192), ("vit fc1", 12608, 1024, 4096), ("llama down", 4096, 14336, 4096)):
    a, w = bf(M, K), bf(N, K, scale=K ** -0.5)
    fl, by = 2.0 * M * N * K, 2.0 * (M * K + N * K + M * N)
    run(f"gemm_nt {name}", "gemm_nt_kernel", fl, by, lambda: C.gemm_nt(a, w))
    run(f"hipBLASLt {name}", "Cijk", fl, by, lambda: torch.mm(a, w.t()))
    if name == "vit fc1":
        bias = bf(N)
        run(f"gemm_nt {name} +bias+GELU", "gemm_nt_kernel", fl, by + 2.0 * M * N,
            lambda: C.gemm_nt(a, w, bias, 2))
    del a, w

out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", "pmc_r3_plan.json")
if "--plan-out" in sys.argv:
    out = sys.argv[sys.argv.index("--plan-out") + 1]
elif ONLY_GEMM:
    out = out.replace("pmc_r3_plan.json", "pmc_r3_gemm_plan.json")
os.makedirs(os.path.dirname(out), exist_ok=True)
with open(out, "w") as fh:
    json.dump(plan, fh, indent=1)
print(f"pmc workload done: {len(plan)} ops x {CALLS} calls", flush=True)
