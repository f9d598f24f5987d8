"""1x1 convolution + BatchNorm(+residual)(+ReLU) with the BN statistics computed in the conv's
epilogue (``csrc/kernels/conv_gemm.hip``: an MFMA GEMM on gfx950).

In the reference stack every BatchNorm after a conv re-reads the conv output for its batch
statistics. For the ResNet-50 1x1 convs the GEMM that produces the
output also reduces it per channel, so the stats pass disappears; the apply pass (scale/shift,
residual, ReLU, ReLU bit mask) and the BN backward reuse the fused-BN kernels. The conv input
gradient of stride-1 convs is the same MFMA GEMM on (dY, Wᵀ); the weight gradient is an MFMA
GEMM over the pixel dimension (``conv1x1_wgrad``: dYᵀ·X with transposed LDS reads, fp32 slabs
split over pixels and summed by a second kernel). The stride-2 input gradient is the stride-1
GEMM over the strided pixels (compact), handed to the next consumer's epilogue or scattered.

The ResNet bottleneck's 3x3 conv + BN + ReLU (``conv3x3_bn_relu``) runs on the implicit-GEMM
kernel of ``csrc/kernels/conv3x3.hip`` with the same statistics epilogue; its stride-1 input
gradient is that kernel on (dY, rot180(W)ᵀ) (the stride-2 one: four phase GEMMs of 1/2/2/4 taps
on the dense GEMM pipeline, ``gemm.hip`` DGS2); both weight gradients are ``conv3x3_wgrad.hip``.

Parameters and buffers stay in the original ``nn.Conv2d`` / ``FusedBatchNorm2d`` modules, so
state_dict layout and DDP bucketing are unchanged.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn as nn

from .._native import load

__all__ = ["conv1x1_bn_act", "conv3x3_bn_relu", "conv_bn_supported"]


class EpiLink:
    """Backward hand-off between a bottleneck's last conv+BN+add+ReLU (the producer of a dual
    output) and the next block's two consumers of that output: its conv3 BN backward leaves the
    identity-path gradient here (``add``) instead of returning it, and its conv1 input-gradient
    GEMM folds ``add``, the producer's ReLU mask and the producer's BN-backward reduction into its
    epilogue (``conv1x1_gemm(..., epi_*)``), leaving the BN partials here (``part``). The producer's
    backward then starts from the finished gradient g and the partials: its separate reduce pass
    over (dout, dout2, y, mask) is gone (csrc/kernels/conv_gemm.hip, EpiBN).

    ``g`` is the exact tensor conv1's backward returned. If the gradient reaching the producer is
    any other tensor (a third consumer of the block output — a feature hook, an auxiliary loss —
    had its gradient summed in), the partials do not describe it and the producer falls back to
    its own masked reduce over the sum (exact: g is already masked, and masking is idempotent).

    Downsample blocks (``add_s2``): the second consumer is the stride-2 1x1 downsample conv. Its
    backward (which runs before conv1's: the downsample is issued after conv2 in the forward, so
    the autograd engine's sequence-number order takes it first) leaves its *compact* input
    gradient dY·W at the strided pixels here; conv1's epilogue adds it at the even (h, w) pixels.
    MIOpen's strided dgrad (zero-fill + full-resolution write, three quarters zeros) and the
    producer's separate reduce pass are both gone. ``c1_done`` marks that conv1's backward already
    ran (any order surprise): the downsample then returns its gradient to autograd instead."""

    __slots__ = ("y", "bits", "mean", "add", "part", "g", "add_s2", "c1_done")

    def __init__(self):
        self.y = self.bits = self.mean = self.add = self.part = self.g = None
        self.add_s2 = self.c1_done = False


class DeferredBN:
    """A downsample conv+BN whose BN apply is folded into its consumer: the downsample's output
    tensor holds the raw conv output y, and the block's final apply pass computes
    relu(bn3(y3) + y·scale + shift) (``bn_apply(..., residual_ss=...)``), so the identity branch
    never makes its own read-y / write-identity pass. Autograd convention: the gradient that
    reaches the downsample node is d(identity) — what its BN backward expects — since the only
    consumer (the final node, or ``_ApplyDeferred`` on a fallback path) passes it through."""

    __slots__ = ("ss", "nbt")

    def __init__(self):
        self.ss = self.nbt = None


class _ApplyDeferred(torch.autograd.Function):
    """identity = y·scale + shift for a consumer that cannot fold it (gradient passes through)."""

    @staticmethod
    def forward(ctx, y, ss, nbt):
        C = y.size(1)
        if nbt is not None:
            nbt.add_(1)
        return (y.float() * ss[:C].view(1, -1, 1, 1) + ss[C:].view(1, -1, 1, 1)).to(y.dtype).contiguous(
            memory_format=torch.channels_last)

    @staticmethod
    def backward(ctx, g):
        return g, None, None


class PendingApply:
    """A BatchNorm apply (``relu(y·s + t [+ r])``) whose output tensor exists but is not written
    yet: its consumer, the next 1x1 conv's GEMM, computes it while staging its A operand and
    stores it as a side output (``conv1x1_gemm(..., pro_out=...)``, csrc/kernels/conv_gemm.hip
    ProOut) — so the activation is written once and never read back by that conv, and the apply
    pass disappears. Two producers: a bottleneck's conv2 + BN2 + ReLU (consumer: conv3, prologue
    1) and a bottleneck's final BN3 + residual + ReLU (consumer: the next block's conv1, prologue
    4 / 5 with the deferred downsample BN; the ReLU mask bits come out of the same prologue).

    Any other reader must call :func:`resolve` first, which runs the ordinary apply into the same
    tensors; the consumers in this module do so whenever they cannot absorb it, and the model
    only creates pending block outputs when nothing else can see them (ResNet.forward: no
    forward hooks, final output resolved). ``nbt`` / ``rnbt``: the counters the apply bumps."""

    __slots__ = ("y", "ss", "res", "rss", "nbt", "rnbt", "out", "bits", "done")

    def __init__(self, y, ss, res, rss, nbt, rnbt, out, bits):
        self.y, self.ss, self.res, self.rss, self.nbt, self.rnbt = y, ss, res, rss, nbt, rnbt
        self.out, self.bits, self.done = out, bits, False

    def resolve(self):
        if not self.done:
            self.done = True
            load().bn_apply(self.y, self.ss, self.res, True, self.bits is not None, self.nbt, self.rss, self.rnbt,
                            self.out, self.bits)
        self.y = self.res = self.ss = self.rss = None


def resolve(t):
    """Make a possibly-pending activation readable (no-op for ordinary tensors)."""
    p = getattr(t, "_xddp_pend", None) if t is not None else None
    if p is not None and not p.done:
        p.resolve()
    return t


def _pending_apply() -> bool:
    """XDDP_PENDING_APPLY=0 keeps the separate apply passes of BN2 and of the block output instead of
    folding them into the consuming 1x1 GEMM's prologue (A/B switch)."""
    return os.environ.get("XDDP_PENDING_APPLY", "1") != "0"


def _new_pending(y, ss, res, rss, nbt, rnbt, with_bits):
    out = torch.empty_like(y, memory_format=torch.channels_last)
    bits = torch.empty(y.numel() // 8, dtype=torch.uint8, device=y.device) if with_bits else None
    return PendingApply(y, ss, res, rss, nbt, rnbt, out, bits)


def _deferred(t):
    return getattr(t, "_xddp_bnss", None) if t is not None else None


def _expand_s2(add, like):
    """Full-resolution gradient of a stride-2 1x1 conv's input from its compact form."""
    full = torch.zeros_like(like, memory_format=torch.channels_last)
    full[:, :, ::2, ::2] = add
    return full


class BNReLULink:
    """Backward hand-off from a bottleneck's conv3 to the conv2 (3x3) + BN2 + ReLU that produced
    its input (a single consumer). conv3's input-gradient GEMM masks its output by BN2's ReLU
    (recomputed from y2 and BN2's scale/shift) and reduces BN2's backward partials in its epilogue
    (``conv1x1_gemm(..., epi_ss=...)``, csrc/kernels/conv_gemm.hip EpiBN second form); BN2's
    backward then skips its reduce pass over (dout, y2). ``g`` is the exact tensor handed to
    autograd: if the gradient that reaches BN2 is any other tensor (another consumer's gradient
    was summed in), the partials do not describe it and BN2 falls back to its own reduce."""

    __slots__ = ("y", "mean", "ss", "part", "g")

    def __init__(self, y, mean, ss):
        self.y, self.mean, self.ss = y, mean, ss
        self.part = self.g = None


def _c1_dma(x, w) -> bool:
    """1x1 forward on the LDS-DMA pipeline? XDDP_C1_DMA = 0 (never, default) | 1 (always) | min Cin.

    Measured on ResNet-50 bs256 (profiles/r2_c1dma_ab.txt): no threshold beats the register-staged
    GEMM (11,662 img/s off, 11,625 at Cin >= 1024, 11,508 for every 1x1), so it stays opt-in."""
    v = os.environ.get("XDDP_C1_DMA", "0")
    if v == "0":
        return False
    return x.size(1) >= (1 if v == "1" else int(v))


def _c1_blas_min_k() -> int:
    """Stride-1 1x1 forwards with Cin >= XDDP_C1_BLAS_MIN_K (default 1024; 0 = never) run the GEMM
    on hipBLASLt + a statistics pass instead of the fused-statistics GEMM."""
    v = int(os.environ.get("XDDP_C1_BLAS_MIN_K", "1024"))
    return v if v > 0 else 1 << 30


def _deep_k_own() -> bool:
    """The deep-K 1x1 forwards run the own LDS-DMA GEMM with the BN-statistics epilogue (gemm.hip
    kEpiStats) instead of hipBLASLt + a bn_moments pass: ResNet-50 bs256 12,896-12,917 vs
    12,695-12,775 img/s interleaved (profiles/README.md r3). XDDP_DEEP_K_OWN=0: hipBLASLt (A/B
    switch; a block output pending on such a conv is resolved by its own apply pass either way —
    absorbing it on the register-staged GEMM measured no gain)."""
    return os.environ.get("XDDP_DEEP_K_OWN", "1") != "0"


def _same_tensor(a, b) -> bool:
    return a is not None and b is not None and a.data_ptr() == b.data_ptr() and a.shape == b.shape and \
        a.stride() == b.stride()


class _Conv1x1BN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, weight, bias, running_mean, running_var, nbt, momentum, cma, eps, residual, relu, dual,
                stride, link_out, link_x, link_res, link_in, link_ds, defer, res_defer, pend_in, pend_out):
        C = load()
        ctx.set_materialize_grads(False)
        dma = _c1_dma(x, w)
        if pend_in is not None:
            # x is a pending BN apply (PendingApply): computed in this GEMM's prologue and stored
            # into x's storage by the N-tile-0 blocks (the caller checked _absorbs)
            p = pend_in
            y, part = C.conv1x1_gemm(p.y, w, 1, p.ss, True, pro_out=p.out, pro_bits=p.bits, pro_res=p.res,
                                     pro_res_ss=p.rss, pro_nbt=p.nbt, pro_res_nbt=p.rnbt)
            p.done = True
            p.y = p.res = p.ss = p.rss = None
        elif dma:  # deep-K / few-tile shapes: the 3-stage LDS-DMA pipeline (csrc/kernels/conv3x3.hip TAPS=1)
            y, part = C.conv1x1_dma_forward(x, w, stride, True)
        elif stride == 1 and x.size(1) >= _c1_blas_min_k() and (w.size(0) % 128 == 0 or not _deep_k_own()):
            # deep-K, few-tile layers (ResNet-50 layer3/4 conv1: K = 1024 / 2048, 400-800 output
            # tiles): the register-staged GEMM waits a memory latency per 64-deep K step there;
            # the LDS-DMA GEMM (gemm.hip) runs them with the statistics in its epilogue (or
            # hipBLASLt + a statistics pass, XDDP_DEEP_K_OWN=0)
            B, K, H, W = x.shape
            if _deep_k_own():  # the own LDS-DMA GEMM with the statistics epilogue (gemm.hip kEpiStats)
                y, part = C.gemm_nt(x.permute(0, 2, 3, 1).reshape(-1, K), w.view(w.size(0), K), None, 5)
                y = y.view(B, H, W, -1).permute(0, 3, 1, 2)
                dma = True  # (group-minor partials, as the LDS-DMA kernels leave them)
            else:
                y = torch.mm(x.permute(0, 2, 3, 1).reshape(-1, K), w.view(w.size(0), K).t())
                y = y.view(B, H, W, -1).permute(0, 3, 1, 2)
                part = C.bn_moments(y).view(1, 3, -1)
        else:
            y, part = C.conv1x1_gemm(x, w, stride, None, True)
        M = y.numel() // y.size(1)
        mean, invstd, ss = C.bn_stats_from_partials(part, M, weight, bias, running_mean, running_var, nbt, momentum,
                                                    cma, eps, dma)
        keep_mask = relu and residual is not None
        if defer is not None:  # the consumer applies this BN (DeferredBN): output the raw conv output
            defer.ss, defer.nbt = ss, nbt
            out, bits = y, None
        elif pend_out is not None and keep_mask:  # the next block's conv1 applies it (PendingApply)
            p = _new_pending(y, ss, residual, res_defer.ss if res_defer is not None else None, nbt,
                             res_defer.nbt if res_defer is not None else None, True)
            pend_out.append(p)
            out, bits = p.out, p.bits
        elif res_defer is not None:
            out, bits = C.bn_apply(y, ss, residual, relu, keep_mask, nbt, res_defer.ss, res_defer.nbt)
        else:
            out, bits = C.bn_apply(y, ss, residual, relu, keep_mask, nbt)
        ctx.relu, ctx.has_res, ctx.stride = relu, residual is not None, stride
        ctx.save_for_backward(x, w, y, bits if keep_mask else None, weight, mean, invstd, ss)
        ctx.link_out, ctx.link_x, ctx.link_res, ctx.link_in = link_out, link_x, link_res, link_in
        ctx.link_ds = link_ds
        if link_out is not None:
            if keep_mask and dual:
                link_out.y, link_out.bits, link_out.mean = y, bits, mean
            else:
                ctx.link_out = None
        if dual:  # two consumers: gradients arrive separately and are summed in the BN backward kernel
            return out, out.view_as(out)
        return out

    @staticmethod
    def backward(ctx, dout, dout2=None):
        try:
            return _Conv1x1BN._backward(ctx, dout, dout2)
        finally:
            if ctx.link_x is not None:
                ctx.link_x.c1_done = True

    @staticmethod
    def _backward(ctx, dout, dout2):
        C = load()
        x, w, y, bits, weight, mean, invstd, ss = ctx.saved_tensors
        lo = ctx.link_out
        epi_part = None
        if lo is not None:  # the next block's conv1 took (or left) the identity-path gradient
            if lo.part is not None:
                if dout2 is None and _same_tensor(dout, lo.g):
                    epi_part = lo.part
                elif dout2 is not None:  # an extra consumer of the residual alias
                    dout = dout2 if dout is None else dout + dout2
                dout2 = None  # (the identity-path gradient is inside g already)
            elif lo.add is not None:  # left unconsumed: back to a plain second gradient
                add = _expand_s2(lo.add, y) if lo.add_s2 else lo.add
                dout2 = add if dout2 is None else dout2 + add
            lo.y = lo.bits = lo.mean = lo.add = lo.part = lo.g = None
            lo.add_s2 = False
        if dout is None:
            dout, dout2 = dout2, None
        if dout is None:
            return (None,) * 23
        need_bn_w = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        s = ctx.stride
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        need_dres = ctx.has_res and ctx.needs_input_grad[10]
        if epi_part is not None:
            # dout is g = mask·(d conv1 + d identity) from the next block's conv1 GEMM epilogue,
            # which also reduced this BN's backward partials
            M = y.numel() // y.size(1)
            coef, dw_bn, db_bn = C.bn_backward_from_partials(epi_part, M, weight, mean, invstd, need_bn_w)
            g = dout
            dres = g if need_dres else None
            dx = dw = None
            if s == 1 and need_x and need_w and _bwd_fused_ok(ctx, C, w):
                dx, dw = C.conv1x1_bwd_fused(g, y, coef, x, w)
            if s == 1 and need_x and dx is None and _dgrad_gemm():
                dx = _dgrad_in(ctx, C, g, w, coef, y)
            if need_w and dw is None and s == 1 and _wgrad_gemm():
                dw = C.conv1x1_wgrad(g, x, 1, w, y, coef)
            if (need_x and dx is None) or (need_w and dw is None):
                v = lambda i: coef[i].view(1, -1, 1, 1)  # noqa: E731
                dy = (v(0) * g.float() + v(1) * y.float() + v(2)).to(g.dtype).contiguous(
                    memory_format=torch.channels_last)
                gx, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0],
                                                                1, [need_x and dx is None, need_w and dw is None,
                                                                    False])
                dx = gx if dx is None else dx
                dw = gw if dw is None else dw
            return _grads(ctx, dx, dw, dw_bn, db_bn, dres)
        if (s == 1 and need_x and need_w and _bwd_prologue() and _dgrad_gemm() and _wgrad_gemm()
                and (need_dres or (dout2 is None and bits is None and (not ctx.relu or _bwd_prologue_masked())))):
            # BN-backward elementwise pass folded into both GEMMs: dY = k1·g + k2·y + k3' is formed
            # while staging (g = the masked gradient the reduce pass writes as d(residual), or the
            # incoming gradient itself, masked in the prologue by relu(y·scale + shift) > 0 when
            # the BN has a ReLU), so dY is never written to and re-read from HBM
            coef, dw_bn, db_bn, dres = C.bn_backward(dout, y, None, weight, mean, invstd, ss, ctx.relu, need_dres,
                                                     need_bn_w, dout2, bits, True)
            g = dres if need_dres else dout.contiguous(memory_format=torch.channels_last)
            if _bwd_fused_ok(ctx, C, w):
                dx, dw = C.conv1x1_bwd_fused(g, y, coef, x, w)
            else:
                dx = _dgrad_in(ctx, C, g, w, coef, y)
                dw = C.conv1x1_wgrad(g, x, 1, w, y, coef)
            return _grads(ctx, dx, dw, dw_bn, db_bn, dres)
        dy, dw_bn, db_bn, dres = C.bn_backward(dout, y, None, weight, mean, invstd, ss, ctx.relu, need_dres,
                                               need_bn_w, dout2, bits)
        dx = dw = None
        if need_x and s == 1 and _dgrad_gemm():
            # dX[M, K] = dY[M, N] · W[N, K] is the same NT GEMM on (dY, Wᵀ): 35 % less time than
            # MIOpen's 1x1 dgrad over the ResNet-50 shapes (scripts/dgrad_bench.py)
            lx = ctx.link_x
            if lx is not None and lx.add is not None and lx.y is not None and _epi():
                # the previous block's output gradient: dX + identity-path gradient (or the
                # downsample's compact one at the even pixels), masked by its ReLU and reduced into
                # its BN-backward partials in this GEMM's epilogue
                dx, lx.part = C.conv1x1_gemm(dy, w, 1, None, False, None, True, lx.add, lx.y, lx.bits, lx.mean, None,
                                             2 if lx.add_s2 else 1)
                lx.add, lx.g, lx.add_s2 = None, dx, False
            else:
                dx = _dgrad_in(ctx, C, dy, w, None, None)
            need_x = False
        elif need_x and s == 2 and _dgrad_gemm():
            # strided 1x1 input gradient: only the stride-2 pixels receive dY·W. The compact product
            # is one stride-1 GEMM; linked (downsample of a bottleneck whose input is the previous
            # block's output) it goes to conv1's epilogue, else it is scattered into zeros
            dxe = _dgrad(C, dy, w, None, None)
            ld = ctx.link_ds
            if ld is not None and ld.y is not None and ld.add is None and not ld.c1_done and _epi():
                ld.add, ld.add_s2 = dxe, True
            else:
                dx = _expand_s2(dxe, x)
            need_x = False
        if need_w and _wgrad_gemm():
            # dW[N, K] = dYᵀ[N, M] · X[M, K] (strided pixel rows for the downsample): 14 % less
            # time than MIOpen's 1x1 wgrad over the ResNet-50 shapes (scripts/dgrad_bench.py)
            dw = C.conv1x1_wgrad(dy, x, s, w)
            need_w = False
        if need_x or need_w:
            gx, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                            [need_x, need_w, False])
            dx = gx if need_x else dx
            dw = gw if need_w else dw
        return _grads(ctx, dx, dw, dw_bn, db_bn, dres)


def _grads(ctx, dx, dw, dw_bn, db_bn, dres):
    """The 23 input gradients of _Conv1x1BN; a linked residual gradient goes to the consumer link."""
    if dres is not None and ctx.link_res is not None:
        ctx.link_res.add, dres = dres, None
    return (dx, dw, dw_bn if ctx.needs_input_grad[2] else None, db_bn if ctx.needs_input_grad[3] else None,
            None, None, None, None, None, None, dres if ctx.has_res else None, None, None, None, None, None, None,
            None, None, None, None, None, None)


def _bwd_fused_ok(ctx, C, w) -> bool:
    """Input and weight gradient of a stride-1 1x1 conv from one staging of its BN-backward dY
    (``conv1x1_bwd_fused``): the ResNet-50 layer-1 shapes (N, K) = (256, 64), (64, 256), where
    both gradient kernels sit at the HBM roofline reading the same two tensors.
    XDDP_CONV_BWD_FUSED=0 keeps the two separate kernels (A/B switch)."""
    if os.environ.get("XDDP_CONV_BWD_FUSED", "1") == "0":
        return False
    if ctx.link_in is not None and _epi() and os.environ.get("XDDP_CONV_EPI2", "0") == "1":
        return False  # the dgrad epilogue has extra work to do there
    return (w.dtype == torch.bfloat16 and w.is_contiguous() and w.shape[2] == 1 and w.shape[3] == 1
            and C.conv1x1_bwd_fused_supported(w.shape[0], w.shape[1]))


def _dgrad_in(ctx, C, g, w, coef, y):
    """Stride-1 input gradient; with a BNReLULink on the input, also the producer's masked BN-backward
    partials (epilogue second form)."""
    li = ctx.link_in
    # XDDP_CONV_EPI2=1 opts in. Off by default: measured 10,534 vs 10,808 img/s (ResNet-50 bs256,
    # MI355X) with 45 spilled registers at 2 blocks/CU, and still 11,746 vs 12,092-12,170 at one
    # block/CU without spills (the EPI default since): the conv3 input-gradient GEMM re-reads y2
    # per output tile, costing more than BN2's separate reduce pass.
    if li is None or not _epi() or os.environ.get("XDDP_CONV_EPI2", "0") != "1":
        return _dgrad(C, g, w, coef, y)
    dx, li.part = C.conv1x1_gemm(g, w, 1, coef, False, y, True, None, li.y, None, li.mean, li.ss)
    li.g = dx
    return dx


class _Conv3x3BNReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, weight, bias, running_mean, running_var, nbt, momentum, cma, eps, stride, link, pend_out):
        C = load()
        ctx.set_materialize_grads(False)
        y, part = C.conv3x3_forward(x, w, stride, True)
        M = y.numel() // y.size(1)
        mean, invstd, ss = C.bn_stats_from_partials(part, M, weight, bias, running_mean, running_var, nbt, momentum,
                                                    cma, eps, True)
        if pend_out is not None:  # conv3's GEMM prologue applies it (PendingApply)
            p = _new_pending(y, ss, None, None, nbt, None, False)
            pend_out.append(p)
            out = p.out
        else:
            out, _ = C.bn_apply(y, ss, None, True, False, nbt)
        ctx.stride = stride
        ctx.save_for_backward(x, w, y, weight, mean, invstd, ss)
        ctx.link = link
        if link is not None:
            link.y, link.mean, link.ss = y, mean, ss
        return out

    @staticmethod
    def backward(ctx, dout):
        if dout is None:
            return (None,) * 13
        C = load()
        x, w, y, weight, mean, invstd, ss = ctx.saved_tensors
        need_bn_w = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        lk = ctx.link
        part = lk.part if (lk is not None and _same_tensor(dout, lk.g)) else None
        if lk is not None:
            lk.y = lk.mean = lk.ss = lk.part = lk.g = None
        if part is not None:
            # dout is already masked by this BN's ReLU and its backward partials were reduced by
            # conv3's input-gradient epilogue: only the finalize + the elementwise pass remain
            M = y.numel() // y.size(1)
            coef, dw_bn, db_bn = C.bn_backward_from_partials(part, M, weight, mean, invstd, need_bn_w, False)
            dy = C.bn_backward_elem(dout, y, mean, coef)
        else:
            # ReLU mask recomputed from y·scale + shift inside the BN backward (no mask tensor kept)
            dy, dw_bn, db_bn, _ = C.bn_backward(dout.contiguous(memory_format=torch.channels_last), y, None, weight,
                                                mean, invstd, ss, True, False, need_bn_w, None, None)
        s = ctx.stride
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        if need_x and s == 1:
            dx = C.conv3x3_forward(dy, C.conv3x3_rot_weight(w), 1, False)[0]
            need_x = False
        elif need_x and s == 2 and _dgrad3_s2():
            # four phase grids of the strided dX, 1/2/2/4 taps each, one launch (conv3x3.hip DG2)
            dx = C.conv3x3_dgrad_s2(dy, C.conv3x3_rot_weight(w), x.size(2), x.size(3))
            need_x = False
        if need_w and _wgrad3() and (s == 1 or os.environ.get("XDDP_CONV3X3_WGRAD_S2", "1") != "0"):
            # 8x8 output patches sharing one staged X halo across the 9 taps (conv3x3_wgrad.hip):
            # 96-98 us vs MIOpen's 120-182 us per stride-1 ResNet-50 shape (bs256); at stride 2 the
            # phase-split halo is shared by 128 output channels (8 waves): 127 / 118 / 108 vs
            # MIOpen's 150 / 139 / 145 us (profiles/r4_s2_bwd_vs_miopen.txt; XDDP_CONV3X3_WGRAD_S2=0
            # hands it back to MIOpen)
            dw = C.conv3x3_wgrad_patch(dy, x, s, w)
            need_w = False
        if need_x or need_w:
            gx, gw, _ = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [1, 1], [1, 1], False, [0, 0], 1,
                                                            [need_x, need_w, False])
            dx = gx if need_x else dx
            dw = gw if need_w else dw
        return (dx, dw, dw_bn if ctx.needs_input_grad[2] else None, db_bn if ctx.needs_input_grad[3] else None,
                None, None, None, None, None, None, None, None, None)


def _dgrad(C, g, w, coef, y):
    """dX = dY · W on the MFMA GEMM, W read K-major through transposed LDS reads (no transposed
    weight copy; XDDP_GEMM_WT=0 makes the copy instead, A/B switch)."""
    if os.environ.get("XDDP_GEMM_WT", "1") != "0":
        return C.conv1x1_gemm(g, w, 1, coef, False, y, True)[0]
    n_out, k_in = w.shape[0], w.shape[1]
    wt = w.reshape(n_out, k_in).t().contiguous().view(k_in, n_out, 1, 1)
    return C.conv1x1_gemm(g, wt, 1, coef, False, y)[0]


def _conv3x3() -> bool:
    """XDDP_CONV3X3=0 sends the bottleneck 3x3 conv back to MIOpen + separate BN (A/B switch)."""
    return os.environ.get("XDDP_CONV3X3", "1") != "0"


def _dgrad3_s2() -> bool:
    """The stride-2 3x3 input gradient as four phase GEMMs on the 4-phase LDS-DMA GEMM pipeline
    (gemm.hip DGS2: 1/2/2/4 taps per phase, written straight to the strided pixels, no zero-fill):
    142 / 97 / 86 us vs MIOpen's 170 / 141 / 136 us on the three ResNet-50 bs256 shapes
    (profiles/r4_s2_bwd_vs_miopen.txt). XDDP_CONV3X3_DGRAD_S2=0 hands it back to MIOpen."""
    return os.environ.get("XDDP_CONV3X3_DGRAD_S2", "1") != "0"


def _epi() -> bool:
    """XDDP_CONV_EPI=0 keeps the previous block's BN-backward reduce pass separate instead of
    folding it into the next block's conv1 input-gradient GEMM epilogue (A/B switch)."""
    return os.environ.get("XDDP_CONV_EPI", "1") != "0"


def _wgrad3() -> bool:
    """XDDP_CONV3X3_WGRAD=0 sends the bottleneck 3x3 weight gradient back to MIOpen (A/B switch)."""
    return os.environ.get("XDDP_CONV3X3_WGRAD", "1") != "0"


def _dgrad_gemm() -> bool:
    """XDDP_CONV_DGRAD_GEMM=0 sends the stride-1 input gradient back to MIOpen (A/B switch)."""
    return os.environ.get("XDDP_CONV_DGRAD_GEMM", "1") != "0"


def _bwd_prologue() -> bool:
    """XDDP_CONV_BWD_PROLOGUE=0 materializes the BN-backward gradient instead of folding it into
    the stride-1 input/weight-gradient GEMMs (A/B switch)."""
    return os.environ.get("XDDP_CONV_BWD_PROLOGUE", "1") != "0"


def _bwd_prologue_masked() -> bool:
    """XDDP_CONV_BWD_PROLOGUE_MASK=1 also folds the BN+ReLU (recomputed-mask) backward of the
    bottleneck's conv1 into its gradient GEMMs. Off by default: that input-gradient GEMM re-reads
    its A operand once per output-channel tile (C_in / 128 of them), so reading two sources there
    costs more than the skipped pass saves (10,378 vs 10,436 img/s, ResNet-50 bs256)."""
    return os.environ.get("XDDP_CONV_BWD_PROLOGUE_MASK", "0") == "1"


def _wgrad_gemm() -> bool:
    """XDDP_CONV_WGRAD_GEMM=0 sends the weight gradient back to MIOpen (A/B switch)."""
    return os.environ.get("XDDP_CONV_WGRAD_GEMM", "1") != "0"


def conv_bn_supported(x: torch.Tensor, conv: nn.Conv2d, bn: nn.Module) -> bool:
    """Whether the fused kernels cover this (input, conv, bn) triple; otherwise use conv then bn."""
    k = conv.kernel_size
    geometry = ((k == (1, 1) and conv.padding == (0, 0))
                or (k == (3, 3) and conv.padding == (1, 1) and conv.stride[0] in (1, 2)
                    and conv.weight.is_contiguous(memory_format=torch.channels_last)))
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0
            and geometry and conv.dilation == (1, 1)
            and conv.groups == 1 and conv.bias is None and conv.stride[0] == conv.stride[1]
            and conv.weight.dtype == torch.bfloat16 and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0
            and bn.training and bn.track_running_stats and bn.momentum is not None
            and getattr(bn, "fuses_relu", False))


def conv3x3_bn_relu(x: torch.Tensor, conv: nn.Conv2d, bn: nn.Module, pending: bool = False):
    """``relu(bn(conv3x3(x)))`` on the implicit-GEMM kernel with BN statistics from its epilogue.

    pending: the caller feeds the result straight to a 1x1 conv through :func:`conv1x1_bn_act`,
    which applies this BN in its GEMM prologue (:class:`PendingApply`)."""
    resolve(x)
    if not (_conv3x3() and conv.kernel_size == (3, 3) and conv_bn_supported(x, conv, bn)):
        return bn(conv(x), relu=True)
    link = BNReLULink(None, None, None) if _epi() else None
    pend = [] if (pending and _pending_apply()) else None
    out = _Conv3x3BNReLU.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                               bn.num_batches_tracked, float(bn.momentum), False, float(bn.eps), int(conv.stride[0]),
                               link, pend)
    if link is not None:
        out._xddp_bnr = link
    if pend:
        out._xddp_pend = pend[0]
    return out


def conv1x1_bn_act(x: torch.Tensor, conv: nn.Conv2d, bn: nn.Module, residual: Optional[torch.Tensor] = None,
                   relu: bool = False, dual_output: bool = False, link_x: Optional[EpiLink] = None,
                   link_res: Optional[EpiLink] = None, link_ds: Optional[EpiLink] = None, defer: bool = False,
                   pending: bool = False):
    """``relu(bn(conv(x)) [+ residual])`` with BN statistics from the conv epilogue when supported.

    link_x / link_res: the :class:`EpiLink` of the block output that is this conv's input /
    this op's residual (``x._xddp_epi`` of a dual output); with dual_output and residual + ReLU
    the returned output carries a fresh link for the next block. link_ds: this stride-2 conv is
    the downsample sharing its input with a linked conv1 (compact input gradient to the link).
    defer: return the raw conv output and leave this BN's apply to the consumer that takes the
    result as its ``residual`` (DeferredBN; only for a BN without ReLU or residual).
    pending: leave this op's apply (residual + ReLU form) to the next block's conv1, which must be
    this output's first reader (:class:`PendingApply`). A pending ``x`` is absorbed into this conv's
    GEMM prologue when the GEMM path allows it, else resolved first."""
    resolve(residual)
    pend_in = getattr(x, "_xddp_pend", None)
    if pend_in is not None and (pend_in.done or not _absorbs(x, conv, bn, pend_in)):
        pend_in.resolve()
        pend_in = None
    res_defer = _deferred(residual)
    if conv.kernel_size != (1, 1) or not conv_bn_supported(x, conv, bn) or (residual is not None and not (
            residual.shape[0] == x.shape[0] and residual.dtype == x.dtype
            and residual.is_contiguous(memory_format=torch.channels_last))):
        if pend_in is not None:
            pend_in.resolve()
        if res_defer is not None:
            residual = _ApplyDeferred.apply(residual, res_defer.ss, res_defer.nbt)
        return bn(conv(x), residual=residual, relu=relu, dual_output=dual_output)
    dfr = DeferredBN() if (defer and residual is None and not relu and not dual_output) else None
    link_out = EpiLink() if (dual_output and residual is not None and relu and _epi()) else None
    link_in = getattr(x, "_xddp_bnr", None) if conv.stride[0] == 1 else None
    pend_out = [] if (pending and dual_output and residual is not None and relu and _pending_apply()) else None
    out = _Conv1x1BN.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                           bn.num_batches_tracked, float(bn.momentum), False, float(bn.eps), residual, relu,
                           dual_output, int(conv.stride[0]), link_out, link_x, link_res, link_in,
                           link_ds if conv.stride[0] == 2 else None, dfr, res_defer, pend_in, pend_out)
    if dfr is not None:
        out._xddp_bnss = dfr
    if link_out is not None:
        out[0]._xddp_epi = link_out
    if pend_out:  # both aliases: whichever a consumer reads first resolves it
        out[0]._xddp_pend = out[1]._xddp_pend = pend_out[0]
    return out


def _absorbs(x, conv, bn, p) -> bool:
    """Can this 1x1 conv's forward GEMM apply the pending BN in its prologue? Its register-staged
    GEMM path only (stride 1; not the LDS-DMA or hipBLASLt deep-K forwards), and the pending form
    must match the tensor (C, 8-channel chunks)."""
    return (conv.kernel_size == (1, 1) and conv.stride[0] == 1 and conv_bn_supported(x, conv, bn)
            and not _c1_dma(x, conv.weight) and x.size(1) < _c1_blas_min_k()
            and p.out.data_ptr() == x.data_ptr() and p.out.shape == x.shape)
