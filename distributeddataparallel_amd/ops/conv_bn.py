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
import weakref
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


# Stride-1 1x1 forwards with Cin >= this run the GEMM on the LDS-DMA kernel with the statistics
# epilogue (gemm.hip kEpiStats): the register-staged GEMM waits a memory latency per 64-deep K step,
# which dominates the deep-K, few-tile layers (ResNet-50 layer3/4 conv1: K = 1024 / 2048).
# (Measured and removed in r5's switch cleanup: hipBLASLt + a statistics pass there, 12,695-12,775 vs
# 12,896-12,917 img/s; the 3-stage LDS-DMA kernel for every 1x1 forward, 11,508-11,625 vs 11,662.)
_DEEP_K = 1024


def _same_tensor(a, b) -> bool:
    return a is not None and b is not None and a.data_ptr() == b.data_ptr() and a.shape == b.shape and \
        a.stride() == b.stride()


class _Conv1x1BN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, weight, bias, running_mean, running_var, nbt, momentum, cma, eps, residual, relu, dual,
                stride, link_out, link_x, link_res, link_ds, defer, res_defer, pend_in, pend_out):
        C = load()
        ctx.set_materialize_grads(False)
        dma = False
        if pend_in is not None:
            # x is a pending BN apply (PendingApply): computed in this GEMM's prologue and stored
            # into x's storage by the N-tile-0 blocks (the caller checked _absorbs)
            p = pend_in
            y, part = C.conv1x1_gemm(p.y, w, 1, p.ss, True, pro_out=p.out, pro_bits=p.bits, pro_res=p.res,
                                     pro_res_ss=p.rss, pro_nbt=p.nbt, pro_res_nbt=p.rnbt)
            p.done = True
            p.y = p.res = p.ss = p.rss = None
        elif stride == 1 and x.size(1) >= _DEEP_K and w.size(0) % 128 == 0:
            # deep-K, few-tile layers: the LDS-DMA GEMM with the statistics epilogue (_DEEP_K)
            B, K, H, W = x.shape
            y, part = C.gemm_nt(x.permute(0, 2, 3, 1).reshape(-1, K), w.view(w.size(0), K), None, 5)
            y = y.view(B, H, W, -1).permute(0, 3, 1, 2)
            dma = True  # (group-minor partials, as the LDS-DMA kernels leave them)
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
        ctx.link_out, ctx.link_x, ctx.link_res = link_out, link_x, link_res
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
            return (None,) * 22
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
            if s == 1 and need_x and dx is None:
                dx = _dgrad(C, g, w, coef, y)
            if need_w and dw is None and s == 1:
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
        if s == 1 and need_x and need_w and (need_dres or (dout2 is None and bits is None and not ctx.relu)):
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
                dx = _dgrad(C, g, w, coef, y)
                dw = C.conv1x1_wgrad(g, x, 1, w, y, coef)
            return _grads(ctx, dx, dw, dw_bn, db_bn, dres)
        dy, dw_bn, db_bn, dres = C.bn_backward(dout, y, None, weight, mean, invstd, ss, ctx.relu, need_dres,
                                               need_bn_w, dout2, bits)
        dx = dw = None
        if need_x and s == 1:
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
                dx = _dgrad(C, dy, w, None, None)
            need_x = False
        elif need_x and s == 2:
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
        if need_w:
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
    """The 22 input gradients of _Conv1x1BN; a linked residual gradient goes to the consumer link."""
    if dres is not None and ctx.link_res is not None:
        ctx.link_res.add, dres = dres, None
    return (dx, dw, dw_bn if ctx.needs_input_grad[2] else None, db_bn if ctx.needs_input_grad[3] else None,
            None, None, None, None, None, None, dres if ctx.has_res else None, None, None, None, None, None, None,
            None, None, None, None, None)


def _bwd_fused_ok(ctx, C, w) -> bool:
    """Input and weight gradient of a stride-1 1x1 conv from one staging of its BN-backward dY
    (``conv1x1_bwd_fused``): the ResNet-50 layer-1 shapes (N, K) = (256, 64), (64, 256), where
    both gradient kernels sit at the HBM roofline reading the same two tensors."""
    return (w.dtype == torch.bfloat16 and w.is_contiguous() and w.shape[2] == 1 and w.shape[3] == 1
            and C.conv1x1_bwd_fused_supported(w.shape[0], w.shape[1]))


# The input gradients read the 180-degree-rotated, channel-swapped 3x3 weights. Each forward marks
# its weight stale; the first 3x3 backward of the step rotates every stale weight in ONE launch
# (conv3x3_rot_weights) instead of one small kernel per layer (16 per ResNet-50 step, ~5 us each).
# Staleness comes from the forward, not from the tensor version: fused optimizers write parameter
# memory without bumping it.
_ROT_PENDING: dict = {}  # id(w) -> weakref(w), marked by a forward, rotated by the next backward
_ROT_CACHE: dict = {}    # id(w) -> (weakref(w), data_ptr, rotated weight)


def _rot_mark(w):
    _ROT_PENDING[id(w)] = weakref.ref(w)
    _ROT_CACHE.pop(id(w), None)


def _rot_weight(C, w):
    hit = _ROT_CACHE.get(id(w))
    if hit is not None and hit[0]() is w and hit[1] == w.data_ptr():
        return hit[2]
    batch = [t for t in (r() for r in _ROT_PENDING.values()) if t is not None and t.device == w.device]
    if not any(t is w for t in batch):
        batch.append(w)
    for k in [k for k, e in _ROT_CACHE.items() if e[0]() is None]:  # weights that are gone
        del _ROT_CACHE[k]
    for t, r in zip(batch, C.conv3x3_rot_weights(batch)):
        _ROT_CACHE[id(t)] = (weakref.ref(t), t.data_ptr(), r)
        _ROT_PENDING.pop(id(t), None)
    return _ROT_CACHE[id(w)][2]


class _Conv3x3BNReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, weight, bias, running_mean, running_var, nbt, momentum, cma, eps, stride, pend_out):
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
        return out

    @staticmethod
    def backward(ctx, dout):
        if dout is None:
            return (None,) * 12
        C = load()
        x, w, y, weight, mean, invstd, ss = ctx.saved_tensors
        need_bn_w = weight is not None and (ctx.needs_input_grad[2] or ctx.needs_input_grad[3])
        # ReLU mask recomputed from y·scale + shift inside the BN backward (no mask tensor kept).
        # (r5: conv3's input-gradient epilogue reducing this BN's backward partials instead, the
        # kernel's EPI mask-recompute form, still lost: 12,940 vs 13,399 img/s interleaved.)
        dy, dw_bn, db_bn, _ = C.bn_backward(dout.contiguous(memory_format=torch.channels_last), y, None, weight,
                                            mean, invstd, ss, True, False, need_bn_w, None, None)
        s = ctx.stride
        need_x, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        dx = dw = None
        if need_x and s == 1:
            dx = C.conv3x3_forward(dy, _rot_weight(C, w), 1, False)[0]
        elif need_x:
            # four phase grids of the strided dX, 1/2/2/4 taps each, one launch (conv3x3.hip DG2):
            # 142 / 97 / 86 vs MIOpen's 170 / 141 / 136 us (profiles/r4_s2_bwd_vs_miopen.txt)
            dx = C.conv3x3_dgrad_s2(dy, _rot_weight(C, w), x.size(2), x.size(3))
        if need_w:
            # 8x8 output patches sharing one staged X halo across the 9 taps (conv3x3_wgrad.hip):
            # 96-98 us vs MIOpen's 120-182 us per stride-1 ResNet-50 shape (bs256); at stride 2 the
            # phase-split halo is shared by 128 output channels (8 waves): 127 / 118 / 108 vs
            # MIOpen's 150 / 139 / 145 us (profiles/r4_s2_bwd_vs_miopen.txt)
            dw = C.conv3x3_wgrad_patch(dy, x, s, w)
        return (dx, dw, dw_bn if ctx.needs_input_grad[2] else None, db_bn if ctx.needs_input_grad[3] else None,
                None, None, None, None, None, None, None, None)


def _dgrad(C, g, w, coef, y):
    """dX = dY · W on the MFMA GEMM, W read K-major through transposed LDS reads (no transposed
    weight copy)."""
    return C.conv1x1_gemm(g, w, 1, coef, False, y, True)[0]


def _conv3x3() -> bool:
    """XDDP_CONV3X3=0 sends the bottleneck 3x3 conv back to MIOpen + separate BN (A/B switch)."""
    return os.environ.get("XDDP_CONV3X3", "1") != "0"


def _epi() -> bool:
    """XDDP_CONV_EPI=0 keeps the previous block's BN-backward reduce pass separate instead of
    folding it into the next block's conv1 input-gradient GEMM epilogue (A/B switch)."""
    return os.environ.get("XDDP_CONV_EPI", "1") != "0"


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
    pend = [] if (pending and _pending_apply()) else None
    if torch.is_grad_enabled() and x.requires_grad:
        # only a forward whose backward reads the rotated weight (the input gradient) marks it:
        # no_grad forwards of other models (an EMA / teacher copy) would otherwise be rotated and
        # pinned every step
        _rot_mark(conv.weight)
    out = _Conv3x3BNReLU.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                               bn.num_batches_tracked, float(bn.momentum), False, float(bn.eps), int(conv.stride[0]),
                               pend)
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
    pend_out = [] if (pending and dual_output and residual is not None and relu and _pending_apply()) else None
    out = _Conv1x1BN.apply(x, conv.weight, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                           bn.num_batches_tracked, float(bn.momentum), False, float(bn.eps), residual, relu,
                           dual_output, int(conv.stride[0]), link_out, link_x, link_res,
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
            and x.size(1) < _DEEP_K
            and p.out.data_ptr() == x.data_ptr() and p.out.shape == x.shape)
