"""Pre-norm transformer encoder block (ViT-L/16, BASELINE.json config 4) as one autograd node.

    x1 = x  + proj(attn(qkv(LN1(x))))          out = x1 + fc2(gelu(fc1(LN2(x1))))

PyTorch's autograd graph of this block spends ~25 % of a ViT-L/16 step outside the GEMMs and
attention (rocprof, ``profiles/r2_transformers_kernel_top.txt``): two residual adds forward and
two backward, four bias-gradient reductions, the GELU backward, and the zero-fill + copy +
add that ``select`` backward uses to assemble the packed q/k/v gradient. Here:

* forward: LN1 also writes ``xb = x + b_proj`` and LN2 ``x1b = x1 + b_fc2``; each residual sum is
  then the beta = 1 GEMM ``xb += o·Wprojᵀ`` (hipBLASLt reads C in its epilogue) — no add passes;
* backward: fc2's input-gradient GEMM forms dh = (g·W_2)·gelu'(h) and Σ dh (fc1's bias gradient)
  in its epilogue (own GEMM; with hipBLASLt ``bias_grad`` does it in one pass after the GEMM);
  LN2's backward adds the residual gradient and also sums both residual gradients (the bias
  gradients of fc2 and of the out projection); LN1's backward adds its residual gradient;
  the flash-attention backward writes dq/dk/dv straight into one packed [B, S, 3, H, Dh] buffer,
  whose column sums are the qkv bias gradient.

Parameters, state_dict and module structure are the unfused ``EncoderBlock``'s; the unfused
path stays the fallback (CPU, non-bf16, autocast, ``XDDP_FUSED_BLOCK=0``).
Reference: the model the reference trains is a torchvision classifier driven by
``ref:dpp.py:44-55``; this block is the ViT-L/16 config of BASELINE.json.
"""
from __future__ import annotations

import math
import os

import torch

from .._native import load
from .linear import _dw, own_gemm_mode

__all__ = ["encoder_block", "encoder_block_supported"]


def encoder_block_supported(x: torch.Tensor, blk) -> bool:
    if os.environ.get("XDDP_FUSED_BLOCK", "1") == "0" or os.environ.get("XDDP_FLASH_ATTN", "1") == "0":
        return False
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 3) or torch.is_autocast_enabled():
        return False
    D = x.shape[-1]
    heads = blk.self_attention.heads
    if D % 8 or D % heads or D // heads not in (64, 128):
        return False
    fc1, fc2 = blk.mlp[0], blk.mlp[2]
    params = [blk.ln_1.weight, blk.ln_1.bias, blk.ln_2.weight, blk.ln_2.bias,
              blk.self_attention.in_proj.weight, blk.self_attention.in_proj.bias,
              blk.self_attention.out_proj.weight, blk.self_attention.out_proj.bias,
              fc1.weight, fc1.bias, fc2.weight, fc2.bias]
    if any(p is None or p.dtype != torch.bfloat16 or not p.is_cuda for p in params):
        return False
    return fc1.out_features % 8 == 0


class _EncoderBlockFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, ln1_w, ln1_b, w_qkv, b_qkv, w_o, b_o, ln2_w, ln2_b, w_1, b_1, w_2, b_2, heads, eps1, eps2):
        C = load()
        B, S, D = x.shape
        dh = D // heads
        scale = 1.0 / math.sqrt(dh)
        x2 = x.reshape(-1, D).contiguous()
        own = _own_gemm(D, w_1.shape[0], backward=False)
        y1, mean1, rstd1, xb = C.ln_forward(x2, ln1_w, ln1_b, eps1, False, b_o)
        qkv = C.gemm_nt(y1, w_qkv, b_qkv, 1)[0] if own else torch.addmm(b_qkv, y1, w_qkv.t())
        q5 = qkv.view(B, S, 3, heads, dh)
        o, lse = C.flash_attn_forward(q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], False, scale)
        o2 = o.view(-1, D)
        if own:  # x + b_o + o·W_oᵀ, the residual added in the GEMM epilogue, in place
            x1 = C.gemm_nt(o2, w_o, None, 3, xb, xb)[0]
        else:
            x1 = xb.addmm_(o2, w_o.t())
        y2, mean2, rstd2, x1b = C.ln_forward(x1, ln2_w, ln2_b, eps2, False, b_2)
        if own:  # fc1 + bias + GELU in one GEMM epilogue: h (for dGELU) and a = gelu(h)
            h, a = C.gemm_nt(y2, w_1, b_1, 2)
            out = C.gemm_nt(a, w_2, None, 3, x1b, x1b)[0]  # x1 + b_2 + a·W_2ᵀ
        else:
            h = torch.addmm(b_1, y2, w_1.t())
            a = C.gelu_forward(h)
            out = x1b.addmm_(a, w_2.t())
        ctx.save_for_backward(x2, ln1_w, mean1, rstd1, y1, w_qkv, b_qkv, qkv, o, lse, w_o, b_o, x1, ln2_w, mean2,
                              rstd2, y2, w_1, b_1, h, a, w_2, b_2)
        ctx.shape, ctx.heads, ctx.scale = (B, S, D), heads, scale
        ctx.params = (w_qkv, w_o, w_1, w_2)  # (the parameter objects: their registered gradient targets)
        return out.view(B, S, D)

    @staticmethod
    def backward(ctx, g):
        C = load()
        (x2, ln1_w, mean1, rstd1, y1, w_qkv, b_qkv, qkv, o, lse, w_o, b_o, x1, ln2_w, mean2, rstd2, y2, w_1, b_1, h, a,
         w_2, b_2) = ctx.saved_tensors
        B, S, D = ctx.shape
        heads, dh = ctx.heads, D // ctx.heads
        g2 = g.reshape(-1, D).contiguous()
        # MLP
        if _own_gemm(D, w_1.shape[0], backward=True):  # dh = (g·W_2)·gelu'(h), Σ dh in the GEMM epilogue
            w_2t = C.transpose16(w_2) if w_2.is_contiguous() else w_2.t().contiguous()  # (LDS-tiled transpose)
            dhid, db_1 = C.gemm_nt(g2, w_2t, b_1, 4, h)
        else:
            db_1, dhid = C.bias_grad(torch.mm(g2, w_2), h, b_1)
        p_qkv, p_o, p_1, p_2 = ctx.params
        # weight gradients straight into the DDP bucket views when registered (ops/linear.py _dw)
        dw_2 = _dw(g2, a, p_2)
        dy2 = torch.mm(dhid, w_1)
        dw_1 = _dw(dhid, y2, p_1)
        # LN2 + residual: g1 = g2 + LN2ᵀ(dy2); Σ g2 = fc2's bias grad, Σ g1 = the out projection's
        g1, dln2_w, dln2_b, db_2, db_o = C.ln_backward(dy2, x1, ln2_w, mean2, rstd2, False, True, True, g2)
        # attention
        do = torch.mm(g1, w_o)
        dw_o = _dw(g1, o.view(-1, D), p_o)
        dqkv = torch.empty_like(qkv)
        d5, q5 = dqkv.view(B, S, 3, heads, dh), qkv.view(B, S, 3, heads, dh)
        # (with bias_like, the one-block ViT kernel also returns Σ rows of dQ, dK, dV = the qkv bias
        # gradient from its own accumulators; None where it does not apply)
        db_qkv = C.flash_attn_backward(do.view(B, S, heads, dh), q5[:, :, 0], q5[:, :, 1], q5[:, :, 2], o, lse,
                                       False, ctx.scale, d5[:, :, 0], d5[:, :, 1], d5[:, :, 2], b_qkv)[3]
        if db_qkv is None:
            db_qkv, _ = C.bias_grad(dqkv, None, b_qkv)
        dy1 = torch.mm(dqkv, w_qkv)
        dw_qkv = _dw(dqkv.view(-1, 3 * D), y1, p_qkv)
        # LN1 + residual: dx = g1 + LN1ᵀ(dy1)
        dx, dln1_w, dln1_b, _, _ = C.ln_backward(dy1, x2, ln1_w, mean1, rstd1, False, True, True, g1)
        return (dx.view(B, S, D), dln1_w, dln1_b, dw_qkv, db_qkv, dw_o, db_o, dln2_w, dln2_b, dw_1, db_1, dw_2, db_2,
                None, None, None)


def _own_gemm(D: int, hidden: int, backward: bool) -> bool:
    """Own LDS-DMA MFMA GEMM (csrc/kernels/gemm.hip) for this block? Forward projections (bias,
    bias+GELU and residual epilogues) only with XDDP_OWN_GEMM=1; fc2's input gradient with the
    dGELU + bias-gradient epilogue also with the default ``bwd`` (ops/linear.own_gemm_mode)."""
    mode = own_gemm_mode()
    if mode == "0" or (mode == "bwd" and not backward):
        return False
    return D % 128 == 0 and hidden % 128 == 0 and (3 * D) % 128 == 0


def encoder_block(x: torch.Tensor, blk) -> torch.Tensor:
    """Run ``blk`` (a ``models.vit.EncoderBlock``) on ``x: [B, S, D]`` as one fused autograd node."""
    att, fc1, fc2 = blk.self_attention, blk.mlp[0], blk.mlp[2]
    return _EncoderBlockFn.apply(x, blk.ln_1.weight, blk.ln_1.bias, att.in_proj.weight, att.in_proj.bias,
                                 att.out_proj.weight, att.out_proj.bias, blk.ln_2.weight, blk.ln_2.bias,
                                 fc1.weight, fc1.bias, fc2.weight, fc2.bias, att.heads, float(blk.ln_1.eps),
                                 float(blk.ln_2.eps))
