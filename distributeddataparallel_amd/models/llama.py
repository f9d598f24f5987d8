"""Llama-3 decoder (8B config) — BASELINE.json config 5 (Llama-3-8B bf16 pure DDP).

RMSNorm on xddp's fused kernel, rotary embeddings and the SwiGLU gate on fused HIP kernels
(``ops/transformer.py``: one pass each instead of ~10 / 3 PyTorch ops), grouped-query causal attention
on xddp's gfx950 flash-attention kernels (``ops/attention.py``: K/V heads shared, not repeated). Pure DDP sizing on MI355X: 8.03B
params → 16 GB bf16 params + 16 GB bf16 grads (bucket views) + 96 GB fp32 master/Adam ≈ 128 GB
of the 288 GB HBM3E, leaving room for activations (optionally checkpointed per layer).
``XDDP_FUSED_TRANSFORMER=0`` selects the PyTorch reference ops (A/B and parity tests).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.attention import flash_attention
from ..ops.layer_norm import FusedRMSNorm
from ..ops.linear import linear, multi_linear
from ..ops.transformer import rope, rope_reference, swiglu

__all__ = ["LlamaConfig", "Llama", "llama3_8b", "llama_tiny"]


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192
    checkpoint_activations: bool = False


def _fused() -> bool:
    return os.environ.get("XDDP_FUSED_TRANSFORMER", "1") != "0"


def _rope_table(head_dim, max_len, theta, device=None):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float32, device=device) / head_dim))
    t = torch.arange(max_len, dtype=torch.float32, device=device)
    f = torch.outer(t, inv)
    return torch.cos(f), torch.sin(f)


class Attention(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.h, self.kvh = cfg.n_heads, cfg.n_kv_heads
        self.hd = cfg.dim // cfg.n_heads
        self.wq = nn.Linear(cfg.dim, self.h * self.hd, bias=False)
        self.wk = nn.Linear(cfg.dim, self.kvh * self.hd, bias=False)
        self.wv = nn.Linear(cfg.dim, self.kvh * self.hd, bias=False)
        self.wo = nn.Linear(self.h * self.hd, cfg.dim, bias=False)

    def forward(self, x, cos, sin, residual=None):
        """Attention output; with ``residual`` (fused path) ``residual + attention`` (the skip
        connection added in the o-projection GEMM's epilogue)."""
        B, S, _ = x.shape
        rot = rope if _fused() else rope_reference
        # rotate in the projection's [B, S, H, Dh] layout, then move heads forward for attention
        if _fused():
            # q / k / v from one input with their input gradient accumulated in GEMMs (ops/linear.py
            # multi_linear); gfx950 flash attention in their [B, S, H, Dh] layout (GQA without
            # materialised K/V repeats; output already in the o-projection's layout); the skip
            # connection as the o-projection GEMM's beta = 1 operand
            q, k, v = multi_linear(x, self.wq.weight, self.wk.weight, self.wv.weight)
            q = rot(q.view(B, S, self.h, self.hd), cos, sin)
            k = rot(k.view(B, S, self.kvh, self.hd), cos, sin)
            v = v.view(B, S, self.kvh, self.hd)
            o = flash_attention(q, k, v, causal=True)
            return linear(o.reshape(B, S, -1), self.wo.weight, residual)
        q = rot(self.wq(x).view(B, S, self.h, self.hd), cos, sin)
        k = rot(self.wk(x).view(B, S, self.kvh, self.hd), cos, sin)
        v = self.wv(x).view(B, S, self.kvh, self.hd)
        q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
        if self.kvh != self.h:
            rep = self.h // self.kvh
            k = k.repeat_interleave(rep, dim=1)
            v = v.repeat_interleave(rep, dim=1)
        o = F.scaled_dot_product_attention(q, k, v, is_causal=True)
        out = self.wo(o.transpose(1, 2).reshape(B, S, -1))
        return out if residual is None else residual + out


class FeedForward(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.w1 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)
        self.w2 = nn.Linear(cfg.ffn_dim, cfg.dim, bias=False)
        self.w3 = nn.Linear(cfg.dim, cfg.ffn_dim, bias=False)

    def forward(self, x, residual=None):
        if _fused():
            return linear(swiglu(*multi_linear(x, self.w1.weight, self.w3.weight)), self.w2.weight, residual)
        out = self.w2(F.silu(self.w1(x)) * self.w3(x))
        return out if residual is None else residual + out


class Block(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.attention_norm = FusedRMSNorm(cfg.dim, eps=cfg.norm_eps)
        self.attention = Attention(cfg)
        self.ffn_norm = FusedRMSNorm(cfg.dim, eps=cfg.norm_eps)
        self.feed_forward = FeedForward(cfg)

    def forward(self, x, cos, sin):
        if _fused() and os.environ.get("XDDP_NORM_SKIP", "1") != "0":
            # each norm's input is also the skip connection: its gradient is summed in the norm's
            # backward kernel (ops/layer_norm.py rms_norm_with_skip), not by an add pass
            y, skip = self.attention_norm.forward_with_skip(x)
            x = self.attention(y, cos, sin, residual=skip)
            y, skip = self.ffn_norm.forward_with_skip(x)
            return self.feed_forward(y, residual=skip)
        x = self.attention(self.attention_norm(x), cos, sin, residual=x)
        return self.feed_forward(self.ffn_norm(x), residual=x)


class Llama(nn.Module):
    def __init__(self, cfg: LlamaConfig):
        super().__init__()
        self.cfg = cfg
        self.tok_embeddings = nn.Embedding(cfg.vocab_size, cfg.dim)
        self.layers = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layers)])
        self.norm = FusedRMSNorm(cfg.dim, eps=cfg.norm_eps)
        self.output = nn.Linear(cfg.dim, cfg.vocab_size, bias=False)
        # rotary tables stay fp32 whatever dtype the model is cast to: a plain attribute cache
        # per device, not a buffer (``.to(bfloat16)`` would round the angles' cos/sin, and DDP
        # would broadcast the tables before every forward)
        self._rope = {}
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)

    def _tables(self, device):
        key = str(device)
        if key not in self._rope:
            cos, sin = _rope_table(self.cfg.dim // self.cfg.n_heads, self.cfg.max_seq_len, self.cfg.rope_theta,
                                   device=device)
            self._rope[key] = (cos.contiguous(), sin.contiguous())
        return self._rope[key]

    def forward(self, tokens):
        cos, sin = self._tables(tokens.device)
        h = self.tok_embeddings(tokens)
        for blk in self.layers:
            if self.cfg.checkpoint_activations and self.training:
                h = torch.utils.checkpoint.checkpoint(blk, h, cos, sin, use_reentrant=False)
            else:
                h = blk(h, cos, sin)
        return linear(self.norm(h), self.output.weight) if _fused() else self.output(self.norm(h))


def llama3_8b(**kw):
    return Llama(LlamaConfig(**kw))


def llama_tiny(**kw):
    base = dict(vocab_size=512, dim=64, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=128, max_seq_len=128)
    base.update(kw)
    return Llama(LlamaConfig(**base))
