"""Vision Transformer (ViT-B/16, ViT-L/16, ...) — BASELINE.json config 4 (ViT-L/16 bf16 DDP).

Pre-norm encoder blocks with xddp's fused LayerNorm kernel, attention on xddp's gfx950 flash
attention kernels (``ops/attention.py``; SDPA fallback), GELU MLP, patch embedding as one GEMM.
On bf16 GPU tensors each block runs as one fused autograd node (``ops/encoder_block.py``). Random init; the
structure/parameter count matches torchvision's ``vit_l_16`` (304,326,632 params at 1000
classes).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops.attention import flash_attention
from ..ops.encoder_block import encoder_block, encoder_block_supported
from ..ops.layer_norm import FusedLayerNorm

__all__ = ["VisionTransformer", "vit_b_16", "vit_l_16", "vit_tiny"]


class _Attention(nn.Module):
    def __init__(self, dim, heads):
        super().__init__()
        self.heads = heads
        self.in_proj = nn.Linear(dim, 3 * dim)
        self.out_proj = nn.Linear(dim, dim)

    def forward(self, x):
        B, N, D = x.shape
        # q/k/v are strided [B, N, H, Dh] views of the fused projection; the flash kernel reads them
        # in place and writes [B, N, H, Dh], which is already the out-projection's input layout
        qkv = self.in_proj(x).view(B, N, 3, self.heads, D // self.heads)
        o = flash_attention(qkv[:, :, 0], qkv[:, :, 1], qkv[:, :, 2])
        return self.out_proj(o.reshape(B, N, D))


class EncoderBlock(nn.Module):
    def __init__(self, dim, heads, mlp_dim, norm_layer):
        super().__init__()
        self.ln_1 = norm_layer(dim, eps=1e-6)
        self.self_attention = _Attention(dim, heads)
        self.ln_2 = norm_layer(dim, eps=1e-6)
        self.mlp = nn.Sequential(nn.Linear(dim, mlp_dim), nn.GELU(), nn.Linear(mlp_dim, dim))

    def forward(self, x):
        # bf16 on the GPU: the whole block is one fused autograd node (ops/encoder_block.py)
        if isinstance(self.mlp[1], nn.GELU) and self.mlp[1].approximate == "none" and encoder_block_supported(x, self):
            return encoder_block(x, self)
        x = x + self.self_attention(self.ln_1(x))
        return x + self.mlp(self.ln_2(x))


class VisionTransformer(nn.Module):
    def __init__(self, image_size=224, patch_size=16, num_layers=24, num_heads=16, hidden_dim=1024, mlp_dim=4096,
                 num_classes=1000, norm_layer=FusedLayerNorm, checkpoint_activations: bool = False):
        super().__init__()
        self.patch_size = patch_size
        self.hidden_dim = hidden_dim
        self.checkpoint_activations = checkpoint_activations
        self.conv_proj = nn.Conv2d(3, hidden_dim, kernel_size=patch_size, stride=patch_size)
        n = (image_size // patch_size) ** 2 + 1
        self.class_token = nn.Parameter(torch.zeros(1, 1, hidden_dim))
        self.pos_embedding = nn.Parameter(torch.empty(1, n, hidden_dim).normal_(std=0.02))
        self.layers = nn.ModuleList([EncoderBlock(hidden_dim, num_heads, mlp_dim, norm_layer)
                                     for _ in range(num_layers)])
        self.ln = norm_layer(hidden_dim, eps=1e-6)
        self.head = nn.Linear(hidden_dim, num_classes)
        nn.init.trunc_normal_(self.conv_proj.weight, std=(1.0 / (3 * patch_size * patch_size)) ** 0.5)
        nn.init.zeros_(self.conv_proj.bias)
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.xavier_uniform_(m.weight)
                nn.init.normal_(m.bias, std=1e-6)
        nn.init.zeros_(self.head.weight)
        nn.init.zeros_(self.head.bias)

    def _patch_embed(self, x):
        """The stride-16 16x16 patch convolution as one GEMM: patches [B*P, 3*16*16] x W^T.

        Same parameters (``conv_proj``, state_dict-compatible with torchvision), but MIOpen has
        no tuned NHWC/NCHW bf16 solver for this shape and falls back to its naive direct-conv
        kernels (~13 ms forward + ~8.5 ms weight gradient per ViT-L bs64 step on MI355X, a third
        of the step); the patchify reshape + hipBLASLt GEMM take ~0.3 ms."""
        B, C, H, W = x.shape
        p = self.patch_size
        gh, gw = H // p, W // p
        patches = x.reshape(B, C, gh, p, gw, p).permute(0, 2, 4, 1, 3, 5).reshape(B, gh * gw, C * p * p)
        w = self.conv_proj.weight.reshape(self.hidden_dim, C * p * p)
        return F.linear(patches, w, self.conv_proj.bias)

    def forward(self, x):
        x = self._patch_embed(x)
        x = torch.cat([self.class_token.expand(x.shape[0], -1, -1), x], dim=1) + self.pos_embedding
        for blk in self.layers:
            if self.checkpoint_activations and self.training:
                x = torch.utils.checkpoint.checkpoint(blk, x, use_reentrant=False)
            else:
                x = blk(x)
        return self.head(self.ln(x)[:, 0])


def vit_b_16(**kw):
    return VisionTransformer(num_layers=12, num_heads=12, hidden_dim=768, mlp_dim=3072, **kw)


def vit_l_16(**kw):
    return VisionTransformer(num_layers=24, num_heads=16, hidden_dim=1024, mlp_dim=4096, **kw)


def vit_tiny(**kw):
    return VisionTransformer(image_size=32, patch_size=8, num_layers=2, num_heads=2, hidden_dim=64, mlp_dim=128, **kw)
