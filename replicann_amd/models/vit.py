"""ViT-B/16 — N20 (absent from the reference).

Patch embedding = 16×16 stride-16 conv, which on NHWC input is a pure
reshape + one MFMA GEMM (``ops.conv2d_nhwc`` takes the non-overlapping
im2col path); a CLS token and learned position embeddings (197 tokens at
224²); 12 pre-LN blocks (non-causal fused attention, GELU MLP); final LN on
the CLS token; linear classifier.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .blocks import LayerNorm, Linear, PreLNBlock


@dataclass(frozen=True)
class ViTConfig:
    image_size: int = 224
    patch: int = 16
    in_chans: int = 3
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    mlp_ratio: int = 4
    num_classes: int = 1000
    dropout: float = 0.0

    @staticmethod
    def base16(**kw):
        return ViTConfig(**kw)

    @staticmethod
    def tiny(**kw):
        d = dict(image_size=32, patch=8, n_layer=2, n_head=4, n_embd=128, num_classes=10)
        d.update(kw)
        return ViTConfig(**d)


class ViT(nn.Module):
    def __init__(self, config: ViTConfig | None = None, **kw):
        super().__init__()
        c = config or ViTConfig(**kw)
        self.config = c
        n_patch = (c.image_size // c.patch) ** 2
        self.patch_weight = nn.Parameter(torch.empty(c.n_embd, c.patch, c.patch, c.in_chans))
        self.patch_bias = nn.Parameter(torch.zeros(c.n_embd))
        nn.init.normal_(self.patch_weight, std=0.02)
        self.cls_token = nn.Parameter(torch.zeros(1, 1, c.n_embd))
        self.pos_embed = nn.Parameter(torch.empty(1, n_patch + 1, c.n_embd))
        nn.init.normal_(self.pos_embed, std=0.02)
        self.blocks = nn.ModuleList(
            PreLNBlock(c.n_embd, c.n_head, causal=False, mlp_ratio=c.mlp_ratio, dropout=c.dropout,
                       n_layer=c.n_layer, eps=1e-6)
            for _ in range(c.n_layer)
        )
        self.norm = LayerNorm(c.n_embd, 1e-6)
        self.head = Linear(c.n_embd, c.num_classes)

    def forward(self, images, targets=None):
        """images (B, H, W, C) NHWC → logits (B, classes) [or mean CE loss]."""
        c = self.config
        B = images.shape[0]
        x = ops.conv2d_nhwc(images, self.patch_weight, self.patch_bias, stride=c.patch)
        x = ops.vit_join(x.reshape(B, -1, c.n_embd), self.cls_token, self.pos_embed)  # [cls; patches] + pos
        prev = None
        for blk in self.blocks:
            x = blk(x, prev)
            prev = blk.out_bias()
        x = self.norm(x[:, 0])
        logits = self.head(x)
        if targets is None:
            return logits
        return ops.cross_entropy(logits, targets)
