"""A token model built from the reference's own block API (``arch.transformer.TransformerDecoder``).

The reference ships blocks only (``/root/reference/src/replicann/arch/transformer.py:120-151``), no
model and no training loop.  This wraps a stack of those blocks — unchanged reference
semantics: post-LN, head dropout ``p_dropout`` (0.1 by default, Q4) in train mode, and the
reference's tril mask ADDED to the scores (Q2: +1 on visible positions, +0 elsewhere, so the block is
not causal) — between a learned token + position embedding and an untied LM head with fused
cross-entropy, so the reference blocks can be trained end to end by ``Trainer`` (model name
``refblock-lm``), data-parallel and graph-captured with their dropout active.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

from .. import ops
from ..arch.transformer import TransformerDecoder


@dataclass(frozen=True)
class RefBlockLMConfig:
    n_layer: int = 4
    n_head: int = 8
    n_embd: int = 256
    block_size: int = 256
    vocab_size: int = 1000
    vocab_pad: int = 1024
    p_dropout: float = 0.1


class RefBlockLM(nn.Module):
    def __init__(self, config: RefBlockLMConfig | None = None, **kw):
        super().__init__()
        cfg = config or RefBlockLMConfig(**kw)
        self.config = cfg
        self.wte = nn.Parameter(torch.empty(cfg.vocab_pad, cfg.n_embd))
        self.wpe = nn.Parameter(torch.empty(cfg.block_size, cfg.n_embd))
        self.head = nn.Parameter(torch.empty(cfg.vocab_pad, cfg.n_embd))
        nn.init.normal_(self.wte, std=0.02)
        nn.init.normal_(self.wpe, std=0.01)
        nn.init.normal_(self.head, std=0.02)
        with torch.no_grad():
            self.head[cfg.vocab_size:].zero_()
        self.blocks = nn.ModuleList(
            TransformerDecoder(cfg.n_head, cfg.n_embd, context_size=cfg.block_size, p_dropout=cfg.p_dropout)
            for _ in range(cfg.n_layer))

    def hidden(self, idx):
        x = ops.embedding(idx, self.wte, self.wpe)
        for blk in self.blocks:
            x = blk(x)
        return x

    def forward(self, idx, targets=None):
        """idx (B, T) → logits (B, T, vocab_size), or the mean CE loss when targets are given."""
        h = self.hidden(idx)
        if targets is None:
            return ops.linear(h, self.head)[..., : self.config.vocab_size]
        return ops.linear_cross_entropy(h, self.head, targets, n_valid_cols=self.config.vocab_size)

    def flops_per_token(self, T=None):
        c = self.config
        T = T or c.block_size
        n_mm = c.n_layer * 12 * c.n_embd**2 + c.vocab_size * c.n_embd
        return 6 * n_mm + 3 * c.n_layer * 4 * T * c.n_embd  # attention is not causal here (Q2)
