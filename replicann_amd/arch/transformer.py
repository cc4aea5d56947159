"""Transformer blocks (after https://arxiv.org/abs/1706.03762) — source-compatible
with the reference ``src/replicann/arch/transformer.py`` (R8–R12).

Same classes, signatures, properties, submodule registration order (hence the
same ``state_dict`` keys/order) and post-LN forward semantics.  Execution:
  * attention through the fused QKV + fused-attention path of
    ``replicann_amd.nn.attention``;
  * FFN up-projection with ReLU fused into the GEMM epilogue (reference
    ``:29-31``);
  * every ``LN(x + sublayer(x))`` is one fused residual-add + LayerNorm kernel
    (reference ``:111-112,149-150,198-200``).

Decoder mask: the reference registers ``tril(ones(ctx, ctx))`` as an fp32
buffer and ADDS it to the scores (``:142-145,149`` with ``nn/attention.py:41-42``),
i.e. +1 on/below the diagonal, which is NOT causal (Q2).  That behaviour is
reproduced exactly (reference checkpoints give identical outputs); the
buffer is kept persistent and first in the ``state_dict`` like the
reference.  Models that need true causality (GPT-2) use ``causal=True``
kernels instead (``replicann_amd.models.gpt2``).
"""

from __future__ import annotations

import torch
import torch.nn as nn
from torch import Tensor

from .. import ops
from ..nn.attention import MultiheadCrossAttention, MultiheadSelfAttention


class _TransformerFFN(nn.Module):
    """Position-wise FFN: Dropout(down(ReLU(up(x)))) (reference ``:13-41``)."""

    def __init__(self, embedding_size: int, *, bias: bool = True, hidden_size: int | None = None,
                 p_dropout: float = 0.1) -> None:
        super().__init__()
        hidden_size = hidden_size or 4 * embedding_size
        self._upscale = nn.Linear(embedding_size, hidden_size, bias=bias)
        self._downscale = nn.Linear(hidden_size, embedding_size, bias=bias)
        self._dropout = nn.Dropout(p_dropout)

    def forward(self, x: Tensor, /) -> Tensor:
        h = ops.linear(x, self._upscale.weight, self._upscale.bias, act="relu")
        y = ops.linear(h, self._downscale.weight, self._downscale.bias)
        return ops.dropout(y, self._dropout.p, self.training)

    @property
    def embedding_size(self) -> int:
        return self._upscale.in_features

    @property
    def hidden_size(self) -> int:
        return self._upscale.out_features


def _add_ln(ln: nn.LayerNorm, x: Tensor, sub: Tensor) -> Tensor:
    """LN(x + sub) as one fused kernel."""
    return ops.layer_norm(sub, ln.weight, ln.bias, ln.eps, residual=x)


class _TransformerBlock(nn.Module):
    """Base block (reference ``:44-84``); registration order = state_dict order."""

    def __init__(self, n_heads: int, embedding_size: int, *, ffn_bias: bool = True,
                 ffn_hidden_size: int | None = None, head_bias: bool = False, proj_bias: bool = True,
                 p_dropout: float = 0.1) -> None:
        super().__init__()
        self._attn = MultiheadSelfAttention(
            n_heads, embedding_size // n_heads, embedding_size,
            head_bias=head_bias, proj_bias=proj_bias, p_dropout=p_dropout,
        )
        self._attn_ln = nn.LayerNorm(embedding_size)
        self._ffn = _TransformerFFN(embedding_size, bias=ffn_bias, hidden_size=ffn_hidden_size,
                                    p_dropout=p_dropout)
        self._ffn_ln = nn.LayerNorm(embedding_size)

    @property
    def embedding_size(self) -> int:
        return self._attn.embedding_size

    @property
    def head_size(self) -> int:
        return self._attn.head_size

    @property
    def n_heads(self) -> int:
        return self._attn.n_heads


class TransformerEncoder(_TransformerBlock):
    """Post-LN encoder block, no mask (reference ``:87-117``)."""

    def __init__(self, n_heads: int, embedding_size: int, *, ffn_bias: bool = True,
                 ffn_hidden_size: int | None = None, head_bias: bool = False, proj_bias: bool = True,
                 p_dropout: float = 0.1) -> None:
        super().__init__(n_heads=n_heads, embedding_size=embedding_size, ffn_bias=ffn_bias,
                         ffn_hidden_size=ffn_hidden_size, head_bias=head_bias, proj_bias=proj_bias,
                         p_dropout=p_dropout)

    def forward(self, x: Tensor, *, return_kv: bool = False):
        if not return_kv:
            x = _add_ln(self._attn_ln, x, self._attn(x))
            return _add_ln(self._ffn_ln, x, self._ffn(x))
        # reference :114-117 — residual uses the unprojected z (Q5)
        z, k, v = self._attn(x, return_kv=True)
        x = _add_ln(self._attn_ln, x, z)
        x = _add_ln(self._ffn_ln, x, self._ffn(x))
        return x, k, v


class TransformerDecoder(_TransformerBlock):
    """Post-LN decoder block with the reference's additive tril mask (``:120-151``)."""

    def __init__(self, n_heads: int, embedding_size: int, *, context_size: int, ffn_bias: bool = True,
                 ffn_hidden_size: int | None = None, head_bias: bool = False, proj_bias: bool = True,
                 p_dropout: float = 0.1) -> None:
        super().__init__(n_heads=n_heads, embedding_size=embedding_size, ffn_bias=ffn_bias,
                         ffn_hidden_size=ffn_hidden_size, head_bias=head_bias, proj_bias=proj_bias,
                         p_dropout=p_dropout)
        self.register_buffer("_attn_mask", torch.tril(torch.ones(context_size, context_size)))

    def forward(self, x: Tensor) -> Tensor:
        n_tokens = x.shape[1]
        mask = self._attn_mask[:n_tokens, :n_tokens]
        x = _add_ln(self._attn_ln, x, self._attn(x, mask=mask))
        return _add_ln(self._ffn_ln, x, self._ffn(x))


class TransformerCrossDecoder(_TransformerBlock):
    """Decoder with cross attention over encoder k/v (reference ``:154-201``)."""

    def __init__(self, n_heads: int, embedding_size: int, *, context_size: int, ffn_bias: bool = True,
                 ffn_hidden_size: int | None = None, head_bias: bool = False, proj_bias: bool = True,
                 p_dropout: float = 0.1) -> None:
        super().__init__(n_heads=n_heads, embedding_size=embedding_size, ffn_bias=ffn_bias,
                         ffn_hidden_size=ffn_hidden_size, head_bias=head_bias, proj_bias=proj_bias,
                         p_dropout=p_dropout)
        self.register_buffer("_attn_mask", torch.tril(torch.ones(context_size, context_size)))
        self._cross_attn = MultiheadCrossAttention(
            n_heads, embedding_size // n_heads, embedding_size,
            head_bias=head_bias, proj_bias=proj_bias, p_dropout=p_dropout,
        )
        self._cross_attn_ln = nn.LayerNorm(embedding_size)

    def forward(self, x: Tensor, /, encoder_k: Tensor, encoder_v: Tensor) -> Tensor:
        n_tokens = x.shape[1]
        mask = self._attn_mask[:n_tokens, :n_tokens]
        x = _add_ln(self._attn_ln, x, self._attn(x, mask=mask))
        x = _add_ln(self._cross_attn_ln, x, self._cross_attn(x, encoder_k, encoder_v))
        return _add_ln(self._ffn_ln, x, self._ffn(x))
