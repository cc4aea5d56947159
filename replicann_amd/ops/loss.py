"""Fused softmax cross-entropy (csrc/kernels/xent.hip) — N9.

Forward: one pass over each logits row (vocab 50257 for GPT-2, padded
storage allowed) computing the row log-sum-exp and the NLL; nothing but the
per-row lse is saved.  Backward: one pass that writes
``(softmax - onehot) · g / n_valid`` **in place over the logits storage**
(the logits are dead after the loss), so the 1.6 GB logits tensor of a
GPT-2 step is read twice and written once in total.

``n_valid_cols`` lets the logits be stored padded (e.g. 50304 = 393·128
columns for GEMM tiling) while the loss only sees the first 50257 columns.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, n_valid_cols, ignore_index, inplace_grad):
        loss_rows, lse = _ext.ops().xent_fwd(logits, target, n_valid_cols, ignore_index)
        n = (target != ignore_index).sum().clamp_min(1).float()
        ctx.save_for_backward(logits, target, lse, n)
        ctx.n_valid_cols, ctx.ignore_index, ctx.inplace = n_valid_cols, ignore_index, inplace_grad
        return loss_rows.sum() / n

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, n = ctx.saved_tensors
        scale = (g.float() / n).reshape(1)
        grad = logits if ctx.inplace else torch.empty_like(logits)
        _ext.ops().xent_bwd(logits, target, lse, scale, grad, ctx.n_valid_cols, ctx.ignore_index)
        return grad, None, None, None, None


def cross_entropy(logits, target, *, n_valid_cols=None, ignore_index=-100, inplace_grad=False):
    """Mean token cross-entropy of (N, V) logits against (N,) int targets."""
    V = logits.shape[-1]
    nv = V if n_valid_cols is None else n_valid_cols
    lg = logits.reshape(-1, V)
    tg = target.reshape(-1)
    if _ext.use_native(lg):
        if not lg.is_contiguous():
            lg = lg.contiguous()
        return _XentFn.apply(lg, tg.long().contiguous(), nv, ignore_index, inplace_grad)
    return F.cross_entropy(lg[:, :nv].float(), tg.long(), ignore_index=ignore_index)
