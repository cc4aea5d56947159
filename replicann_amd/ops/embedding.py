"""Token + position embedding gather / scatter-add (csrc/kernels/embedding.hip) — N14.

Forward fuses ``wte[ids] + wpe[pos]`` into one row-gather kernel (16-B
vectors, one row per wave).  Backward scatter-adds the token gradient with
fp32 ``global_atomic_add_f32`` shaped as whole 256-B wave-instructions (the
MI355X guide's atomic-rate recipe) into an fp32 scratch, then rounds to the
parameter dtype once; the position gradient is a column-sum over the batch.
With flat-buffer parameters the scratch is persistent and kept zero, and only
the touched rows are folded into the bf16 gradient (no full-table memset or
conversion pass; tied LM-head + embedding contributions meet in place).
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext


class _EmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, wte, wpe):
        x = _ext.ops().embedding_fwd(ids, wte, wpe)
        ctx.save_for_backward(ids)
        ctx.wte_ref, ctx.wpe_ref = wte, wpe
        ctx.V, ctx.has_pos = wte.shape[0], wpe is not None
        ctx.dt = wte.dtype
        ctx.Tp = wpe.shape[0] if wpe is not None else 0
        return x

    @staticmethod
    def backward(ctx, gx):
        from .linear import _direct_grad, _notify
        (ids,) = ctx.saved_tensors
        wte, wpe = ctx.wte_ref, ctx.wpe_ref
        gw = _direct_grad(wte)
        gp = _direct_grad(wpe) if wpe is not None else None
        if gw is not None and (wpe is None or gp is not None):
            # accumulate straight into the flat gradient views (touched rows only)
            _ext.ops().embedding_bwd_acc(gx.contiguous(), ids, gw, gp)
            _notify(wte)
            if wpe is not None:
                _notify(wpe)
            return None, None, None
        dwte, dwpe = _ext.ops().embedding_bwd(gx.contiguous(), ids, ctx.V, ctx.Tp)
        return None, dwte.to(ctx.dt), (dwpe.to(ctx.dt) if ctx.has_pos else None)


def embedding(ids, wte, wpe=None):
    """ids (B, T) int → (B, T, E) = wte[ids] (+ wpe[:T])."""
    if _ext.use_native(wte):
        return _EmbFn.apply(ids.to(torch.int64).contiguous(), wte, wpe)
    x = F.embedding(ids, wte)
    if wpe is not None:
        x = x + wpe[: ids.shape[-1]]
    return x


class _VitJoinFn(torch.autograd.Function):
    """x = concat(cls, patches) + pos in one kernel; the backward returns the patch gradient and
    accumulates the cls / pos gradients straight into their flat-buffer views (or fresh zeros)."""

    @staticmethod
    def forward(ctx, patches, cls, pos):
        ctx.cls_ref, ctx.pos_ref = cls, pos
        return _ext.ops().vit_join_fwd(patches.contiguous(), cls, pos)

    @staticmethod
    def backward(ctx, gx):
        from .linear import _direct_grad, _notify
        cls, pos = ctx.cls_ref, ctx.pos_ref
        gc, gp = _direct_grad(cls), _direct_grad(pos)
        direct = gc is not None and gp is not None
        if not direct:
            gc, gp = torch.zeros_like(cls), torch.zeros_like(pos)
        dpatch = _ext.ops().vit_join_bwd(gx.contiguous(), gc, gp)
        if direct:
            _notify(cls)
            _notify(pos)
            return dpatch, None, None
        return dpatch, gc, gp


def vit_join(patches, cls, pos):
    """ViT token sequence: (B, P, E) patch embeddings → (B, 1 + P, E) = [cls; patches] + pos, with
    ``cls`` (1, 1, E) and ``pos`` (1, 1 + P, E) parameters.  GPU: one fused kernel each way."""
    if _ext.use_native(patches) and patches.dtype == torch.bfloat16 and cls.dtype == torch.bfloat16:
        return _VitJoinFn.apply(patches, cls, pos)
    B = patches.shape[0]
    return torch.cat([cls.expand(B, -1, -1).to(patches.dtype), patches], dim=1) + pos.to(patches.dtype)
