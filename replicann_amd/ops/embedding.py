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
