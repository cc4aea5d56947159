"""LayerNorm and BatchNorm on gfx950 (csrc/kernels/layernorm.hip, batchnorm.hip).

LayerNorm replaces ``nn.LayerNorm`` used at reference
``arch/transformer.py:65,72,188`` (post-LN ``LN(x + sublayer(x))``,
``:111-112,149-150,198-200``).  The kernel handles one row per wave (E ≤ 8192,
bf16 vectorised 16-B loads, fp32 statistics) and optionally fuses the residual
add in forward (h = x + r; y = LN(h), h is returned for the backward) and the
residual-gradient add in backward.

BatchNorm2d (N11; needed by ResNet-18, absent from the reference) works on
NHWC activations with a fused ReLU.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext


# the fp8 linear that produced a LayerNorm's input takes its e5m2 dY from the LayerNorm backward kernel
# (_LayerNormFn, producer_fp8); 0: its own quantisation pass (A/B)
FP8_LN_Q8 = True  # (a test hook, not an env knob: tests/test_fp8_ln_q8_gpu.py compares both paths)


class _LayerNormFn(torch.autograd.Function):
    """y = LN(x [+ residual]).

    Second output (``two_out``): the pre-norm sum h = x + residual, or — with no
    residual — a pass-through alias of x.  Either way the gradient arriving on
    it is added to dx inside the backward kernel (no separate add), which is
    what a pre-LN block needs: x feeds both the LayerNorm and the residual
    branch.

    ``producer_bias``: bias of the linear layer whose output IS x (x = x_prev +
    a·Wᵀ + b).  Its gradient Σ_rows dx is then produced by this backward kernel
    for free and accumulated straight into the flat gradient buffer; the
    linear's backward sees ``_rn_bias_done`` and skips its own bias pass.

    ``producer_fp8``: the :class:`~replicann_amd.ops.fp8.Fp8State` of that linear when it is an fp8 layer whose
    backward takes dY in e5m2 (``bwd_plan``): the backward kernel then also writes dx in e5m2 with that layer's
    delayed gradient scale and offers it (``Fp8State.goffer``), so the linear needs no quantisation pass over
    its dY (``FP8_LN_Q8``).
    """

    @staticmethod
    def forward(ctx, x, weight, bias, eps, residual, two_out, producer_bias, fp8=None, producer_fp8=None):
        shp = x.shape
        E = shp[-1]
        x2 = x.reshape(-1, E).contiguous()
        r2 = residual.reshape(-1, E).contiguous() if residual is not None else None
        if fp8 is not None and fp8.producer_ready(x2.device):
            # the consumer's e4m3 activation comes out of this kernel (delayed scaling)
            slot = fp8.roll_slot(0)  # (inference: a scratch copy — the training slot stays untouched)
            y, h, mean, rstd, q8 = _ext.ops().layernorm_fwd_q8(x2, r2, weight, bias, eps, slot)
            fp8.offer(y, q8, slot)
        else:
            y, h, mean, rstd = _ext.ops().layernorm_fwd(x2, r2, weight, bias, eps)
        ctx.save_for_backward(x2 if residual is None else h, weight, mean, rstd)
        ctx.set_materialize_grads(False)  # an unused second output → gh None → no zero-tensor read
        ctx.bias_ref = bias
        ctx.producer_bias = producer_bias if residual is None else None
        ctx.producer_fp8 = producer_fp8 if residual is None else None
        ctx.has_res = residual is not None
        ctx.has_bias = bias is not None
        ctx.shp = shp
        if residual is not None:
            return y.reshape(shp), h.reshape(shp)
        if two_out:
            return y.reshape(shp), x.view_as(x)
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, gy, gh=None):
        from .linear import _direct_grad, _notify
        h, weight, mean, rstd = ctx.saved_tensors
        bias = ctx.bias_ref
        E = ctx.shp[-1]
        if gy is None:
            gy = torch.zeros(ctx.shp, dtype=h.dtype, device=h.device)
        gy2 = gy.reshape(-1, E).contiguous()
        gh2 = gh.reshape(-1, E).contiguous() if gh is not None else None
        dw_acc = _direct_grad(weight)
        db_acc = _direct_grad(bias) if bias is not None else None
        direct = dw_acc is not None and db_acc is not None
        pb = ctx.producer_bias
        pb_acc = _direct_grad(pb) if (pb is not None and direct) else None
        # the producing fp8 linear's dY in e5m2 from this kernel (its delayed gradient scale seeded, and its
        # backward planned in fp8)
        pf = ctx.producer_fp8
        q8 = slot = None
        if (pf is not None and FP8_LN_Q8 and pf.g_ready and any(pf.bwd_plan) and pf.gt is not None
                and pf.gt.device == gy2.device):
            slot = pf.gslot(gy2.device)
            q8 = torch.empty(gy2.shape, dtype=torch.uint8, device=gy2.device)
        dx, dw, db = _ext.ops().layernorm_bwd(gy2, gh2, h, weight, mean, rstd, dw_acc if direct else None,
                                              db_acc if direct else None, pb_acc, q8, slot)
        if q8 is not None:
            pf.goffer(dx, q8)
        dx = dx.reshape(ctx.shp)
        if pb_acc is not None:
            pb._rn_bias_done = True  # consumed (and reset) by the producer linear's backward
            _notify(pb)
        g_res = dx if ctx.has_res else None
        if direct:  # gradients already accumulated in the flat buffer
            _notify(weight)
            _notify(bias)
            return dx, None, None, None, g_res, None, None, None, None
        return (dx, dw.to(weight.dtype), db.to(weight.dtype) if ctx.has_bias else None, None, g_res, None, None, None,
                None)


def layer_norm(x, weight, bias=None, eps=1e-5, residual=None, return_sum=False, producer_bias=None, fp8=None,
               producer_fp8=None):
    """LayerNorm over the last dim.  With ``residual``: h = x + residual, y = LN(h).

    Returns y, or (y, h) when ``return_sum`` (h = x when there is no residual;
    use that h as the block's residual so both gradients meet in one kernel).
    ``producer_bias``, ``producer_fp8``: see :class:`_LayerNormFn`.
    ``fp8``: the :class:`~replicann_amd.ops.fp8.Fp8State` of the fp8 GEMM that consumes y — the
    kernel then also writes y in e4m3 (delayed scaling) and hands it to that GEMM, which skips its
    own quantisation pass.
    """
    if _ext.use_native(x):
        if fp8 is not None:
            fp8.enter()
        out = _LayerNormFn.apply(x, weight, bias, eps, residual, return_sum, producer_bias, fp8, producer_fp8)
        if residual is None and not return_sum:
            return out
        return out if return_sum else out[0]
    h = x + residual if residual is not None else x
    y = F.layer_norm(h, (h.shape[-1],), weight, bias, eps)
    return (y, h) if return_sum else y


# --------------------------------------------------------------------------
# BatchNorm2d (NHWC, training uses batch statistics, fused ReLU)
# --------------------------------------------------------------------------
class _BatchNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, momentum, eps, relu, residual, join=None):
        # x: (N, H, W, C) contiguous channels-last storage
        ctx.join = join  # GradJoin of the residual's gradient (see ops.conv.GradJoin)
        C = x.shape[-1]
        x2 = x.reshape(-1, C)
        r2 = residual.reshape(-1, C).contiguous() if residual is not None else None
        # Σ | Σ² partials of x from its producer's epilogue (implicit-conv forward), if it left them
        part = getattr(x, "_rn_bn_partials", None)
        if part is not None and (part.dim() != 2 or part.shape[1] != 2 * C):
            part = None
        if part is not None and getattr(x, "_rn_bn_version", -1) != x._version:
            part = None  # x was modified in place after the conv: recompute the statistics
        # mask: relu'(y) as bits (1/16 of y's bytes) — all the backward needs of y
        y, mean, rstd, mask = _ext.ops().batchnorm_fwd(x2, weight, bias, running_mean, running_var,
                                                       momentum, eps, relu, r2, part)
        ctx.save_for_backward(x2, mask, weight, bias, mean, rstd)
        ctx.params = (weight, bias)  # the Parameters themselves (direct gradient accumulation)
        ctx.relu = relu
        ctx.has_res = residual is not None
        ctx.shp = x.shape
        return y.reshape(x.shape)

    @staticmethod
    def backward(ctx, gy):
        from .linear import _direct_grad, _notify
        x2, mask, weight, bias, mean, rstd = ctx.saved_tensors
        C = ctx.shp[-1]
        pw, pb = ctx.params
        dw_acc, db_acc = _direct_grad(pw), _direct_grad(pb)
        direct = (dw_acc is not None and db_acc is not None and dw_acc.dtype == torch.bfloat16
                  and db_acc.dtype == torch.bfloat16)
        dx, dw, db, gres = _ext.ops().batchnorm_bwd(gy.reshape(-1, C).contiguous(), x2, mask, weight, mean,
                                                    rstd, ctx.relu, ctx.has_res,
                                                    dw_acc if direct else None, db_acc if direct else None)
        gr = gres.reshape(ctx.shp) if ctx.has_res else None
        if ctx.join is not None:
            gr = ctx.join.settle(gr)
            ctx.join = None
        if direct:  # the reduction added dw / db into the flat gradient views
            _notify(pw)
            _notify(pb)
            return dx.reshape(ctx.shp), None, None, None, None, None, None, None, gr, None
        return dx.reshape(ctx.shp), dw.to(weight.dtype), db.to(bias.dtype), None, None, None, None, None, gr, None


def batch_norm_nhwc(x, weight, bias, running_mean, running_var, training, momentum=0.1, eps=1e-5,
                    relu=False, residual=None, join=None):
    """BatchNorm over (N,H,W) of an NHWC tensor; optional fused residual add and ReLU:
    y = [relu](BN(x) [+ residual])  (ResNet's block output in one pass).  ``join``: a
    :class:`~replicann_amd.ops.conv.GradJoin` that meets the residual's gradient with the other
    consumer's (training, GPU)."""
    if _ext.use_native(x):
        if training:
            return _BatchNormFn.apply(x, weight, bias, running_mean, running_var, momentum, eps, relu, residual,
                                      join if residual is not None else None)
        C = x.shape[-1]
        r2 = residual.reshape(-1, C).contiguous() if residual is not None else None
        y = _ext.ops().batchnorm_eval(x.reshape(-1, C).contiguous(), weight, bias, running_mean, running_var,
                                      eps, relu, r2)
        return y.reshape(x.shape)
    xc = x.permute(0, 3, 1, 2)
    y = F.batch_norm(xc, running_mean, running_var, weight, bias, training, momentum, eps).permute(0, 2, 3, 1)
    if residual is not None:
        y = y + residual
    if relu:
        y = F.relu(y)
    return y
