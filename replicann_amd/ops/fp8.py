"""FP8 (OCP e4m3fn) linear layers on the CDNA4 block-scaled MFMA (csrc/kernels/fp8.hip) — N3.

``linear_fp8`` runs the FORWARD GEMM in fp8: activations and weights are
quantised per tensor with current scaling (amax → scale = amax/448, computed
on device), multiplied by ``v_mfma_scale_f32_16x16x128_f8f6f4`` at twice the
bf16 MFMA rate, and the two tensor scales are folded into the epilogue alpha
together with bias / GELU / residual.  The backward keeps the bf16 master
weight and bf16 gradients (dgrad/wgrad on the bf16 MFMA GEMM), the recipe
used for "fp8 weights" training in BASELINE.json's GPT-2-medium config.

CPU tensors emulate the numerics (quantise → dequantise → fp32 matmul).
"""

from __future__ import annotations

import torch

from .. import _ext
from .linear import ACT_NONE, _ACTS, _act_ref, bias_act_grad, gemm

E4M3_MAX = 448.0


def quantize_fp8(x):
    """(q uint8 e4m3 storage, state[0] = scale) with x ≈ q·scale."""
    if _ext.use_native(x):
        return _ext.ops().fp8_quantize(x.contiguous())
    amax = x.detach().abs().max().float()
    scale = amax / E4M3_MAX if amax > 0 else torch.tensor(1.0)
    q = (x.float() / scale).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), torch.stack([scale, amax, scale * 0, scale * 0]).float()


def dequantize_fp8(q, state):
    if _ext.use_native(q):
        return _ext.ops().fp8_dequantize(q, state)
    return (q.view(torch.float8_e4m3fn).float() * state[0]).to(torch.bfloat16)


class _LinearFp8Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act, residual):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        res2 = residual.reshape(-1, weight.shape[0]).contiguous() if residual is not None else None
        xq, xs = quantize_fp8(x2)
        wq, ws = quantize_fp8(weight)
        preact = None
        if act != ACT_NONE:
            preact = torch.empty(x2.shape[0], weight.shape[0], device=x.device, dtype=x.dtype)
        if _ext.use_native(x2):
            y = _ext.ops().gemm_fp8(xq, wq, xs, ws, bias, res2, act, preact)
        else:
            h = dequantize_fp8(xq, xs).float() @ dequantize_fp8(wq, ws).float().t()
            if bias is not None:
                h = h + bias.float()
            if preact is not None:
                preact.copy_(h)
            y = _act_ref(h, act)
            if res2 is not None:
                y = y + res2.float()
            y = y.to(x.dtype)
        ctx.save_for_backward(x2, weight, preact)
        ctx.act, ctx.has_bias, ctx.has_res, ctx.shp = act, bias is not None, residual is not None, shp
        ctx.bias_ref = bias
        return y.reshape(*shp[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, weight, preact = ctx.saved_tensors
        gy2 = gy.reshape(-1, weight.shape[0]).contiguous()
        want_b = ctx.has_bias
        if want_b and getattr(ctx.bias_ref, "_rn_bias_done", False):  # see ops.norm._LayerNormFn
            ctx.bias_ref._rn_bias_done = False
            want_b = False
        dh, db = bias_act_grad(gy2, preact, ctx.act, want_b)
        gx = gemm(dh, weight, out_dtype=x2.dtype).reshape(ctx.shp) if ctx.needs_input_grad[0] else None
        gw = gemm(dh, x2, ta=True, split_k=-1, out_dtype=weight.dtype) if ctx.needs_input_grad[1] else None
        gb = db.to(weight.dtype) if (db is not None and ctx.needs_input_grad[2]) else None
        return gx, gw, gb, None, (gy if ctx.has_res else None)


def linear_fp8(x, weight, bias=None, act=None, residual=None):
    """Linear with an fp8 e4m3 forward GEMM (per-tensor current scaling)."""
    a = _ACTS[act] if not isinstance(act, int) else act
    return _LinearFp8Fn.apply(x, weight, bias, a, residual)
