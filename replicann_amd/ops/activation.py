"""Elementwise activations, row softmax and dropout (csrc/kernels/elementwise.hip, softmax.hip).

* GELU / ReLU standalone fwd+bwd (N7).  Inside Linear layers the activation is
  fused into the GEMM epilogue instead (ops/linear.py); these standalone
  kernels serve the remaining call sites (e.g. ResNet's ReLU after a residual).
* Row softmax fwd/bwd (N8), with an optional scale, used by classifier heads
  and by the reference-parity attention path.
* Dropout with a counter-based RNG (hash of seed and element index), so the
  backward regenerates the mask instead of storing it.

All kernels move bf16 as 16-byte vectors and compute in fp32.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext

_GELU, _RELU = 2, 1


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kind):
        y = _ext.ops().act_fwd(x.contiguous(), kind)
        ctx.save_for_backward(x)
        ctx.kind = kind
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        return _ext.ops().act_bwd(gy.contiguous(), x.contiguous(), ctx.kind), None


def gelu(x):
    """tanh-approximate GELU (GPT-2 / ViT)."""
    if _ext.use_native(x):
        return _ActFn.apply(x, _GELU)
    return F.gelu(x, approximate="tanh")


def relu(x):
    if _ext.use_native(x):
        return _ActFn.apply(x, _RELU)
    return F.relu(x)


class _SoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, scale):
        shp = x.shape
        y = _ext.ops().softmax_fwd(x.reshape(-1, shp[-1]).contiguous(), scale)
        ctx.save_for_backward(y)
        ctx.scale = scale
        ctx.shp = shp
        return y.reshape(shp)

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        dx = _ext.ops().softmax_bwd(gy.reshape(y.shape).contiguous(), y, ctx.scale)
        return dx.reshape(ctx.shp), None


def softmax(x, dim=-1, scale=1.0):
    """softmax(scale·x) over the last dim."""
    assert dim in (-1, x.dim() - 1), "row softmax only"
    if _ext.use_native(x):
        return _SoftmaxFn.apply(x, float(scale))
    return torch.softmax(x.float() * scale, dim=-1).to(x.dtype)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed_buf):
        y = _ext.ops().dropout_fwd(x.contiguous(), p, 0, seed_buf)
        ctx.p, ctx.seed_buf = p, seed_buf
        return y

    @staticmethod
    def backward(ctx, gy):
        return _ext.ops().dropout_fwd(gy.contiguous(), ctx.p, 0, ctx.seed_buf), None, None


def dropout(x, p, training=True):
    if not training or p == 0.0:
        return x
    if _ext.use_native(x):
        from .rng import next_seed
        return _DropoutFn.apply(x, float(p), next_seed(x.device))  # seed drawn on the device
    return F.dropout(x, p, True)
