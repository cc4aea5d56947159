"""NHWC pooling for ResNet-18 (csrc/kernels/conv.hip): 3×3/2 max-pool and global
average pool.  The max-pool forward stores the window position of each maximum (one byte
per output element); the backward gathers the gradient through it."""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = _ext.ops().maxpool_fwd(x.contiguous(), k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg = (k, s, p, x.shape[1], x.shape[2])
        return y

    @staticmethod
    def backward(ctx, gy):
        (idx,) = ctx.saved_tensors
        k, s, p, H, W = ctx.cfg
        return _ext.ops().maxpool_bwd(gy.contiguous(), idx, H, W, k, s, p), None, None, None


def maxpool_nhwc(x, kernel=3, stride=2, padding=1):
    if _ext.use_native(x):
        return _MaxPoolFn.apply(x, kernel, stride, padding)
    y = F.max_pool2d(x.permute(0, 3, 1, 2), kernel, stride, padding)
    return y.permute(0, 2, 3, 1)


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.shp = x.shape
        return _ext.ops().avgpool_fwd(x.contiguous())

    @staticmethod
    def backward(ctx, gy):
        return _ext.ops().avgpool_bwd(gy.contiguous(), ctx.shp[1], ctx.shp[2])


def avgpool_nhwc(x):
    """(N, H, W, C) → (N, C) mean over H, W."""
    if _ext.use_native(x):
        return _AvgPoolFn.apply(x)
    return x.float().mean(dim=(1, 2)).to(x.dtype)
