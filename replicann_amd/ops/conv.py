"""conv2d as im2col + MFMA GEMM on NHWC bf16 (csrc/kernels/conv.hip) — N10.

Activations are channels-last (N, H, W, C), so the GEMM output
``[N·OH·OW, OC] = cols[N·OH·OW, K] · Wᵀ[K, OC]`` *is* the NHWC output.
``K = KH·KW·C`` is laid out (kh, kw, c) with c fastest, matching a weight
stored as (OC, KH, KW, C); K is zero-padded to a multiple of 8 so every GEMM
row is 16-B aligned (only the 7×7×3 stem needs it).

Backward: dW = dYᵀ·cols (split-K GEMM over the N·OH·OW rows), dcols = dY·W
(NN GEMM), then col2im as a *gather* (each input pixel sums the ≤KH·KW
columns that read it — deterministic, no atomics).

1×1 stride-1 convolutions skip im2col entirely (cols = x).  The ViT patch
embedding (16×16 stride-16) is the non-overlapping case: im2col is a pure
reshape/permute, done by the same kernel.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext
from .linear import gemm


def _out_hw(H, W, kh, kw, stride, pad):
    return (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad):
        N, H, W, C = x.shape
        OC, KH, KW, _ = weight.shape
        OH, OW = _out_hw(H, W, KH, KW, stride, pad)
        K = KH * KW * C
        Kp = (K + 7) // 8 * 8
        ops = _ext.ops()
        if KH == 1 and KW == 1 and stride == 1 and pad == 0 and Kp == K:
            cols = x.reshape(N * H * W, C)
        else:
            cols = ops.im2col(x.contiguous(), KH, KW, stride, pad, Kp)
        w2 = weight.reshape(OC, K)
        if Kp != K:
            w2 = F.pad(w2, (0, Kp - K))
        y = ops.gemm(cols, w2.contiguous(), False, True, bias, None, 0, None, None, False, 0, False, None, -1)
        ctx.save_for_backward(x, cols, w2)
        ctx.meta = (N, H, W, C, OC, KH, KW, OH, OW, K, Kp, stride, pad, bias is not None)
        return y.reshape(N, OH, OW, OC)

    @staticmethod
    def backward(ctx, gy):
        x, cols, w2 = ctx.saved_tensors
        N, H, W, C, OC, KH, KW, OH, OW, K, Kp, stride, pad, has_bias = ctx.meta
        ops = _ext.ops()
        gy2 = gy.reshape(-1, OC).contiguous()
        gx = gw = gb = None
        if has_bias:
            _, gb = ops.bias_act_grad(gy2, None, 0, True)
            gb = gb.to(w2.dtype)
        if ctx.needs_input_grad[1]:
            gw = gemm(gy2, cols, ta=True, split_k=-1, out_dtype=w2.dtype)[:, :K].reshape(OC, KH, KW, C)
        if ctx.needs_input_grad[0]:
            dcols = gemm(gy2, w2, out_dtype=x.dtype)
            if KH == 1 and KW == 1 and stride == 1 and pad == 0 and Kp == K:
                gx = dcols.reshape(N, H, W, C)
            else:
                gx = ops.col2im(dcols, N, H, W, C, KH, KW, stride, pad, Kp)
        return gx, gw, gb, None, None


def conv2d_nhwc(x, weight, bias=None, stride=1, padding=0):
    """x (N,H,W,C), weight (OC,KH,KW,C) → (N,OH,OW,OC)."""
    if _ext.use_native(x):
        return _ConvFn.apply(x, weight, bias, int(stride), int(padding))
    y = F.conv2d(x.permute(0, 3, 1, 2), weight.permute(0, 3, 1, 2), bias, stride, padding)
    return y.permute(0, 2, 3, 1)
