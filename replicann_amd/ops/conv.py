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

Convolutions whose input and output channels are multiples of 64 (all of
ResNet-18 after the 7×7 stem) take the implicit-GEMM path instead
(``_ConvImplicitFn``, csrc/kernels/gemm_conv.hip): the GEMM's LDS-DMA loaders
gather each K-tile (one filter tap × 64 channels) straight from the NHWC
tensor, so the 9×-sized im2col matrix is never written, read or saved.
"""

from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .. import _ext
from .linear import _direct_grad, _notify, gemm


# BatchNorm statistics reduced by the producing conv's epilogue (a test hook, not an env knob:
# tests/test_ops_gpu.py compares it with the BN's own statistics pass)
BN_FUSED_STATS = True


def _fused_bn_stats():
    return BN_FUSED_STATS


class GradJoin:
    """Meeting point of two gradients of one tensor (ResNet: a block input x feeds conv1 and the
    shortcut).  Autograd would run both producing nodes and then a separate add kernel; with a join
    the FIRST of the two nodes to run parks its gradient here and returns None for that input, and
    the SECOND adds its own into it inside its producing kernel (the dgrad GEMM epilogue's
    accumulate, or the col2im gather) and returns the sum — whatever order the engine picks.

    Both nodes run in any backward that needs x's gradient (each lies on a path from the loss to x).
    One join per forward call, so gradient accumulation over micro-batches and captured step graphs
    are unaffected."""

    __slots__ = ("g",)

    def __init__(self):
        self.g = None

    def take(self):
        g, self.g = self.g, None
        return g

    def settle(self, g):
        """Result of a node that did NOT fuse the add: park it (first) or add it (second)."""
        if g is None:
            return None
        other = self.take()
        if other is None:
            self.g = g
            return None
        return other.add_(g)


def weight_param(ctx):
    w = ctx.weight
    return w if isinstance(w, torch.nn.Parameter) and w.is_contiguous() else None


def _out_hw(H, W, kh, kw, stride, pad):
    return (H + 2 * pad - kh) // stride + 1, (W + 2 * pad - kw) // stride + 1


def implicit_ok(C, OC, KH, KW, stride, pad):
    """Implicit-GEMM path (no im2col matrix): channels in multiples of 64 (ResNet-18 past the stem)."""
    return C % 64 == 0 and OC % 64 == 0 and not (KH == 1 and KW == 1 and stride == 1 and pad == 0)


def conv_implicit_ok(conv):
    """Whether a Conv2d module (weight (OC, KH, KW, C), ``stride``, ``padding``) runs on the
    implicit-GEMM path."""
    OC, KH, KW, C = conv.weight.shape
    return implicit_ok(C, OC, KH, KW, int(conv.stride), int(conv.padding))


class _ConvImplicitFn(torch.autograd.Function):
    """conv2d whose GEMM loaders gather the filter taps straight from the NHWC activation:
    fwd (A gathered), wgrad (B gathered, split-K over pixels), dgrad (stride 1: the
    transposed conv, A = dY gathered; stride 2: dcols GEMM + col2im gather)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, join=None):
        ops = _ext.ops()
        ctx.join = join
        x = x.contiguous()
        w = weight.contiguous()
        if _fused_bn_stats() and any(ctx.needs_input_grad[:2]):
            # training: the GEMM epilogue also emits per-256-row Σ | Σ² of y, which the BatchNorm
            # that follows every ResNet conv reduces instead of re-reading y for its statistics
            y, part = ops.conv_fwd_implicit_stats(x, w, bias, stride, pad)
            y._rn_bn_partials = part
            y._rn_bn_version = y._version  # partials describe THIS version of y (see norm.py)
        else:
            y = ops.conv_fwd_implicit(x, w, bias, stride, pad)
        ctx.save_for_backward(x, w)
        ctx.weight = weight  # the Parameter itself (direct gradient accumulation), not saved data
        ctx.stride, ctx.pad, ctx.has_bias = stride, pad, bias is not None
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        ops = _ext.ops()
        N, H, W, C = x.shape
        OC, KH, KW, _ = w.shape
        gy = gy.contiguous()
        gy2 = gy.reshape(-1, OC)
        gx = gw = gb = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            _, gb = ops.bias_act_grad(gy2, None, 0, True)
        if ctx.needs_input_grad[1]:
            w_acc = _direct_grad(weight_param(ctx))
            if w_acc is not None and w_acc.dtype == torch.bfloat16:  # straight into the flat gradient buffer
                ops.conv_wgrad_implicit(gy2, x, KH, KW, ctx.stride, ctx.pad, w_acc.view(OC, -1), True)
                _notify(ctx.weight)
            else:
                gw = ops.conv_wgrad_implicit(gy2, x, KH, KW, ctx.stride, ctx.pad).reshape(OC, KH, KW, C)
        if ctx.needs_input_grad[0]:
            join, ctx.join = ctx.join, None
            acc = join.take() if join is not None else None  # the other gradient of x, if it came first
            if ctx.stride == 1:
                gx = ops.conv_dgrad_implicit(gy, w, H, W, ctx.pad, acc, acc is not None)
            else:
                K = KH * KW * C
                dcols = gemm(gy2, w.reshape(OC, K), out_dtype=x.dtype)
                gx = ops.col2im(dcols, N, H, W, C, KH, KW, ctx.stride, ctx.pad, K, acc, acc is not None)
            if join is not None and acc is None:  # first of the two: park it for the other node
                join.g, gx = gx, None
        return gx, gw, gb, None, None, None


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


def conv2d_nhwc(x, weight, bias=None, stride=1, padding=0, join=None):
    """x (N,H,W,C), weight (OC,KH,KW,C) → (N,OH,OW,OC).

    ``join``: a :class:`GradJoin` shared with the other consumer of ``x`` whose backward also
    produces x's gradient (implicit-GEMM path; ignored elsewhere)."""
    if _ext.use_native(x):
        OC, KH, KW, C = weight.shape
        if implicit_ok(C, OC, KH, KW, int(stride), int(padding)):
            return _ConvImplicitFn.apply(x, weight, bias, int(stride), int(padding), join)
        assert join is None, "gradient joins need the implicit-GEMM convolution"
        return _ConvFn.apply(x, weight, bias, int(stride), int(padding))
    y = F.conv2d(x.permute(0, 3, 1, 2), weight.permute(0, 3, 1, 2), bias, stride, padding)
    return y.permute(0, 2, 3, 1)
