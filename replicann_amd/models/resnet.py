"""ResNet-18 — N18 (absent from the reference).

NHWC bf16 throughout: convolutions are im2col + MFMA GEMM
(``ops.conv2d_nhwc``), BatchNorm runs on channels-last rows with a fused ReLU
(``ops.batch_norm_nhwc``), pooling kernels are NHWC.  BasicBlock ×[2,2,2,2],
3×224×224 input, 1000 classes.  Conv weights are stored (OC, KH, KW, C).
"""

from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops
from .blocks import Linear


class Conv2d(nn.Module):
    def __init__(self, cin, cout, k, stride=1, padding=0, bias=False):
        super().__init__()
        self.stride, self.padding = stride, padding
        self.weight = nn.Parameter(torch.empty(cout, k, k, cin))
        nn.init.normal_(self.weight, std=math.sqrt(2.0 / (k * k * cout)))  # kaiming fan_out
        self.bias = nn.Parameter(torch.zeros(cout)) if bias else None

    def forward(self, x, join=None):
        return ops.conv2d_nhwc(x, self.weight, self.bias, self.stride, self.padding, join=join)


class BatchNorm(nn.Module):
    def __init__(self, c, momentum=0.1, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.momentum, self.eps = momentum, eps

    def forward(self, x, relu=False, residual=None, join=None):
        return ops.batch_norm_nhwc(x, self.weight, self.bias, self.running_mean, self.running_var,
                                   self.training, self.momentum, self.eps, relu, residual, join=join)


class BasicBlock(nn.Module):
    def __init__(self, cin, cout, stride):
        super().__init__()
        self.conv1 = Conv2d(cin, cout, 3, stride, 1)
        self.bn1 = BatchNorm(cout)
        self.conv2 = Conv2d(cout, cout, 3, 1, 1)
        self.bn2 = BatchNorm(cout)
        self.has_down = stride != 1 or cin != cout
        if self.has_down:
            self.down_conv = Conv2d(cin, cout, 1, stride, 0)
            self.down_bn = BatchNorm(cout)
        self.join_grads = True  # x's two gradients meet inside a kernel (ops.conv.GradJoin)

    def forward(self, x):
        # x feeds conv1 and the shortcut: its two gradients are summed by the second producing kernel
        # (conv1's dgrad epilogue / col2im, or the shortcut's) instead of an autograd add
        join = (ops.GradJoin() if self.join_grads and self.training and x.is_cuda and x.requires_grad
                and torch.is_grad_enabled() and ops.conv_implicit_ok(self.conv1)
                and (not self.has_down or ops.conv_implicit_ok(self.down_conv)) else None)
        out = self.bn1(self.conv1(x, join=join), relu=True)
        if self.has_down:
            sc = self.down_bn(self.down_conv(x, join=join))
            # relu(bn2(conv2(out)) + sc) in one BatchNorm pass (its backward also returns sc's gradient)
            return self.bn2(self.conv2(out), relu=True, residual=sc)
        return self.bn2(self.conv2(out), relu=True, residual=x, join=join)


class ResNet18(nn.Module):
    def __init__(self, num_classes=1000, in_chans=3, widths=(64, 128, 256, 512)):
        super().__init__()
        self.conv1 = Conv2d(in_chans, widths[0], 7, 2, 3)
        self.bn1 = BatchNorm(widths[0])
        layers = []
        cin = widths[0]
        for i, w in enumerate(widths):
            for j in range(2):
                layers.append(BasicBlock(cin, w, 2 if (j == 0 and i > 0) else 1))
                cin = w
        self.layers = nn.ModuleList(layers)
        self.fc = Linear(cin, num_classes, std=0.01)

    def forward(self, images, targets=None):
        """images (B, H, W, C) NHWC → logits (B, classes) [or mean CE loss]."""
        x = self.bn1(self.conv1(images), relu=True)
        x = ops.maxpool_nhwc(x, 3, 2, 1)
        for blk in self.layers:
            x = blk(x)
        x = ops.avgpool_nhwc(x)
        logits = self.fc(x)
        if targets is None:
            return logits
        return ops.cross_entropy(logits, targets)
