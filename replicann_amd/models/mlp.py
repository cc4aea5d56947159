"""2-layer MLP on MNIST-shaped input — N17 (BASELINE config 1, CPU plumbing)."""

from __future__ import annotations

import torch.nn as nn

from .. import ops
from .blocks import Linear


class MLP(nn.Module):
    def __init__(self, in_features=784, hidden=256, num_classes=10):
        super().__init__()
        self.fc1 = Linear(in_features, hidden, std=(2.0 / in_features) ** 0.5)
        self.fc2 = Linear(hidden, num_classes, std=(1.0 / hidden) ** 0.5)

    def forward(self, x, targets=None):
        x = x.reshape(x.shape[0], -1)
        logits = self.fc2(self.fc1(x, act="relu"))
        if targets is None:
            return logits
        return ops.cross_entropy(logits, targets)
