"""Synthetic data generators (N22): every BASELINE config uses synthetic data.

Batches are generated once, ON the target device, into a small pool that the
training loop cycles through — no host→device copies inside the timed step.
"""

from __future__ import annotations

import torch


class SyntheticLM:
    """Random token sequences (B, T+1) → (inputs, next-token targets)."""

    def __init__(self, batch, seq_len, vocab, device, pool=4, seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.pool = [torch.randint(0, vocab, (batch, seq_len + 1), generator=g).to(device) for _ in range(pool)]
        self.i = 0

    def __next__(self):
        t = self.pool[self.i % len(self.pool)]
        self.i += 1
        return t[:, :-1], t[:, 1:]

    def __iter__(self):
        return self


class SyntheticImages:
    """Random NHWC images + labels."""

    def __init__(self, batch, size, chans, classes, device, dtype=torch.bfloat16, pool=2, seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.pool = [(torch.randn(batch, size, size, chans, generator=g).to(device=device, dtype=dtype),
                      torch.randint(0, classes, (batch,), generator=g).to(device)) for _ in range(pool)]
        self.i = 0

    def __next__(self):
        b = self.pool[self.i % len(self.pool)]
        self.i += 1
        return b

    def __iter__(self):
        return self


class SyntheticMNIST:
    """MNIST-shaped (B, 784) inputs with a learnable labelling (a fixed random
    linear teacher), so a model trained on it measurably reduces its loss."""

    def __init__(self, batch, device="cpu", seed=0, n=4096):
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.x = torch.rand(n, 784, generator=g)
        teacher = torch.randn(784, 10, generator=g)
        self.y = (self.x @ teacher).argmax(-1)
        self.x, self.y = self.x.to(device), self.y.to(device)
        self.batch, self.i = batch, 0

    def __next__(self):
        n = self.x.shape[0]
        s = (self.i * self.batch) % n
        self.i += 1
        idx = torch.arange(s, s + self.batch) % n
        return self.x[idx], self.y[idx]

    def __iter__(self):
        return self
