"""Synthetic data generators (N22): every BASELINE config uses synthetic data.

Batches are generated once, ON the target device, into a small pool that the
training loop cycles through — no host→device copies inside the timed step.
"""

from __future__ import annotations

import torch


class SyntheticLM:
    """Synthetic token sequences (B, T+1) → (inputs, next-token targets).

    ``structured=True`` (default): a learnable source — tokens from a random
    ``active``-id subset of the vocabulary, each followed by a fixed random
    successor with probability ``p_follow`` (else a uniform active id), so a
    model that trains correctly shows a falling loss within a few steps.  The
    shapes, and therefore every kernel and its cost, are those of uniform
    random tokens over the full vocabulary (``structured=False``); the logits
    still span all ``vocab`` ids.  The source (id subset, successor table) is
    shared by all data-parallel ranks; ``seed`` only draws the sequences."""

    def __init__(self, batch, seq_len, vocab, device, pool=4, seed=0, structured=True, active=1024,
                 p_follow=0.75):
        g = torch.Generator(device="cpu").manual_seed(seed)
        if not structured:
            self.pool = [torch.randint(0, vocab, (batch, seq_len + 1), generator=g).to(device) for _ in range(pool)]
        else:
            active = min(active, vocab)
            gs = torch.Generator(device="cpu").manual_seed(1234)  # the SAME source on every rank
            ids = torch.randperm(vocab, generator=gs)[:active]
            succ = torch.randint(0, active, (active,), generator=gs)
            self.pool = []
            for _ in range(pool):
                t = torch.empty(batch, seq_len + 1, dtype=torch.long)
                t[:, 0] = torch.randint(0, active, (batch,), generator=g)
                follow = torch.rand(batch, seq_len, generator=g) < p_follow
                rnd = torch.randint(0, active, (batch, seq_len), generator=g)
                for i in range(seq_len):
                    t[:, i + 1] = torch.where(follow[:, i], succ[t[:, i]], rnd[:, i])
                self.pool.append(ids[t].to(device))
        self.i = 0

    def __next__(self):
        t = self.pool[self.i % len(self.pool)]
        self.i += 1
        return t[:, :-1], t[:, 1:]

    def __iter__(self):
        return self

    def state_dict(self):
        return {"i": self.i}

    def load_state_dict(self, sd):
        self.i = int(sd["i"])


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

    def state_dict(self):
        return {"i": self.i}

    def load_state_dict(self, sd):
        self.i = int(sd["i"])


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

    def state_dict(self):
        return {"i": self.i}

    def load_state_dict(self, sd):
        self.i = int(sd["i"])
