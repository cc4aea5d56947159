"""Data parallelism: bucketed in-place gradient all-reduce overlapped with backward — N15/N16.

One process per GPU, ``torch.distributed`` with backend ``"nccl"`` (= RCCL on
ROCm) over xGMI; ``gloo`` for the CPU tests.  The reference has no
parallelism at all; this is built MI355X-first:

* gradients live in ONE flat buffer (:class:`~replicann_amd.utils.flat.FlatParams`);
  a bucket is a contiguous slice of it, so the all-reduce runs IN PLACE on the
  gradient memory — no bucket copy-in/copy-out kernels;
* buckets are formed in reverse parameter order (the order backward produces
  gradients) and sized for point-to-point xGMI rings (default 64 MB of bf16:
  large enough that RCCL's per-collective latency is amortised over 7 links,
  small enough that the first bucket launches early in the backward);
* a post-accumulate-grad hook per parameter counts arrivals; when a bucket is
  complete its ``all_reduce(SUM, async_op=True)`` is issued at once — RCCL
  runs it on its own HIP stream, ordered after the producing kernels, and it
  overlaps the rest of the backward;
* buckets are always LAUNCHED in index order (a ready bucket waits for its
  predecessors) so every rank issues the same collective sequence;
* the 1/world averaging is NOT a separate pass: it is folded into the fused
  optimizer's ``grad_scale``;
* ``finish()`` waits on the outstanding works (stream-ordered, no host sync),
  launches buckets whose parameters received no gradient (unused parameters:
  their slice is zero on every rank), and checks every bucket was reduced
  exactly once;
* ``no_sync()`` disables reduction for gradient accumulation;
* construction broadcasts rank 0's parameters and buffers (one flat broadcast).
"""

from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist
import torch.nn as nn

from ..utils.flat import FlatParams


class DistributedDataParallel(nn.Module):
    def __init__(self, module: nn.Module, flat: FlatParams, bucket_mb: float = 64.0,
                 process_group=None, broadcast: bool = True, check_unused: bool = False):
        super().__init__()
        self.module = module
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.check_unused = check_unused
        self._sync = True
        self._works = []
        if broadcast and self.world > 1:
            self._broadcast_state()
        # ---- bucket assignment (reverse layout order) ----
        elem = flat.grad.element_size()
        cap = max(1, int(bucket_mb * 1024 * 1024 / elem))
        segs = flat.segments()
        self.buckets = []  # (lo, hi, n_params)
        self.param_bucket = {}
        cur_hi = None
        cur_lo = None
        cur_n = 0
        for p, off, n in reversed(segs):
            end = off + ((n + 63) // 64) * 64
            if cur_hi is None:
                cur_hi, cur_lo, cur_n = end, off, 0
            elif cur_hi - off > cap and cur_n > 0:
                self.buckets.append([cur_lo, cur_hi, cur_n])
                cur_hi, cur_lo, cur_n = end, off, 0
            cur_lo = off
            cur_n += 1
            self.param_bucket[id(p)] = len(self.buckets)
        self.buckets.append([cur_lo, cur_hi, cur_n])
        self._pending = [b[2] for b in self.buckets]
        self._ready = [False] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._next = 0
        self._seen = set()
        self.launched_in_backward = 0  # buckets whose all-reduce was issued from a gradient hook (last step)
        self._hooks = [p.register_post_accumulate_grad_hook(self._hook) for p, _, _ in segs]
        flat.ready_hooks.append(self._hook)  # parameters whose grads are accumulated directly by kernels

    # ------------------------------------------------------------------
    def _broadcast_state(self):
        dist.broadcast(self.flat.data, 0, group=self.pg)
        for b in self.module.buffers():
            dist.broadcast(b.data, 0, group=self.pg)

    def _reset(self):
        self._pending = [b[2] for b in self.buckets]
        self._ready = [False] * len(self.buckets)
        self._launched = [False] * len(self.buckets)
        self._next = 0
        self._works = []
        self._seen = set()
        self.launched_in_backward = 0

    def _launch_ready(self, from_hook=False):
        while self._next < len(self.buckets) and self._ready[self._next]:
            self.launched_in_backward += int(from_hook)
            lo, hi, _ = self.buckets[self._next]
            w = dist.all_reduce(self.flat.grad[lo:hi], op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            self._works.append(w)
            self._launched[self._next] = True
            self._next += 1

    def _hook(self, p):
        if not self._sync or self.world == 1:
            return
        if id(p) in self._seen:  # a parameter used twice accumulates twice: count once
            return
        self._seen.add(id(p))
        bi = self.param_bucket[id(p)]
        self._pending[bi] -= 1
        if self._pending[bi] == 0:
            self._ready[bi] = True
            self._launch_ready(from_hook=True)

    # ------------------------------------------------------------------
    def forward(self, *args, **kwargs):
        if self._sync:
            self._reset()
        return self.module(*args, **kwargs)

    def finish(self):
        """Complete the gradient reduction (call after backward, before the optimizer)."""
        if not self._sync or self.world == 1:
            return
        unused = [i for i, r in enumerate(self._ready) if not r]
        if unused and self.check_unused:
            names = [self.flat.names.get(id(p), "?") for p, _, _ in self.flat.segments()
                     if id(p) not in self._seen]
            raise RuntimeError(f"parameters received no gradient this step: {names[:8]}")
        for i in unused:
            self._ready[i] = True
        self._launch_ready()
        for w in self._works:
            w.wait()
        assert all(self._launched), "a gradient bucket was never reduced"
        self._works = []

    @contextlib.contextmanager
    def no_sync(self):
        prev = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = prev

    @property
    def grad_scale(self):
        return 1.0 / self.world
