"""Fused optimizers over a :class:`FlatParams` buffer (csrc/kernels/optim.hip) — N12/N13.

Mixed-precision policy (N23): model parameters live in bf16 (what the GEMMs
read), the optimizer owns an fp32 master copy and fp32 moments.  One step is:

0. ``opt_prep`` (1 thread): step counter, LR schedule (constant or warmup +
   cosine) and Adam bias corrections are computed IN DEVICE MEMORY, so a
   captured hipGraph of the whole training step replays correct per-step
   hyper-parameters;
1. ``grad_norm`` kernel: Σ g² over the flat bf16 gradient → a device scalar
   (block partials + a fixed-order final reduce: deterministic);
2. ONE update kernel over every parameter: reads g (bf16), applies the DDP
   averaging factor and the clip coefficient min(1, max_norm/‖g‖) *from
   device memory* (no host sync), updates m, v and the fp32 master, writes the
   bf16 parameter.  A non-finite ‖g‖ turns the whole step into a no-op
   in-kernel (the NaN/Inf step guard of SURVEY.md §5).

Weight decay applies to ≥2-D parameters only (per-64-element granule mask).
On CPU the same math runs as vectorised torch ops on the flat buffers.
"""

from __future__ import annotations

import math

import torch

from .. import _ext
from ..utils.flat import ALIGN, FlatParams


class _FlatOptimizer:
    def __init__(self, flat: FlatParams, lr, weight_decay, max_grad_norm, grad_scale):
        self.flat = flat
        self.lr = lr
        self.weight_decay = weight_decay
        self.max_grad_norm = max_grad_norm
        self.grad_scale = grad_scale  # e.g. 1/world_size for DDP SUM-reduced grads
        self.step_count = 0
        self.post_step_hooks = []  # callables run at the end of every step (fp8 weight cache refresh)
        # gradient the step reads: the flat bf16 .grad buffer, or (data parallel) the fp32
        # all-reduced copy the DDP reducer owns (``DistributedDataParallel.grad_source``)
        self.grad_source = None
        dev = flat.data.device
        self.master = flat.data.float() if flat.data.dtype != torch.float32 else flat.data
        # device state: [‖g‖², skipped flag, step t, lr, bc1, bc2, -, -]
        self.norm_buf = torch.zeros(8, dtype=torch.float32, device=dev)
        self.schedule = None  # (warmup, total, min_ratio) → warmup + cosine; None → constant lr
        self._wd_elem = None

    @property
    def native(self):
        return _ext.use_native(self.flat.data)

    @property
    def grad(self):
        return self.grad_source if self.grad_source is not None else self.flat.grad

    def grad_norm(self):
        """Global L2 norm of the (scaled) gradient as a device tensor."""
        if self.native:
            _ext.ops().sumsq(self.grad, self.norm_buf)
        else:
            self.norm_buf[0] = self.grad.float().pow(2).sum()
        return self.norm_buf[0].sqrt() * self.grad_scale

    def _wd_elementwise(self):
        if self._wd_elem is None:
            self._wd_elem = self.flat.wd_mask.repeat_interleave(ALIGN).to(torch.float32)
        return self._wd_elem

    def zero_grad(self):
        self.flat.zero_grad()

    def _post_step(self):
        """Run the registered post-step hooks (e.g. the fp8 weight cache refresh): stream-ordered
        after the update, and captured with it when the step is graph-captured."""
        for h in self.post_step_hooks:
            h()

    def set_schedule(self, warmup, total, min_ratio=0.1):
        """Warmup + cosine decay, evaluated on device each step (graph-safe)."""
        self.schedule = (float(warmup), float(total), float(min_ratio))

    def _host_lr(self, lr):
        if lr is not None:
            return lr
        if self.schedule is None:
            return self.lr
        w, t, r = self.schedule
        return cosine_lr(self.step_count - 1, self.lr, int(w), int(t), r)

    def _prep(self, lr, b1=0.0, b2=0.0):
        w, t, r = self.schedule if self.schedule is not None else (0.0, 1.0, 1.0)
        _ext.ops().opt_prep(self.norm_buf, self.lr, w, t, r, self.schedule is not None,
                            -1.0 if lr is None else float(lr), b1, b2)

    def state_tensors(self):
        """Every device tensor a step mutates (parameters, master, moments, device state)."""
        ts = [self.flat.data, self.norm_buf] + [t for t in self._extra_state() if t is not None]
        if self.master is not self.flat.data:
            ts.append(self.master)
        return ts

    def _extra_state(self):
        return []

    def _load_flat(self, sd, key, dst):
        """Restore one flat fp32 state tensor, remapping it when the checkpoint's parameter layout
        (``sd["layout"]``) differs from this buffer's (e.g. a fusion-group repacking since)."""
        src = sd[key]
        lay = sd.get("layout")
        if lay is None:
            if src.numel() != dst.numel():
                raise ValueError(f"optimizer state {key!r} has {src.numel()} elements, the model {dst.numel()}")
            import warnings
            warnings.warn("optimizer state has no parameter layout record (older checkpoint): "
                          "assuming it matches this model's flat layout")
            dst.copy_(src)
            return
        lay = [tuple(e) for e in lay]
        if lay == self.flat.layout():
            dst.copy_(src)
        else:
            tmp = torch.zeros_like(dst)
            self.flat.remap_from(lay, src.to(dst.device), tmp)
            dst.copy_(tmp)

    def skipped_last_step(self):
        return bool(self.norm_buf[1].item())


class FusedAdamW(_FlatOptimizer):
    """AdamW on the flat buffer (fp32 master, moments).  ``stochastic_round``: the bf16 weight copy
    the forward reads is written with stochastic rounding (unbiased), so updates smaller than half a
    bf16 ulp of the weight — every update at warm-up learning rates for |w| ≳ 4e-3 — still move the
    weights the model computes with in expectation instead of being rounded away."""

    def __init__(self, flat: FlatParams, lr=6e-4, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1,
                 max_grad_norm=1.0, grad_scale=1.0, stochastic_round=False):
        super().__init__(flat, lr, weight_decay, max_grad_norm, grad_scale)
        self.betas, self.eps = betas, eps
        self.stochastic_round = bool(stochastic_round)
        self.m = torch.zeros_like(self.master)
        self.v = torch.zeros_like(self.master)

    def step(self, lr=None):
        """One update.  ``lr`` overrides the schedule for this step (eager use only:
        under graph capture leave it None so the device schedule is used)."""
        self.step_count += 1
        b1, b2 = self.betas
        clip = self.max_grad_norm if self.max_grad_norm else 0.0
        if self.native:
            ops = _ext.ops()
            self._prep(lr, b1, b2)
            ops.sumsq(self.grad, self.norm_buf)
            ops.adamw_step(self.flat.data, self.master, self.grad, self.m, self.v, self.flat.wd_mask,
                           self.norm_buf, b1, b2, self.eps, self.weight_decay, self.grad_scale, clip,
                           self.stochastic_round)
            self._post_step()
            return
        lr = self._host_lr(lr)
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        g = self.grad.float() * self.grad_scale
        norm = g.pow(2).sum().sqrt()
        if not torch.isfinite(norm):
            return
        if clip > 0:
            g = g * min(1.0, clip / (float(norm) + 1e-6))
        self.m.mul_(b1).add_(g, alpha=1 - b1)
        self.v.mul_(b2).addcmul_(g, g, value=1 - b2)
        denom = (self.v / bc2).sqrt_().add_(self.eps)
        upd = (self.m / bc1) / denom + self.weight_decay * self._wd_elementwise() * self.master
        self.master.add_(upd, alpha=-lr)
        if self.master is not self.flat.data:
            self.flat.data.copy_(self.master)
        self._post_step()

    def _extra_state(self):
        return [self.m, self.v]

    def state_dict(self):
        return {"step": self.step_count, "master": self.master, "m": self.m, "v": self.v, "lr": self.lr,
                "layout": self.flat.layout()}

    def load_state_dict(self, sd):
        self.step_count = sd["step"]
        self.norm_buf[2] = float(self.step_count)
        self._load_flat(sd, "master", self.master)
        self._load_flat(sd, "m", self.m)
        self._load_flat(sd, "v", self.v)
        self.lr = sd.get("lr", self.lr)
        # the parameters themselves are NOT re-derived from the fp32 master: the model state_dict
        # carries the exact (stochastically rounded) bf16 copy the saving run used, and a
        # round-to-nearest master -> bf16 copy here made a resumed GPU run diverge from the
        # uninterrupted one at its first forward


class FusedSGD(_FlatOptimizer):
    """SGD with momentum (+ Nesterov) and decoupled-free L2 weight decay (torch semantics)."""

    def __init__(self, flat: FlatParams, lr=0.1, momentum=0.9, weight_decay=1e-4, nesterov=False,
                 max_grad_norm=0.0, grad_scale=1.0):
        super().__init__(flat, lr, weight_decay, max_grad_norm, grad_scale)
        self.momentum, self.nesterov = momentum, nesterov
        self.buf = torch.zeros_like(self.master)

    def step(self, lr=None):
        self.step_count += 1
        clip = self.max_grad_norm if self.max_grad_norm else 0.0
        first = self.step_count == 1
        if self.native:
            ops = _ext.ops()
            self._prep(lr)
            ops.sumsq(self.grad, self.norm_buf)
            ops.sgd_step(self.flat.data, self.master, self.grad, self.buf, self.flat.wd_mask,
                         self.norm_buf, self.momentum, self.weight_decay, self.nesterov, self.grad_scale, clip)
            self._post_step()
            return
        lr = self._host_lr(lr)
        g = self.grad.float() * self.grad_scale
        norm = g.pow(2).sum().sqrt()
        if not torch.isfinite(norm):
            return
        if clip > 0:
            g = g * min(1.0, clip / (float(norm) + 1e-6))
        g = g + self.weight_decay * self._wd_elementwise() * self.master
        if first:
            self.buf.copy_(g)
        else:
            self.buf.mul_(self.momentum).add_(g)
        d = g + self.momentum * self.buf if self.nesterov else self.buf
        self.master.add_(d, alpha=-lr)
        if self.master is not self.flat.data:
            self.flat.data.copy_(self.master)

    def _extra_state(self):
        return [self.buf]

    def state_dict(self):
        return {"step": self.step_count, "master": self.master, "buf": self.buf, "lr": self.lr,
                "layout": self.flat.layout()}

    def load_state_dict(self, sd):
        self.step_count = sd["step"]
        self.norm_buf[2] = float(self.step_count)
        self._load_flat(sd, "master", self.master)
        self._load_flat(sd, "buf", self.buf)  # parameters: from the model state_dict (see FusedAdamW)


def cosine_lr(step, base_lr, warmup, total, min_ratio=0.1):
    if step < warmup:
        return base_lr * (step + 1) / warmup
    t = min(1.0, (step - warmup) / max(1, total - warmup))
    return base_lr * (min_ratio + (1 - min_ratio) * 0.5 * (1 + math.cos(math.pi * t)))
