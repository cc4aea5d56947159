"""Flat, HBM-resident parameter / gradient storage.

Every trainable parameter becomes a view into ONE contiguous buffer (and its
``.grad`` a view into ONE contiguous gradient buffer), each parameter aligned
to 64 elements (128 B for bf16) so vector kernels never straddle parameters.
Consequences that the rest of the framework is built on:

* the fused optimizers are one kernel launch over the whole model (no
  multi-tensor-apply gather lists);
* data-parallel gradient buckets are contiguous slices of the gradient buffer,
  all-reduced in place (no copy into / out of bucket staging buffers);
* ``zero_grad`` is one memset; the global grad-norm is one reduction.

Parameters are laid out in registration order; backward produces gradients
roughly in reverse of that, which is what the DDP bucketing exploits.
"""

from __future__ import annotations

import torch
import torch.nn as nn

ALIGN = 64


def _round(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class FlatParams:
    def __init__(self, module: nn.Module, dtype=None, device=None, grad_dtype=None, direct=True):
        self.params = [p for p in module.parameters() if p.requires_grad]
        if not self.params:
            raise ValueError("module has no trainable parameters")
        dtype = dtype or self.params[0].dtype
        device = torch.device(device) if device is not None else self.params[0].device
        grad_dtype = grad_dtype or dtype
        self.offsets = []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            off += _round(p.numel())
        self.numel = off
        self.data = torch.zeros(off, dtype=dtype, device=device)
        self.grad = torch.zeros(off, dtype=grad_dtype, device=device)
        for p, o in zip(self.params, self.offsets):
            n = p.numel()
            view = self.data[o:o + n].view(p.shape)
            view.copy_(p.data.reshape(p.shape))
            p.data = view
            p.grad = self.grad[o:o + n].view(p.shape)
        self.names = {}
        for name, p in module.named_parameters():
            self.names[id(p)] = name
        # Direct gradient accumulation: backward kernels of single-use parameters
        # write/accumulate straight into the flat .grad views and then call
        # mark_ready() (which drives DDP bucketing) instead of going through
        # autograd's AccumulateGrad add.
        self.direct = direct
        self.ready_hooks = []
        self.contribution_hooks = []  # (param, final) per direct contribution of a multi-use parameter
        for p in self.params:
            p._rn_flat = self
        # per-64-element-granule weight-decay flag (matrices decay; vectors don't)
        wd = torch.zeros(off // ALIGN, dtype=torch.uint8)
        for p, o in zip(self.params, self.offsets):
            if p.dim() >= 2:
                wd[o // ALIGN:(o + _round(p.numel())) // ALIGN] = 1
        self.wd_mask = wd.to(device)

    def zero_grad(self):
        self.grad.zero_()
        for p in self.params:  # multi-use parameters restart their contribution count
            if hasattr(p, "_rn_pending"):
                del p._rn_pending
        # autograd may have replaced a .grad (e.g. set_to_none elsewhere): re-point
        for p, o in zip(self.params, self.offsets):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + 1].data_ptr():
                p.grad = self.grad[o:o + p.numel()].view(p.shape)

    def mark_ready(self, p):
        for h in self.ready_hooks:
            h(p)

    def contributed(self, p, final):
        for h in self.contribution_hooks:
            h(p, final)

    def segments(self):
        """[(param, offset, numel)] in layout order."""
        return [(p, o, p.numel()) for p, o in zip(self.params, self.offsets)]
