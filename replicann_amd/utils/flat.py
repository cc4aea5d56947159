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

Fusion groups: a module may declare ``_rn_fuse_groups()`` → lists of parameters that
one kernel consumes as ONE tensor (the reference blocks' per-head Q/K/V ``nn.Linear``
weights, reference ``nn/attention.py:131-137``, are a fused QKV projection here).  A
group is packed back to back, in the listed order, at the position of its first
member, so the fused weight (and its gradient) is a zero-copy view of the flat buffers
(:meth:`fused_view`) — no ``torch.cat`` per forward, no split of the gradient.
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
        trainable = {id(p) for p in self.params}
        group_of = {}
        for m in module.modules():
            fg = getattr(m, "_rn_fuse_groups", None)
            if not callable(fg):
                continue
            for g in fg():
                g = list(g)
                if (len(g) > 1 and all(id(p) in trainable and id(p) not in group_of for p in g)
                        and len({id(p) for p in g}) == len(g) and len({p.dtype for p in g}) == 1):
                    for p in g:
                        group_of[id(p)] = g
        order, seen = [], set()
        for p in self.params:
            if id(p) in seen:
                continue
            for q in group_of.get(id(p), [p]):
                order.append(q)
                seen.add(id(q))
        self.params = order
        self.offsets = []
        self.ends = []  # allocation end of each parameter (packed group members: the next member's start)
        off = 0
        for i, p in enumerate(self.params):
            self.offsets.append(off)
            g = group_of.get(id(p))
            packed_next = g is not None and p is not g[-1]
            off = off + p.numel() if packed_next else _round(off + p.numel())
            self.ends.append(off)
        self._group_of = group_of
        self._index = {id(p): i for i, p in enumerate(self.params)}
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
        for p, o, e in zip(self.params, self.offsets, self.ends):
            if p.dim() >= 2:  # (a packed group is all matrices or all vectors)
                wd[o // ALIGN:_round(e) // ALIGN] = 1
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

    def layout(self):
        """[(name, offset, numel)] of every parameter in layout order: what a raw flat-buffer
        snapshot (optimizer master / moments) means.  Saved with optimizer state so a checkpoint
        written under another packing (fusion groups, alignment) is remapped, never misread."""
        return [(self.names.get(id(p), f"#{i}"), int(o), int(p.numel()))
                for i, (p, o) in enumerate(zip(self.params, self.offsets))]

    def remap_from(self, saved_layout, flat_tensor, out):
        """Copy a flat tensor laid out by ``saved_layout`` into ``out`` (this buffer's layout),
        parameter by parameter, matched by name and size.  Raises if a parameter is missing."""
        old = {n: (o, k) for n, o, k in saved_layout}
        for n, o, k in self.layout():
            if n not in old or old[n][1] != k:
                raise ValueError(f"optimizer state has no entry of {k} elements for parameter {n!r}")
            so = old[n][0]
            out[o:o + k].copy_(flat_tensor[so:so + k])

    def span(self, p):
        """(offset, allocation end) of parameter ``p`` in the flat buffers."""
        i = self._index[id(p)]
        return self.offsets[i], self.ends[i]

    def fused_view(self, members, shape):
        """(data view, grad view) of a packed fusion group, in ``shape``, or None when ``members``
        is not one of this buffer's groups (packed back to back in exactly this order)."""
        g = self._group_of.get(id(members[0]))
        if g is None or len(g) != len(members) or any(a is not b for a, b in zip(g, members)):
            return None
        lo = self.offsets[self._index[id(g[0])]]
        n = sum(p.numel() for p in g)
        return self.data[lo:lo + n].view(shape), self.grad[lo:lo + n].view(shape)
