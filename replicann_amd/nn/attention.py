"""Scaled dot-product attention heads and multi-head wrappers (after
https://arxiv.org/abs/1706.03762) — source-compatible with the reference
``src/replicann/nn/attention.py`` (R2–R7 in SURVEY.md §2.1).

Same class names, constructor signatures, properties and ``state_dict`` keys
(``_heads.{i}._query.weight`` …, ``_proj.weight/bias``); the per-head
``nn.Linear`` modules stay the parameter storage.  What changes is the
execution: a multi-head forward concatenates the per-head weights into ONE
fused QKV projection (one MFMA GEMM instead of 3·n_heads skinny ones,
reference ``:135-137`` × ``:180``) and runs ONE fused attention kernel over
all heads (``replicann_amd.ops.attention``), whose (B, T, H, D) output is
already the concatenated-heads layout (no ``torch.cat``).

Reference behaviour that is kept on purpose (parity-tested):
  * scale = 1/sqrt(in_dim) = 1/sqrt(embedding size), not 1/sqrt(head size)
    (reference ``:24``; Q1);
  * bool masks: True = masked out; float masks are ADDED (``:39-42``; Q2);
  * head dropout is the head's own ``_dropout.p`` (0.1 unless passed via
    head kwargs) — ``p_dropout`` of the multi-head module is not forwarded
    (``:82``; Q4);
  * ``return_kv=True`` returns the unprojected concatenated outputs
    (``:183-192``; Q5).
Deliberate deviations (crashes in the reference):
  * any floating mask dtype is accepted (reference raises for non-fp32, Q3);
  * ``MultiheadCrossAttention(return_kv=True)`` returns ``(z, k, v)`` like the
    self-attention path (reference crashes, ``:165``; Q6).
"""

from __future__ import annotations

from math import sqrt

import torch
import torch.nn as nn
from torch import Tensor

from .. import ops


def _flatten_lead(x: Tensor):
    """(*lead, T, C) → (N, T, C) and the lead shape (unbatched (T, C) → N=1)."""
    lead = x.shape[:-2]
    return x.reshape(-1, x.shape[-2], x.shape[-1]), lead


def _mask_bias(mask, lead, Tq, Tk, device):
    """Broadcast a reference-semantics mask to a (N|1, Tq, Tk) additive bias."""
    if mask is None:
        return None
    bias = ops.mask_to_bias(mask.to(device))
    if bias.dim() <= 2:
        return bias.reshape(1, *bias.shape[-2:]).expand(1, Tq, Tk)
    full = torch.broadcast_shapes(bias.shape, (*lead, Tq, Tk))
    return bias.expand(full).reshape(-1, Tq, Tk)


class _AttentionHead(nn.Module):
    """Base single head (reference ``nn/attention.py:14-62``)."""

    def __init__(self, in_dim: int, out_dim: int, *, bias: bool = False, p_dropout: float = 0.1) -> None:
        super().__init__()
        self._scale_coeff = 1 / sqrt(in_dim)
        self._query = nn.Linear(in_dim, out_dim, bias=bias)
        self._dropout = nn.Dropout(p_dropout)

    def _attention(self, q: Tensor, k: Tensor, v: Tensor, mask: Tensor | None = None, *,
                   return_kv: bool = False):
        q3, lead = _flatten_lead(q)
        k3, _ = _flatten_lead(k)
        v3, _ = _flatten_lead(v)
        Tq, Tk = q3.shape[1], k3.shape[1]
        bias = _mask_bias(mask, lead, Tq, Tk, q.device)
        z = ops.attention(q3.unsqueeze(2), k3.unsqueeze(2), v3.unsqueeze(2), scale=self._scale_coeff,
                          bias=bias, dropout_p=self._dropout.p, training=self.training)
        z = z.reshape(*lead, Tq, v3.shape[-1])
        if return_kv:
            return z, k, v
        return z

    @property
    def embeddings_size(self) -> int:  # (sic) reference name, Q8
        return self.query.in_features

    @property
    def embedding_size(self) -> int:
        return self.query.in_features

    @property
    def head_size(self) -> int:
        return self.query.out_features

    @property
    def query(self) -> nn.Linear:
        return self._query


class _MultiheadAttention(nn.Module):
    """Base multi-head wrapper (reference ``nn/attention.py:65-98``)."""

    AttentionHead: type

    def __init__(self, n_heads: int, head_size: int, embedding_size: int | None = None, *,
                 head_bias: bool = False, proj_bias: bool = True, p_dropout: float = 0.1,
                 **head_kwargs) -> None:
        super().__init__()
        embedding_size = embedding_size or head_size
        self._heads = nn.ModuleList(
            self.AttentionHead(embedding_size, head_size, bias=head_bias, **head_kwargs)
            for _ in range(n_heads)
        )
        self._proj = nn.Linear(n_heads * head_size, embedding_size, bias=proj_bias)
        self._dropout = nn.Dropout(p_dropout)

    @property
    def embedding_size(self) -> int:
        return self._proj.out_features

    @property
    def head_size(self) -> int:
        return self._proj.in_features // self.n_heads

    @property
    def n_heads(self) -> int:
        return len(self._heads)

    # fused-parameter views --------------------------------------------------
    _FUSED = ("_query",)  # per-head Linears fused into one projection (self-attention: q, k, v)

    def _members(self, kind):
        return [getattr(getattr(h, n), kind) for n in self._FUSED for h in self._heads]

    def _rn_fuse_groups(self):
        """FlatParams packs the per-head weights (and biases) back to back in fused order, so the
        fused projection is a zero-copy view of the flat buffers (utils/flat.py)."""
        groups = [self._members("weight")]
        if self._heads[0]._query.bias is not None:
            groups.append(self._members("bias"))
        return groups

    def _fused_param(self, kind):
        """A leaf Parameter aliasing the packed flat-buffer region of the fused weight / bias
        (its .grad aliases the flat gradient region), or None when the parameters do not live
        in a FlatParams buffer.  Backward kernels accumulate straight into that region and
        notify every member (ops.linear._notify); the optimizer sees only the members."""
        members = self._members(kind)
        if members[0] is None:
            return None
        flat = getattr(members[0], "_rn_flat", None)
        if flat is None:
            return None
        cache = self.__dict__.setdefault("_rn_fused", {})
        hit = cache.get(kind)
        if hit is not None and hit[0] is flat and hit[1] == members[0].data_ptr():
            return hit[2]
        shape = (sum(p.shape[0] for p in members),) + tuple(members[0].shape[1:])
        views = flat.fused_view(members, shape)
        if views is None:
            return None
        proxy = nn.Parameter(views[0], requires_grad=True)
        proxy.grad = views[1]
        proxy._rn_flat = flat
        proxy._rn_members = members

        def _ready(p, flat=flat, members=members):  # autograd-accumulated (non-direct) path
            for m in members:
                flat.mark_ready(m)
        proxy.register_post_accumulate_grad_hook(_ready)
        cache[kind] = (flat, members[0].data_ptr(), proxy)
        return proxy

    def _cat_weights(self, names=None):
        """(weight, bias) of the fused projection: flat-buffer views when the parameters are
        packed (training runs), else a concatenation — cached by the members' versions when no
        gradient is recorded (eval / inference), so repeated forwards do not re-concatenate."""
        w = self._fused_param("weight")
        if w is not None:
            b = self._fused_param("bias") if self._heads[0]._query.bias is not None else None
            return w, b
        ws, bs = self._members("weight"), self._members("bias")
        key = None
        if not torch.is_grad_enabled():
            key = tuple((p.data_ptr(), p._version) for p in ws + [q for q in bs if q is not None])
            hit = self.__dict__.get("_rn_cat_cache")
            if hit is not None and hit[0] == key:
                return hit[1], hit[2]
        w = torch.cat(ws, 0)
        b = torch.cat(bs, 0) if bs[0] is not None else None
        if key is not None:
            self.__dict__["_rn_cat_cache"] = (key, w, b)
        return w, b

    def _out(self, z: Tensor) -> Tensor:
        y = ops.linear(z, self._proj.weight, self._proj.bias)
        return ops.dropout(y, self._dropout.p, self.training)


class CrossAttentionHead(_AttentionHead):
    """Query-only head; k and v arrive already projected (reference ``:101-113``)."""

    def forward(self, x: Tensor, /, k: Tensor, v: Tensor, mask: Tensor | None = None, *,
                return_kv: bool = False):
        q = ops.linear(x, self.query.weight, self.query.bias)
        return self._attention(q, k, v, mask=mask, return_kv=return_kv)


class SelfAttentionHead(_AttentionHead):
    """Head with its own Q/K/V projections (reference ``:116-146``)."""

    def __init__(self, in_dim: int, out_dim: int, *, bias: bool = False, p_dropout: float = 0.1) -> None:
        super().__init__(in_dim=in_dim, out_dim=out_dim, bias=bias, p_dropout=p_dropout)
        self._key = nn.Linear(in_dim, out_dim, bias=bias)
        self._value = nn.Linear(in_dim, out_dim, bias=bias)

    def forward(self, x: Tensor, /, mask: Tensor | None = None, return_kv: bool = False):
        hs = self.head_size
        w = torch.cat([self._query.weight, self._key.weight, self._value.weight], 0)
        b = None
        if self._query.bias is not None:
            b = torch.cat([self._query.bias, self._key.bias, self._value.bias], 0)
        qkv = ops.linear(x, w, b)
        q, k, v = qkv.split(hs, dim=-1)
        return self._attention(q, k, v, mask=mask, return_kv=return_kv)

    @property
    def key(self) -> nn.Linear:
        return self._key

    @property
    def value(self) -> nn.Linear:
        return self._value


class MultiheadCrossAttention(_MultiheadAttention):
    """Multi-head cross attention (reference ``:149-172``).

    k and v (…, Tk, ≥n_heads·(E//n_heads)) are split into n_heads chunks of
    E//n_heads on the last dim (extra columns ignored, reference ``:153-154``).
    """

    AttentionHead = CrossAttentionHead

    def forward(self, x: Tensor, /, k: Tensor, v: Tensor, mask: Tensor | None = None, *,
                return_kv: bool = False):
        H = self.n_heads
        split = self.embedding_size // H
        wq, bq = self._cat_weights()
        q = ops.linear(x, wq, bq)
        kk = k[..., : H * split]
        vv = v[..., : H * split]
        q3, lead = _flatten_lead(q)
        k3, _ = _flatten_lead(kk)
        v3, _ = _flatten_lead(vv)
        N, Tq, Tk = q3.shape[0], q3.shape[1], k3.shape[1]
        if k3.shape[0] != N:
            k3 = k3.expand(N, -1, -1)
            v3 = v3.expand(N, -1, -1)
        bias = _mask_bias(mask, lead, Tq, Tk, x.device)
        h0 = self._heads[0]
        z = ops.attention(q3.reshape(N, Tq, H, -1), k3.reshape(N, Tk, H, split),
                          v3.reshape(N, Tk, H, split), scale=h0._scale_coeff, bias=bias,
                          dropout_p=h0._dropout.p, training=self.training)
        z = z.reshape(*lead, Tq, H * split)
        if return_kv:
            return z, kk, vv
        return self._out(z)


class MultiheadSelfAttention(_MultiheadAttention):
    """Multi-head self attention (reference ``:175-192``), fused QKV + fused attention."""

    AttentionHead = SelfAttentionHead
    _FUSED = ("_query", "_key", "_value")

    def fused_qkv(self, x: Tensor) -> Tensor:
        w, b = self._cat_weights()
        return ops.linear(x, w, b)

    def forward(self, x: Tensor, /, mask: Tensor | None = None, *, return_kv: bool = False):
        H, hs = self.n_heads, self.head_size
        qkv = self.fused_qkv(x)
        qkv3, lead = _flatten_lead(qkv)
        N, T = qkv3.shape[0], qkv3.shape[1]
        packed = qkv3.reshape(N, T, 3, H, hs)
        bias = _mask_bias(mask, lead, T, T, x.device)
        h0 = self._heads[0]
        z = ops.attention_packed(packed, scale=h0._scale_coeff, bias=bias, dropout_p=h0._dropout.p,
                                 training=self.training)
        z = z.reshape(*lead, T, H * hs)
        if return_kv:
            k = packed[:, :, 1].reshape(*lead, T, H * hs)
            v = packed[:, :, 2].reshape(*lead, T, H * hs)
            return z, k, v
        return self._out(z)
