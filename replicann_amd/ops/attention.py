"""Fused scaled-dot-product attention (csrc/kernels/attention.hip).

Replaces the reference's per-head Python loop
(``src/replicann/nn/attention.py:28-50`` — ``q@kᵀ*scale`` → mask → softmax →
dropout → ``@v`` — called once per head at ``:180``) with one flash-style
kernel over all (batch, head) pairs: scores never reach HBM, the online softmax
runs in registers, dropout is a counter-based in-kernel RNG regenerated in the
backward, and the backward recomputes P from the saved log-sum-exp.

Layout is "token-major, heads interleaved": q, k, v are (B, T, H, D) views
straight out of the fused QKV GEMM (row stride 3·H·D), and the output is
(B, T, H, D) contiguous — i.e. already the (B, T, H·D) input of the output
projection, so the reference's ``torch.cat`` of heads disappears.

Supported semantics (all needed for reference parity, SURVEY.md §2.1 Q1–Q4):
  * arbitrary ``scale`` (the reference uses 1/sqrt(embedding_size), Q1);
  * ``causal`` — true causal tile skipping (GPT-2);
  * ``bias`` — an additive float mask (B|1, Tq, Tk) (the reference's 0/1
    "tril" float mask is *added*, Q2; bool masks become -inf biases);
  * ``dropout_p`` on the attention probabilities (Q4).
"""

from __future__ import annotations


import torch

from .. import _ext


MFMA_HEAD_DIMS = (32, 64, 128)


def attention_is_mfma(head_dim: int) -> bool:
    """True if ``head_dim`` runs on the MFMA flash kernels (deterministic, no atomics); other head
    sizes take the generic per-query-row kernels (fp32 atomics in the backward)."""
    return int(head_dim) in MFMA_HEAD_DIMS


def mask_to_bias(mask, dtype=torch.float32):
    """Reference mask semantics → additive bias.

    bool: True = masked out (-inf), ``nn/attention.py:39-40``;
    float (any float dtype — the reference only accepts fp32, Q3): added as-is.
    """
    if mask is None:
        return None
    if mask.dtype == torch.bool:
        return torch.zeros(mask.shape, dtype=dtype, device=mask.device).masked_fill(mask, float("-inf"))
    if mask.is_floating_point():
        return mask.to(dtype)
    raise TypeError(f"Unexpected type `{mask.dtype}` of the `mask`.")


def _bias_3d(bias, B, Tq, Tk):
    if bias is None:
        return None
    b = bias
    while b.dim() < 3:
        b = b.unsqueeze(0)
    if b.dim() > 3:
        b = b.reshape(-1, b.shape[-2], b.shape[-1])
    return b.expand(b.shape[0] if b.shape[0] in (1, B) else B, Tq, Tk).float().contiguous()


def attention_reference(q, k, v, scale, causal=False, bias=None, dropout_p=0.0, training=False):
    """fp32 math reference in the (B, T, H, D) layout."""
    qt = q.transpose(1, 2).float()
    kt = k.transpose(1, 2).float()
    vt = v.transpose(1, 2).float()
    w = qt @ kt.transpose(-2, -1) * scale
    if bias is not None:
        b = bias.float()
        if b.dim() == 3:
            b = b.unsqueeze(1)
        w = w + b
    if causal:
        Tq, Tk = w.shape[-2], w.shape[-1]
        m = torch.ones(Tq, Tk, dtype=torch.bool, device=w.device).triu(1 + Tk - Tq)
        w = w.masked_fill(m, float("-inf"))
    p = torch.softmax(w, dim=-1)
    if dropout_p > 0 and training:
        p = torch.nn.functional.dropout(p, dropout_p, True)
    o = p @ vt
    return o.transpose(1, 2).to(q.dtype)


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, bias, scale, causal, dropout_p, seed):
        # seed: None, or a 1-element int64 device tensor (ops/rng.py) the kernels read
        o, lse = _ext.ops().attn_fwd(q, k, v, bias, scale, causal, dropout_p, 0, seed)
        ctx.save_for_backward(q, k, v, o, lse, bias)
        ctx.scale, ctx.causal, ctx.dropout_p, ctx.seed = scale, causal, dropout_p, seed
        return o

    @staticmethod
    def backward(ctx, do):
        from ..parallel.windows import open_window
        q, k, v, o, lse, bias = ctx.saved_tensors
        open_window()
        dq, dk, dv = _ext.ops().attn_bwd(do.contiguous(), q, k, v, o, lse, bias, ctx.scale, ctx.causal,
                                         ctx.dropout_p, 0, ctx.seed)
        return dq, dk, dv, None, None, None, None, None


def attention(q, k, v, *, scale=None, causal=False, bias=None, mask=None, dropout_p=0.0,
              training=False):
    """O = softmax(q·kᵀ·scale + bias [causal]) [dropout] · v, all in (B, T, H, D)."""
    B, Tq, H, D = q.shape
    Tk = k.shape[1]
    if scale is None:
        scale = D ** -0.5
    if mask is not None:
        bias = mask_to_bias(mask) if bias is None else bias + mask_to_bias(mask)
    p = dropout_p if training else 0.0
    if _ext.use_native(q):
        b3 = _bias_3d(bias, B, Tq, Tk)
        from .rng import next_seed
        seed = next_seed(q.device) if p > 0 else None  # drawn on the device: graph-capturable
        return _AttnFn.apply(q, k, v, b3, float(scale), bool(causal), float(p), seed)
    return attention_reference(q, k, v, scale, causal, bias, p, training)


# the attention backward's e5m2 dQKV for an fp8 QKV projection (a test hook, not an env knob: the tests
# compare it with the path where c_attn quantises a bf16 dQKV itself)
ATTN_Q8 = True


class _AttnPackedFn(torch.autograd.Function):
    """Attention on a packed (B, T, 3, H, D) QKV tensor; backward writes one packed dQKV."""

    @staticmethod
    def forward(ctx, qkv, bias, scale, causal, dropout_p, seed, producer_bias, consumer8=None):
        q, k, v = qkv.unbind(2)
        o, lse = _ext.ops().attn_fwd(q, k, v, bias, scale, causal, dropout_p, 0, seed)
        ctx.save_for_backward(qkv, o, lse, bias)
        ctx.scale, ctx.causal, ctx.dropout_p, ctx.seed = scale, causal, dropout_p, seed
        ctx.producer_bias = producer_bias
        # the fp8 projection that produced qkv (its backward consumes dQKV): the plan its forward recorded
        ctx.consumer8 = consumer8
        ctx.plan8 = tuple(consumer8.bwd_plan) if consumer8 is not None else (False, False)
        return o

    @staticmethod
    def backward(ctx, do):
        from .linear import _direct_grad, _notify
        from ..parallel.windows import open_window
        qkv, o, lse, bias = ctx.saved_tensors
        q, k, v = qkv.unbind(2)
        open_window()  # queued gradient collectives run beside the attention backward's short workgroups
        dqkv = torch.empty_like(qkv)
        dq, dk, dv = dqkv.unbind(2)
        pb = ctx.producer_bias
        B, T, _, H, D = qkv.shape
        pb_acc = _direct_grad(pb) if (pb is not None and attention_is_mfma(D) and pb.numel() == 3 * H * D) else None
        c8 = ctx.consumer8
        done = False
        if ATTN_Q8 and c8 is not None and c8.g_ready and (pb_acc is not None or pb is None) and any(ctx.plan8):
            # dQKV also in e5m2 from the kernels (the consumer's delayed scale): the projection's fp8
            # gradients skip their quantisation pass; when it takes BOTH in fp8 (and its bias gradient came
            # from these kernels) the bf16 dQKV is never read, so it is not written at all
            q8 = torch.empty(qkv.shape, device=qkv.device, dtype=torch.uint8)
            q8_only = all(ctx.plan8)
            done = _ext.ops().attn_bwd_out_q8(do.contiguous(), q, k, v, o, lse, bias, ctx.scale, ctx.causal,
                                              ctx.dropout_p, 0, dq, dk, dv, pb_acc, ctx.seed, q8,
                                              c8.gslot(qkv.device), q8_only)
            if done:
                c8.goffer(dqkv, q8)
        if not done:
            _ext.ops().attn_bwd_out(do.contiguous(), q, k, v, o, lse, bias, ctx.scale, ctx.causal,
                                    ctx.dropout_p, 0, dq, dk, dv, pb_acc, ctx.seed)
        if pb_acc is not None:  # Σ_rows dQKV reduced in the kernels: the c_attn bias gradient
            pb._rn_bias_done = True
            _notify(pb)
        return dqkv, None, None, None, None, None, None, None


def attention_packed(qkv, *, scale=None, causal=False, bias=None, mask=None, dropout_p=0.0,
                     training=False, producer_bias=None, consumer8=None):
    """Attention over a packed (B, T, 3, H, D) tensor → (B, T, H, D).

    ``producer_bias``: bias of the projection that produced ``qkv`` (3·H·D); its gradient
    Σ_rows dQKV is then reduced by the attention backward kernels (per-block column
    partials) and accumulated into the flat gradient, and the projection skips its own
    bias pass.  ``consumer8``: the Fp8State of that projection when it runs in fp8 — the backward kernels
    then also emit dQKV in e5m2 for its fp8 gradients (see _AttnPackedFn.backward)."""
    B, T, three, H, D = qkv.shape
    if scale is None:
        scale = D ** -0.5
    if mask is not None:
        bias = mask_to_bias(mask) if bias is None else bias + mask_to_bias(mask)
    p = dropout_p if training else 0.0
    if _ext.use_native(qkv):
        b3 = _bias_3d(bias, B, T, T)
        from .rng import next_seed
        seed = next_seed(qkv.device) if p > 0 else None
        return _AttnPackedFn.apply(qkv, b3, float(scale), bool(causal), float(p), seed, producer_bias, consumer8)
    q, k, v = qkv.unbind(2)
    return attention_reference(q, k, v, scale, causal, bias, p, training)


def attention_decode(q, k, v, mask=None, scale=None):
    """One new query per (batch, head) against a KV cache — q (B, 1, H, D), k / v (B, Tk, H, D) —
    with an additive key mask (Tk values shared by the batch, or None).  Inference only.  On the GPU
    at head size 64 one launch of the one-query kernel (csrc/kernels/attention_decode.hip: a workgroup
    per (batch, head), no query tiling); otherwise the general attention."""
    B, Tq, H, D = q.shape
    if scale is None:
        scale = D ** -0.5
    Tk = k.shape[1]
    if _ext.use_native(q) and Tq == 1 and D == 64 and Tk <= 1024 and not torch.is_grad_enabled():
        m = mask.reshape(-1) if mask is not None else None
        if m is None or (m.numel() == Tk and m.dtype == torch.float32 and m.is_contiguous()):
            return _ext.ops().attn_decode(q, k, v, m, float(scale))
    return attention(q, k, v, scale=scale, bias=mask)
