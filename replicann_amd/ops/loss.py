"""Fused softmax cross-entropy (csrc/kernels/xent.hip) — N9.

Forward: one pass over each logits row (vocab 50257 for GPT-2, padded
storage allowed) computing the row log-sum-exp and the NLL; nothing but the
per-row lse is saved.  Backward: one pass that writes
``(softmax - onehot) · g / n_valid`` **in place over the logits storage**
(the logits are dead after the loss), so the 1.6 GB logits tensor of a
GPT-2 step is read twice and written once in total.

``n_valid_cols`` lets the logits be stored padded (e.g. 50304 = 393·128
columns for GEMM tiling) while the loss only sees the first 50257 columns.
"""

from __future__ import annotations

import torch
import torch.nn.functional as F

from .. import _ext


class _XentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, n_valid_cols, ignore_index, inplace_grad):
        loss_rows, lse = _ext.ops().xent_fwd(logits, target, n_valid_cols, ignore_index, False)
        n = (target != ignore_index).sum().clamp_min(1).float()
        ctx.save_for_backward(logits, target, lse, n)
        ctx.n_valid_cols, ctx.ignore_index, ctx.inplace = n_valid_cols, ignore_index, inplace_grad
        return loss_rows.sum() / n

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, n = ctx.saved_tensors
        scale = (g.float() / n).reshape(1)
        grad = logits if ctx.inplace else torch.empty_like(logits)
        _ext.ops().xent_bwd(logits, target, lse, scale, grad, ctx.n_valid_cols, ctx.ignore_index)
        return grad, None, None, None, None


def cross_entropy(logits, target, *, n_valid_cols=None, ignore_index=-100, inplace_grad=False):
    """Mean token cross-entropy of (N, V) logits against (N,) int targets."""
    V = logits.shape[-1]
    nv = V if n_valid_cols is None else n_valid_cols
    lg = logits.reshape(-1, V)
    tg = target.reshape(-1)
    if _ext.use_native(lg):
        if not lg.is_contiguous():
            lg = lg.contiguous()
        return _XentFn.apply(lg, tg.long().contiguous(), nv, ignore_index, inplace_grad)
    return F.cross_entropy(lg[:, :nv].float(), tg.long(), ignore_index=ignore_index)


class _LinearXentFn(torch.autograd.Function):
    """LM head + cross-entropy fused at the autograd level:
    logits = h·Wᵀ (MFMA GEMM) → CE forward writes the UNSCALED gradient
    (softmax − onehot) over the logits in place → backward runs the two LM-head
    GEMMs on that buffer with alpha = g / n_valid read from device memory in
    their epilogues.  The 1.6 GB logits tensor of a GPT-2 step is written once
    and read twice (CE pass + the two backward GEMMs read it anyway)."""

    @staticmethod
    def forward(ctx, h, weight, target, n_valid_cols, ignore_index):
        ops = _ext.ops()
        shp = h.shape
        h2 = h.reshape(-1, shp[-1]).contiguous()
        logits = ops.gemm(h2, weight, False, True, None, None, 0, None, None, False, 0, False, None, -1)
        tg = target.reshape(-1).long().contiguous()
        loss_rows, _ = ops.xent_fwd(logits, tg, n_valid_cols, ignore_index, True)
        n = (tg != ignore_index).sum().clamp_min(1).float()
        ctx.save_for_backward(h2, weight, logits, n)
        ctx.shp = shp
        return loss_rows.sum() / n

    @staticmethod
    def backward(ctx, g):
        from .linear import _direct_grad, _notify
        h2, weight, dlogits, n = ctx.saved_tensors
        alpha = (g.float() / n).reshape(1)
        ops = _ext.ops()
        gh = gw = None
        if ctx.needs_input_grad[0]:
            # g/n as the epilogue alpha (fp32, before the bf16 rounding): no separate scaling pass
            gh = ops.gemm(dlogits, weight, False, False, None, None, 0, None, None, False, 0, False, alpha, -1)
            gh = gh.reshape(ctx.shp)
        if ctx.needs_input_grad[1]:
            acc = _direct_grad(weight)
            if acc is not None:
                ops.gemm(dlogits, h2, True, False, None, None, 0, None, acc, True, -1, False, alpha, -1)
                _notify(weight)
            else:
                gw = ops.gemm(dlogits, h2, True, False, None, None, 0, None, None, False, -1, False, alpha, -1)
        return gh, gw, None, None, None


class _ChunkedLinearXentFn(torch.autograd.Function):
    """LM head + cross-entropy over row chunks: peak logits memory rows·V → chunk·V.

    The loss's gradients are formed DURING the forward, one chunk at a time, while that
    chunk's logits are live: logits_c = h_c·Wᵀ → CE writes (softmax − onehot) in place →
    dh_c = that·W / n (straight into dh's rows) and dW += thatᵀ·h_c / n (fp32, accumulated
    by the GEMM epilogue).  One logits buffer of ``chunk`` rows is reused by every chunk.
    The backward only scales the two stored gradients by the incoming g.

    Cost (GPT-2-small b64, 65,536 rows, V = 50,304): the unchunked path holds a 6.6 GB bf16
    logits tensor; chunks of 16,384 rows hold 1.65 GB plus dh (bf16, 100 MB) and dW (fp32,
    154 MB).  The GEMM FLOPs are the same; the smaller-M dgrad shapes need split-K to fill
    256 CUs (the runtime autotuner picks it).  Measured cost in ``profiles/lmhead_chunk_*``.
    Default off (``GPT2Config.ce_chunk = 0``): on a 288 GB device the whole-batch logits fit,
    and the chunked form pays the split-K reduction and the backward scaling passes."""

    @staticmethod
    def forward(ctx, h, weight, target, n_valid_cols, ignore_index, chunk):
        ops = _ext.ops()
        shp = h.shape
        h2 = h.reshape(-1, shp[-1]).contiguous()
        tg = target.reshape(-1).long().contiguous()
        M, V = h2.shape[0], weight.shape[0]
        need_h, need_w = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        want = need_h or need_w
        n = (tg != ignore_index).sum().clamp_min(1).float()
        inv_n = (1.0 / n).reshape(1)
        gh = torch.empty_like(h2) if need_h else None
        gw = torch.zeros(weight.shape, dtype=torch.float32, device=h2.device) if need_w else None
        buf = torch.empty(min(chunk, M), V, dtype=h2.dtype, device=h2.device)
        loss = torch.zeros((), dtype=torch.float32, device=h2.device)
        for r0 in range(0, M, chunk):
            r1 = min(M, r0 + chunk)
            hc, lg = h2[r0:r1], buf[: r1 - r0]
            ops.gemm(hc, weight, False, True, None, None, 0, None, lg, False, 0, False, None, -1)
            rows, _ = ops.xent_fwd(lg, tg[r0:r1], n_valid_cols, ignore_index, want)
            loss += rows.sum()
            if need_h:
                ops.gemm(lg, weight, False, False, None, None, 0, None, gh[r0:r1], False, -1, False, inv_n, -1)
            if need_w:
                ops.gemm(lg, hc, True, False, None, None, 0, None, gw, True, -1, False, inv_n, -1)
        del buf
        ctx.save_for_backward(weight, gh, gw)
        ctx.shp = shp
        return loss / n

    @staticmethod
    def backward(ctx, g):
        from .linear import _direct_grad, _notify
        weight, gh, gw = ctx.saved_tensors
        g = g.float()
        out_h = out_w = None
        if ctx.needs_input_grad[0]:
            out_h = (gh * g).reshape(ctx.shp)  # bf16 result, fp32 arithmetic
        if ctx.needs_input_grad[1]:
            gw = gw * g
            acc = _direct_grad(weight)
            if acc is not None:
                acc.add_(gw)
                _notify(weight)
            else:
                out_w = gw.to(weight.dtype)
        return out_h, out_w, None, None, None, None


XQ8_SCALE = 32768.0  # e5m2 loss-gradient scale of the fp8 LM head (csrc/kernels/softmax_xent.hip XQ8_SCALE)


class _LinearXentFp8Fn(torch.autograd.Function):
    """The LM head + cross-entropy in fp8 (training steps of the fp8 models, ``GPT2Config.fp8_head``):

    * logits = e4m3(h) · e4m3(W)ᵀ on the one-wave-per-SIMD fp8 GEMM (h's e4m3 copy from the final LayerNorm
      kernel, W = the tied embedding quantised with delayed scaling), bf16 logits;
    * the CE kernel writes the UNSCALED gradient (softmax − onehot) as e5m2 · 2^15 (``xent_fwd_q8``): a fixed
      power-of-two scale, |softmax − onehot| <= 1, so no amax pass.  The bf16 logits die with the forward;
      the 1-byte gradient is what the backward keeps;
    * backward: dh = dlogits8 · W8 (fp8 data-gradient GEMM, W read as stored) and dW += dlogits8ᵀ · h8 (fp8
      split-K weight gradient into the flat fp32 gradient), with g / n as one more device scalar (the
      GEMM's alpha / the split-K reduction's multiplier).

    Same operand shapes as :class:`_LinearXentFn`; GPT-2-medium b64: 3 × 6.75 TFLOP of bf16 GEMM → fp8.
    ``fp8_logits`` False: the logits GEMM stays bf16 (the loss value carries no e4m3 noise), the two gradient
    GEMMs are fp8 as above."""

    @staticmethod
    def forward(ctx, h, weight, target, n_valid_cols, ignore_index, state, fp8_logits=True):
        ops = _ext.ops()
        shp = h.shape
        h2 = h.reshape(-1, shp[-1]).contiguous()
        xq, xs = state.quant(h2, 0)
        wq, ws = state.quant(weight.contiguous(), 1)
        if fp8_logits:
            logits = ops.gemm_fp8(xq, wq, xs, ws, None, None, 0, None)
        else:
            logits = ops.gemm(h2, weight, False, True, None, None, 0, None, None, False, 0, False, None, -1)
        tg = target.reshape(-1).long().contiguous()
        q8 = torch.empty(logits.shape, dtype=torch.uint8, device=logits.device)
        loss_rows, _ = ops.xent_fwd_q8(logits, tg, n_valid_cols, ignore_index, q8)
        del logits
        n = (tg != ignore_index).sum().clamp_min(1).float()
        gs = torch.full((4,), 1.0 / XQ8_SCALE, dtype=torch.float32, device=h2.device)
        ctx.save_for_backward(weight, xq, xs.clone(), wq, ws.clone(), q8, n, gs)
        ctx.shp = shp
        return loss_rows.sum() / n

    @staticmethod
    def backward(ctx, g):
        from .linear import _direct_grad, _notify
        weight, xq, xs, wq, ws, q8, n, gs = ctx.saved_tensors
        alpha = (g.float() / n).reshape(1)
        ops = _ext.ops()
        gh = gw = None
        if ctx.needs_input_grad[0]:
            gh = ops.gemm_fp8_dgrad(q8, wq, gs, ws, True, alpha).reshape(ctx.shp)
        if ctx.needs_input_grad[1]:
            acc = _direct_grad(weight)
            if acc is not None:
                ops.gemm_fp8_wgrad(q8, xq, gs, xs, acc, True, True, alpha)
                _notify(weight)
            else:
                gw = torch.empty(weight.shape, dtype=torch.float32, device=q8.device)
                ops.gemm_fp8_wgrad(q8, xq, gs, xs, gw, False, True, alpha)
                gw = gw.to(weight.dtype)
        return gh, gw, None, None, None, None, None


def fp8_head_ok(h, weight) -> bool:
    """Shapes the fp8 LM head takes: vocab rows % 128, >= 256 (the data gradient's K-tiles), width % 16,
    tokens % 128 (the weight gradient's K-tiles), vocab <= 65536 (the CE row kernel)."""
    rows = h.numel() // h.shape[-1]
    V, E = weight.shape
    return V % 128 == 0 and 256 <= V <= 65536 and E % 16 == 0 and rows % 128 == 0 and rows > 0


def linear_cross_entropy(h, weight, target, *, n_valid_cols=None, ignore_index=-100, chunk_rows=0, fp8=None,
                         fp8_logits=True):
    """mean CE(h·weightᵀ, target) without materialising a separate logits gradient.

    ``chunk_rows`` > 0 (GPU): the LM head and the loss run over row chunks of that size, so
    the logits never exist for more than ``chunk_rows`` rows at once (``_ChunkedLinearXentFn``).
    ``fp8``: an :class:`~replicann_amd.ops.fp8.Fp8State` — the head in fp8 (``_LinearXentFp8Fn``; GPU, whole
    batch, shapes per :func:`fp8_head_ok`; ``fp8_logits`` False: bf16 logits, fp8 gradients)."""
    nv = weight.shape[0] if n_valid_cols is None else n_valid_cols
    if _ext.use_native(h):
        rows = h.numel() // h.shape[-1]
        if fp8 is not None and not (chunk_rows and chunk_rows < rows) and fp8_head_ok(h, weight):
            fp8.enter()
            return _LinearXentFp8Fn.apply(h, weight, target, nv, ignore_index, fp8, bool(fp8_logits))
        if chunk_rows and chunk_rows < rows:
            return _ChunkedLinearXentFn.apply(h, weight, target, nv, ignore_index, int(chunk_rows))
        return _LinearXentFn.apply(h, weight, target, nv, ignore_index)
    logits = F.linear(h, weight)
    return F.cross_entropy(logits.reshape(-1, logits.shape[-1])[:, :nv].float(), target.reshape(-1),
                           ignore_index=ignore_index)
