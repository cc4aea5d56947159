"""Linear layers on the gfx950 MFMA GEMM (csrc/kernels/gemm_bf16.hip).

Replaces the reference's per-head ``nn.Linear`` launches
(reference ``src/replicann/nn/attention.py:135-137``, ``arch/transformer.py:29-31``)
with one GEMM per projection whose epilogue fuses bias, activation
(ReLU / tanh-GELU), residual add and bf16 down-cast.

Backward = one dgrad GEMM (dX = dH·W, "NN") + one wgrad GEMM
(dW = dHᵀ·X, "TN", split-K over the token dimension) + a fused
activation-backward / bias-gradient reduction kernel.  All three GEMM layouts
run on the same kernel: K-contiguous operands are read from LDS with
``ds_read_b128``, M/N-contiguous ones with the ``ds_read_b64_tr_b16``
hardware transpose, so no operand is ever transposed in HBM.

CPU tensors take the plain ATen path (same math, fp32 accumulation).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .. import _ext

ACT_NONE, ACT_RELU, ACT_GELU = 0, 1, 2
# GEMM-epilogue-only codes: 5 = GELU whose pre-activation buffer receives gelu'(h) instead of h;
# 6 = its fused backward, out = (A·B) ⊙ pre (one multiply; see csrc/include/common.h)
ACT_GELU_D, ACT_MUL_BWD = 5, 6
_ACTS = {None: ACT_NONE, "none": ACT_NONE, "relu": ACT_RELU, "gelu": ACT_GELU}


def _act_ref(h: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return F.relu(h)
    if act in (ACT_GELU, ACT_GELU_D):
        return F.gelu(h, approximate="tanh")
    return h


def _pre_ref(h: torch.Tensor, act: int) -> torch.Tensor:
    """What the forward epilogue writes into the pre-activation buffer."""
    if act == ACT_GELU_D:
        return _act_grad_ref(torch.ones_like(h), h, ACT_GELU)
    return h


def _act_grad_ref(dy: torch.Tensor, h: torch.Tensor, act: int) -> torch.Tensor:
    if act == ACT_RELU:
        return dy * (h > 0).to(dy.dtype)
    if act == ACT_GELU:
        hf = h.float()
        c = math.sqrt(2.0 / math.pi)
        u = c * (hf + 0.044715 * hf**3)
        t = torch.tanh(u)
        d = 0.5 * (1 + t) + 0.5 * hf * (1 - t * t) * c * (1 + 3 * 0.044715 * hf * hf)
        return (dy.float() * d).to(dy.dtype)
    return dy


# --------------------------------------------------------------------------
# raw GEMM entry point (used by linear, conv2d, attention fallbacks)
# --------------------------------------------------------------------------
def gemm(a, b, *, ta=False, tb=False, bias=None, residual=None, act=ACT_NONE, preact=None,
         out=None, accumulate=False, split_k=0, out_dtype=None, alpha=None, cfg=-1):
    """C = act(alpha · op(A) @ op(B) + bias) + residual  (op = transpose if flag set).

    A, B are 2-D row-major bf16.  On CPU it is the ATen reference.
    ``accumulate`` adds into ``out`` (fp32 or bf16) instead of overwriting.
    ``alpha`` is an optional 1-element fp32 DEVICE tensor (read in the epilogue,
    graph-safe).  ``cfg`` forces a tile config (-1 = auto; 0..3 see gemm_bf16.hip).
    """
    if _ext.use_native(a):
        return _ext.ops().gemm(a, b, ta, tb, bias, residual, act, preact, out, accumulate, split_k,
                               out_dtype == torch.float32, alpha, cfg)
    A = a.t() if ta else a
    B = b.t() if tb else b
    h = A.float() @ B.float()
    if alpha is not None:
        h = h * alpha.float()
    if bias is not None:
        h = h + bias.float()
    if act == ACT_MUL_BWD:
        h = h * preact.float()
    elif preact is not None:
        preact.copy_(_pre_ref(h, act))
    y = _act_ref(h, act)
    if residual is not None:
        y = y + residual.float()
    dt = out_dtype or (out.dtype if out is not None else a.dtype)
    if out is not None:
        if accumulate:
            out.add_(y.to(out.dtype))
        else:
            out.copy_(y)
        return out
    return y.to(dt)


def bias_act_grad(dy2d, h2d, act, want_bias):
    """dH = dY ⊙ act'(H) and db = Σ_rows dH in one pass (fused kernel on GPU)."""
    if _ext.use_native(dy2d):
        dh, db = _ext.ops().bias_act_grad(dy2d, h2d if act != ACT_NONE else None, act, want_bias)
        return dh, (db if want_bias else None)
    dh = _act_grad_ref(dy2d, h2d, act) if act != ACT_NONE else dy2d
    db = dh.float().sum(0) if want_bias else None
    return dh, db


def _direct_grad(p):
    """The flat-buffer ``.grad`` view of parameter ``p`` if its gradient may be
    accumulated directly by a backward kernel (GEMM epilogue / reduction with
    ``accumulate``), bypassing autograd's AccumulateGrad add.  Parameters used
    once per forward qualify; a shared (tied) parameter qualifies when it
    declares how many direct contributions a backward makes (``_rn_direct_uses``,
    e.g. 2 for GPT-2's token embedding + LM head)."""
    f = getattr(p, "_rn_flat", None)
    if f is None or not f.direct or p.grad is None:
        return None
    if getattr(p, "_rn_shared", False) and getattr(p, "_rn_direct_uses", 0) < 2:
        return None
    return p.grad


def _notify(p):
    """Tell the flat buffer (and thus DDP's bucketing) that ``p``'s gradient is
    final — for a multi-use parameter, after its last contribution.  A fused-view parameter
    (nn/attention.py ``_fused_param``) stands for its members: each of them is final."""
    members = getattr(p, "_rn_members", None)
    if members is not None:
        for m in members:
            p._rn_flat.mark_ready(m)
        return
    uses = getattr(p, "_rn_direct_uses", 1)
    if uses > 1:
        left = getattr(p, "_rn_pending", uses) - 1
        p._rn_flat.contributed(p, left == 0)  # DDP reduces each contribution of a tied parameter
        if left > 0:
            p._rn_pending = left
            return
        p._rn_pending = uses
    p._rn_flat.mark_ready(p)


def _pick_split_k(m_out: int, n_out: int, k: int) -> int:
    tiles = math.ceil(m_out / 128) * math.ceil(n_out / 128)
    if tiles >= 512 or k < 1024:
        return 1
    s = 1
    while tiles * s < 512 and k // (s * 2) >= 512:
        s *= 2
    return s


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, act, residual, fp8=None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        res2 = residual.reshape(-1, weight.shape[0]) if residual is not None else None
        native = _ext.use_native(x2)
        preact = None
        if act != ACT_NONE:
            preact = torch.empty(x2.shape[0], weight.shape[0], device=x.device, dtype=x.dtype)
        ctx.x8 = None
        if fp8 is not None:
            from .fp8 import fp8_forward
            fp8.bwd_plan = (False, False)  # re-decided by every forward (a stale plan would skip a bf16 dY)
            if res2 is not None and not res2.is_contiguous():
                res2 = res2.contiguous()
            if fp8.fp8_bwd and (ctx.needs_input_grad[0] or ctx.needs_input_grad[1]):
                # keep the e4m3 operands for the fp8 weight / data gradients
                y, ctx.x8 = fp8_forward(x2, weight, bias, res2, act, preact, fp8, keep=True)
                from .fp8 import fp8_dgrad_ok, fp8_wgrad_ok
                dy_meta = torch.empty((x2.shape[0], weight.shape[0]), device="meta")
                # which gradients the backward will take in fp8 (then nothing reads dY in bf16 there)
                fp8.bwd_plan = (not ctx.needs_input_grad[1] or (ctx.x8[0] is not None and fp8_wgrad_ok(dy_meta, ctx.x8[0])),
                                not ctx.needs_input_grad[0] or (ctx.x8[2] is not None and fp8_dgrad_ok(dy_meta, weight.shape[1])))
            else:
                y = fp8_forward(x2, weight, bias, res2, act, preact, fp8)
        elif native:
            y = _ext.ops().gemm(x2, weight, False, True, bias, res2, act, preact, None, False, 0, False, None, -1)
        else:
            y = gemm(x2, weight, tb=True, bias=bias, residual=res2, act=act, preact=preact,
                     out_dtype=x.dtype)
        ctx.save_for_backward(x2, weight, preact)
        ctx.bias_ref = bias
        ctx.act = act
        ctx.has_bias = bias is not None
        ctx.has_res = residual is not None
        ctx.shp = shp
        return y.reshape(*shp[:-1], weight.shape[0])

    @staticmethod
    def backward(ctx, gy):
        x2, weight, preact = ctx.saved_tensors
        bias = ctx.bias_ref
        gy2 = gy.reshape(-1, weight.shape[0])
        if not gy2.is_contiguous():
            gy2 = gy2.contiguous()
        native = _ext.use_native(gy2)
        gx = gw = gb = None
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if want_b and getattr(bias, "_rn_bias_done", False):
            # the downstream LayerNorm backward already accumulated Σ_rows gy into bias.grad
            bias._rn_bias_done = False
            want_b = False
        db_acc = _direct_grad(bias) if (native and want_b) else None
        if native:
            dh, db = _ext.ops().bias_act_grad(gy2, preact if ctx.act != ACT_NONE else None, ctx.act, want_b, db_acc)
        else:
            dh, db = bias_act_grad(gy2, preact, ctx.act, want_b)
        sv, dyq = _fp8_bwd_operands(ctx, dh, weight)
        if ctx.needs_input_grad[0]:
            if dyq is not None and sv[2] is not None:  # fp8 data gradient: e5m2 dY · the e4m3 weight
                from .fp8 import fp8_dgrad
                gx = fp8_dgrad(dyq, sv[2], sv[3]).to(x2.dtype).reshape(ctx.shp)
            else:
                gx = gemm(dh, weight, out_dtype=x2.dtype).reshape(ctx.shp)
        if ctx.needs_input_grad[1]:
            w_acc = _direct_grad(weight) if native else None
            if sv is not None and sv[0] is not None and _fp8_wgrad_ok(dh, sv[0]):
                # fp8 weight gradient: e5m2 dY · the forward's e4m3 input
                from .fp8 import fp8_wgrad
                x8, xs, st = sv[0], sv[1], sv[4]
                if w_acc is not None:
                    fp8_wgrad(dh, x8, xs, st, out=w_acc, accumulate=True, dyq=dyq)
                    _notify(weight)
                else:
                    gw = fp8_wgrad(dh, x8, xs, st, dyq=dyq).to(weight.dtype)
            elif w_acc is not None:  # accumulate straight into the flat gradient buffer
                gemm(dh, x2, ta=True, split_k=-1, out=w_acc, accumulate=True)
                _notify(weight)
            else:
                gw = gemm(dh, x2, ta=True, split_k=-1, out_dtype=weight.dtype)  # split-K chosen natively
        ctx.x8 = None
        if want_b:
            if db_acc is not None:
                _notify(bias)
            else:
                gb = db.to(weight.dtype)
        gres = gy if ctx.has_res else None
        return gx, gw, gb, None, gres, None


def linear(x, weight, bias=None, act=None, residual=None, fp8=None):
    """y = act(x @ weightᵀ + bias) [+ residual].  ``act`` ∈ {None,'relu','gelu'}.
    ``fp8``: an :class:`~replicann_amd.ops.fp8.Fp8State` → the forward GEMM runs in e4m3."""
    a = _ACTS[act] if not isinstance(act, int) else act
    if fp8 is None and not x.is_cuda and not torch.is_grad_enabled() and residual is None and a == ACT_NONE:
        return F.linear(x, weight, bias)
    if fp8 is not None:
        fp8.enter()
    return _LinearFn.apply(x, weight, bias, a, residual, fp8)


def linear_kv_append(x, weight, bias, kv, pos):
    """Decode-step QKV projection: y = x·weightᵀ + bias for one new token per batch row (x (B, 1, K)),
    and y's last 2·H·D columns (keys, values) written into the KV cache buffer ``kv`` (B, L, 2, H, D)
    at the device-side row ``pos`` (1 int64).  Inference only.  On the GPU one launch: the append
    is part of the skinny GEMM's epilogue (``torch.ops.replicann.linear_kv``)."""
    B = x.shape[0]
    if (_ext.use_native(x) and x.dim() == 3 and x.shape[1] == 1 and B <= 64 and not torch.is_grad_enabled()
            and kv.is_contiguous()):
        return _ext.ops().linear_kv(x.reshape(B, -1).contiguous(), weight, bias, kv, pos).view(B, 1, -1)
    y = linear(x, weight, bias)
    w = kv[0, 0].numel()
    kv.index_copy_(1, pos, y[..., -w:].reshape(B, y.shape[1], *kv.shape[2:]))
    return y


# --------------------------------------------------------------------------
# fused two-layer MLP: y = act(x·W1ᵀ + b1)·W2ᵀ + b2 (+ residual)
# --------------------------------------------------------------------------
ACT_BWD = {ACT_RELU: 3, ACT_GELU: 4}  # GEMM epilogue codes: out = (A·B) ⊙ act'(pre)
# The MLP's GELU saves gelu'(h) (forward epilogue code 5) and its dgrad multiplies by it (code 6)
_MLP_FWD_ACT = {ACT_RELU: ACT_RELU, ACT_GELU: ACT_GELU_D}
_MLP_BWD_ACT = {ACT_RELU: 3, ACT_GELU: ACT_MUL_BWD}


def _bias_grad(g2, bias, native):
    """Σ_rows g2 into ``bias``'s gradient: (returned grad or None, done_direct)."""
    if bias is None or not bias.requires_grad:
        return None
    if getattr(bias, "_rn_bias_done", False):  # reduced by the downstream LayerNorm backward
        bias._rn_bias_done = False
        return None
    acc = _direct_grad(bias) if native else None
    if native:
        _, db = _ext.ops().bias_act_grad(g2, None, ACT_NONE, True, acc)
    else:
        db = g2.float().sum(0)
    if acc is not None:
        _notify(bias)
        return None
    return db.to(bias.dtype)


def _fp8_wgrad_ok(dy2, x8):
    from .fp8 import fp8_wgrad_ok
    return fp8_wgrad_ok(dy2, x8)


def _fp8_bwd_operands(ctx, dy2, weight):
    """(saved, dyq): the fp8 forward's kept operands (x8, xs, w8, ws, state) and dY quantised ONCE
    to e5m2 for whichever of the fp8 data / weight gradients applies (None when neither does)."""
    sv = ctx.x8
    ctx.x8 = None
    if sv is None:
        return None, None
    from .fp8 import fp8_dgrad_ok
    use_d = sv[2] is not None and ctx.needs_input_grad[0] and fp8_dgrad_ok(dy2, weight.shape[1])
    use_w = sv[0] is not None and ctx.needs_input_grad[1] and _fp8_wgrad_ok(dy2, sv[0])
    if not (use_d or use_w):
        return sv, None
    return sv, sv[4].gquant(dy2)


def _wgrad(g2, x2, weight, native, x8=None, dyq=None):
    """Weight gradient g2ᵀ·x2 into the flat gradient view (or returned).  ``x8``: (e4m3 x2, its scale,
    Fp8State) kept by an fp8 forward → the fp8 weight-gradient GEMM (e5m2 g2, or ``dyq`` if the data
    gradient already quantised it)."""
    if x8 is not None and x8[0] is not None and _fp8_wgrad_ok(g2, x8[0]):
        from .fp8 import fp8_wgrad
        acc = _direct_grad(weight) if native else None
        if acc is not None:
            fp8_wgrad(g2, x8[0], x8[1], x8[2], out=acc, accumulate=True, dyq=dyq)
            _notify(weight)
            return None
        return fp8_wgrad(g2, x8[0], x8[1], x8[2], dyq=dyq).to(weight.dtype)
    acc = _direct_grad(weight) if native else None
    if acc is not None:
        gemm(g2, x2, ta=True, split_k=-1, out=acc, accumulate=True)
        _notify(weight)
        return None
    return gemm(g2, x2, ta=True, split_k=-1, out_dtype=weight.dtype)


class _MLPFn(torch.autograd.Function):
    """One autograd node for the whole MLP so the activation backward runs in the
    epilogue of the second layer's dgrad GEMM:  dH = (dY·W2) ⊙ act'(pre)  — the
    separate activation-backward pass over dU (read dU + pre, write dH) is gone."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, act, residual, fp8=None):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        res2 = residual.reshape(-1, w2.shape[0]).contiguous() if residual is not None else None
        ops = _ext.ops()
        pre = torch.empty(x2.shape[0], w1.shape[0], device=x.device, dtype=x.dtype)
        ctx.x8 = (None, None)
        ctx.pre_is_h = False
        if fp8 is not None:  # re-decided by every forward (a stale plan would skip a bf16 dY)
            for st in fp8:
                if st is not None:
                    st.bwd_plan = (False, False)
        if fp8 is not None and _MLPFn._fp8_keep_h(ctx, x2, w1, w2, act, fp8):
            # the all-fp8 MLP (both layers' fp8 gradients, fused backward): c_fc on the one-wave-per-SIMD
            # fp8 GEMM writes h = x·W1ᵀ + b1 only, ONE pass makes e4m3(gelu(h)) for the MLP c_proj
            # (ops gelu_q8, the consumer's delayed scale), and the backward re-derives gelu'(h) inside its
            # fused e5m2 pass: gelu(h) / gelu'(h) are never written in bf16
            from .fp8 import fp8_forward
            h, sv1 = fp8_forward(x2, w1, b1, None, ACT_NONE, None, fp8[0], keep=True)
            slot = fp8[1].roll_slot(0)
            fp8[1].offer(h, ops.gelu_q8(h, slot), slot)
            fp8[1].bwd_plan = (True, True)  # the fused backward takes dY in e5m2 (a producer may offer it)
            y, sv2 = fp8_forward(h, w2, b2, res2, ACT_NONE, None, fp8[1], keep=True)
            ctx.x8 = (sv1, sv2)
            ctx.pre_is_h = True
            ctx.save_for_backward(x2, w1, h, h, w2)  # (pre = h; "u" only lends its shape to the backward)
            ctx.b1, ctx.b2, ctx.act, ctx.shp, ctx.has_res = b1, b2, act, shp, residual is not None
            return y.reshape(*shp[:-1], w2.shape[0])
        if fp8 is not None:  # (state of layer 1, state of layer 2 or None): e4m3 forward GEMMs
            from .fp8 import fp8_forward
            # layer 2's e4m3 input comes out of layer 1's epilogue (its delayed scale permitting)
            # the e4m3 operands are kept for the fp8 weight gradients and layer 1's fp8 data gradient
            # (layer 2's data gradient carries the fused activation backward: bf16)
            if (ctx.needs_input_grad[1] and fp8[0].wgrad) or (ctx.needs_input_grad[0] and fp8[0].dgrad):
                u, sv = fp8_forward(x2, w1, b1, None, _MLP_FWD_ACT[act], pre, fp8[0], out8=fp8[1], keep=True)
                ctx.x8 = (sv, None)
            else:
                u = fp8_forward(x2, w1, b1, None, _MLP_FWD_ACT[act], pre, fp8[0], out8=fp8[1])
            if fp8[1] is not None and ((ctx.needs_input_grad[3] and fp8[1].wgrad) or fp8[1].dgrad):
                # (the e4m3 weight also for layer 2's fp8 data gradient: see _MLPFn._fp8_backward)
                y, sv2 = fp8_forward(u, w2, b2, res2, ACT_NONE, None, fp8[1], keep=True)
                ctx.x8 = (ctx.x8[0], sv2)
            elif fp8[1] is not None:
                y = fp8_forward(u, w2, b2, res2, ACT_NONE, None, fp8[1])
            else:
                y = ops.gemm(u, w2, False, True, b2, res2, ACT_NONE, None, None, False, 0, False, None, -1)
        else:
            u = ops.gemm(x2, w1, False, True, b1, None, _MLP_FWD_ACT[act], pre, None, False, 0, False, None, -1)
            y = ops.gemm(u, w2, False, True, b2, res2, ACT_NONE, None, None, False, 0, False, None, -1)
        ctx.save_for_backward(x2, w1, pre, u, w2)
        ctx.b1, ctx.b2, ctx.act, ctx.shp, ctx.has_res = b1, b2, act, shp, residual is not None
        return y.reshape(*shp[:-1], w2.shape[0])

    @staticmethod
    def _fp8_keep_h(ctx, x2, w1, w2, act, fp8):
        """The forward may keep h instead of gelu(h) / gelu'(h) only when the backward is certain to take
        the fused fp8 path (which reads neither): GELU, both layers fp8 with fp8 data AND weight gradients,
        training, and the consumer's delayed scale already seeded."""
        from .fp8 import FP8_MLP_FUSE, fp8_dgrad_ok, fp8_wgrad_ok
        f1, f2 = fp8
        nig = ctx.needs_input_grad
        if not (FP8_MLP_FUSE and f2 is not None and _MLP_FWD_ACT.get(act) == ACT_GELU_D and nig[0] and nig[1] and nig[3]):
            return False
        if not (f1.wgrad and f1.dgrad and f2.wgrad and f2.dgrad and f2.producer_ready(x2.device) and not f2.inference()):
            return False
        M, N = x2.shape[0], w1.shape[0]
        probe = x2.new_empty((M, N))  # (shape only)
        dy_probe = x2.new_empty((M, w2.shape[0]))
        # both weight gradients must take the fp8 GEMM too (tokens % 128): the bf16 fallback of _wgrad would
        # read h where it needs gelu(h) (c_proj) and dU where it needs dH (c_fc) — ADVICE r5 (high)
        return (N % 8 == 0 and fp8_dgrad_ok(probe, w1.shape[1]) and fp8_dgrad_ok(dy_probe, N)
                and x2.shape[1] % 16 == 0 and N % 16 == 0
                and fp8_wgrad_ok(probe, x2) and fp8_wgrad_ok(dy_probe, probe))

    @staticmethod
    def _fp8_backward(ctx, gy, gy2, x2, w1, pre, u, w2, sv1, sv2):
        """Both layers' gradients in fp8 with the GELU backward fused into the e5m2 quantisation of
        dH: dY → e5m2 once (layer 2's dgrad + wgrad), dU = dY·W2 on the fp8 dgrad GEMM, then ONE pass
        dH8 = e5m2(dU ⊙ gelu'(h)) that also reduces layer 1's bias gradient (csrc/kernels/fp8.hip
        act_mul_bf8_k), and layer 1's fp8 dgrad / wgrad from dH8.  Replaces the bf16 dgrad GEMM with
        the multiply in its epilogue + the separate e5m2 pass over dH (profiles/gpt2m_fp8_r5g.txt).
        Returns the gradient tuple, or None when an operand of that plan is missing."""
        from .fp8 import FP8_MLP_FUSE, fp8_dgrad, fp8_dgrad_ok
        nig = ctx.needs_input_grad
        if ctx.pre_is_h:  # the forward kept h: this path is the only one that can take it (_fp8_keep_h)
            assert sv1 is not None and sv2 is not None and sv1[0] is not None and sv2[0] is not None
            # ... and both weight gradients must run on the fp8 GEMM (the bf16 fallback would read h / dU)
            assert _fp8_wgrad_ok(gy2, sv2[0]) and _fp8_wgrad_ok(u, sv1[0]), "keep-h MLP without fp8 weight gradients"
        elif not (FP8_MLP_FUSE and nig[0] and nig[1] and _MLP_BWD_ACT[ctx.act] == ACT_MUL_BWD and sv1 is not None and sv2 is not None
                and sv1[0] is not None and sv1[2] is not None and sv2[2] is not None
                and fp8_dgrad_ok(gy2, w2.shape[1]) and fp8_dgrad_ok(u, w1.shape[1]) and _fp8_wgrad_ok(u, sv1[0])
                and pre.shape[1] % 8 == 0):
            return None
        dyq2 = sv2[4].gquant(gy2)
        x8_2 = (sv2[0], sv2[1], sv2[4]) if sv2[0] is not None else None
        gw2 = _wgrad(gy2, u, w2, True, x8_2, dyq2 if x8_2 is not None else None) if nig[3] else None
        gb2 = _bias_grad(gy2, ctx.b2, True) if nig[4] else None
        du = fp8_dgrad(dyq2, sv2[2], sv2[3])
        b1 = ctx.b1
        b1_acc, gb1 = None, None
        if nig[2] and b1 is not None:
            if not getattr(b1, "_rn_bias_done", False):
                b1_acc = _direct_grad(b1)
            if b1_acc is None:
                gb1 = torch.zeros(b1.shape, device=b1.device, dtype=torch.bfloat16)
        dyq = sv1[4].gquant_mul(du, pre, b1_acc if b1_acc is not None else gb1, from_h=ctx.pre_is_h)
        if b1_acc is not None:
            _notify(b1)
        elif gb1 is not None:
            gb1 = gb1.to(b1.dtype)
        x8_1 = (sv1[0], sv1[1], sv1[4])
        gw1 = _wgrad(du, x2, w1, True, x8_1, dyq)  # (du: the dH shape for the fp8 path's checks)
        gx = fp8_dgrad(dyq, sv1[2], sv1[3])
        return gx.reshape(ctx.shp), gw1, gb1, gw2, gb2, None, gy if ctx.has_res else None, None

    @staticmethod
    def backward(ctx, gy):
        x2, w1, pre, u, w2 = ctx.saved_tensors
        ops = _ext.ops()
        gy2 = gy.reshape(-1, w2.shape[0]).contiguous()
        nig = ctx.needs_input_grad
        sv1, sv2 = ctx.x8
        ctx.x8 = (None, None)
        out = _MLPFn._fp8_backward(ctx, gy, gy2, x2, w1, pre, u, w2, sv1, sv2)
        if out is not None:
            return out
        x8_2 = (sv2[0], sv2[1], sv2[4]) if sv2 is not None else None
        gw2 = _wgrad(gy2, u, w2, True, x8_2) if nig[3] else None
        gb2 = _bias_grad(gy2, ctx.b2, True) if nig[4] else None
        b1 = ctx.b1
        b1_acc = None
        if nig[2] and b1 is not None and not getattr(b1, "_rn_bias_done", False):
            b1_acc = _direct_grad(b1)
        # dH = (dY·W2) ⊙ act'(pre); with a flat-buffer b1 its gradient Σ_rows dH comes from the
        # same GEMM's epilogue (per-tile column partials + one small reduction)
        dh = ops.gemm(gy2, w2, False, False, None, None, _MLP_BWD_ACT[ctx.act], pre, None, False, 0, False, None, -1,
                      b1_acc)
        if b1_acc is not None:
            _notify(b1)
            gb1 = None
        else:
            gb1 = _bias_grad(dh, b1, True) if nig[2] else None
        dyq = None
        if sv1 is not None:
            from .fp8 import fp8_dgrad, fp8_dgrad_ok
            use_d = sv1[2] is not None and nig[0] and fp8_dgrad_ok(dh, w1.shape[1])
            use_w = sv1[0] is not None and nig[1] and _fp8_wgrad_ok(dh, sv1[0])
            if use_d or use_w:  # dH in e5m2 once, for both
                dyq = sv1[4].gquant(dh)
        x8_1 = (sv1[0], sv1[1], sv1[4]) if sv1 is not None else None
        gw1 = _wgrad(dh, x2, w1, True, x8_1, dyq) if nig[1] else None
        if dyq is not None and sv1[2] is not None and nig[0]:
            gx = fp8_dgrad(dyq, sv1[2], sv1[3])
        else:
            gx = ops.gemm(dh, w1, False, False, None, None, ACT_NONE, None, None, False, 0, False, None, -1)
        return (gx.reshape(ctx.shp) if nig[0] else None, gw1, gb1, gw2, gb2, None,
                gy if ctx.has_res else None, None)


def mlp(x, w1, b1, w2, b2, act="gelu", residual=None, fp8=None):
    """act(x·W1ᵀ + b1)·W2ᵀ + b2 [+ residual] — fused backward on GPU, plain linears on CPU.
    ``fp8``: (Fp8State, Fp8State) of the two layers → e4m3 forward GEMMs."""
    a = _ACTS[act] if not isinstance(act, int) else act
    if _ext.use_native(x) and a in ACT_BWD:
        if fp8 is not None:
            for st in fp8:
                if st is not None:
                    st.enter()
        return _MLPFn.apply(x, w1, b1, w2, b2, a, residual, fp8)
    f1, f2 = fp8 if fp8 is not None else (None, None)
    return linear(linear(x, w1, b1, act=a, fp8=f1), w2, b2, residual=residual, fp8=f2)
