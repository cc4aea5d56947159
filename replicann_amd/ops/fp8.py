"""FP8 (OCP e4m3fn) linear layers on the CDNA4 block-scaled MFMA (csrc/kernels/fp8.hip) — N3.

``linear_fp8`` (and ``linear`` / ``mlp`` with an ``fp8=`` state) runs the FORWARD
GEMM in fp8: activations and weights are quantised per tensor (delayed scaling,
see :class:`Fp8State`), multiplied by ``v_mfma_scale_f32_16x16x128_f8f6f4`` at
twice the bf16 MFMA rate, and the two tensor scales are folded into the epilogue
alpha together with bias / GELU / residual.  The backward is the bf16 one (bf16
master weight, bf16 gradients, fused activation-backward / bias reductions), the
recipe used for "fp8 weights" training in BASELINE.json's GPT-2-medium config.

CPU tensors emulate the numerics (quantise → dequantise → fp32 matmul).
"""

from __future__ import annotations

import os

import torch

from .. import _ext
from .linear import _act_ref, _pre_ref

E4M3_MAX = 448.0
E5M2_MAX = 57344.0
# fp8 backward of the fp8 layers (the Transformer-Engine hybrid recipe: dY quantised once to e5m2 with its
# own delayed scale): weight gradients dW = dYᵀ·X against the forward's e4m3 input copy
# (REPLICANN_FP8_WGRAD, Fp8State.wgrad) and data gradients dX = dY·W against the forward's e4m3 weight,
# for the layers whose dgrad has a plain epilogue (REPLICANN_FP8_DGRAD, Fp8State.dgrad).  On by default
# since round 5: on the one-wave-per-SIMD kernels (csrc/include/gemm_w1.h) the fp8 dgrad runs 1.5-2.0
# PF/s and the fp8 wgrad 1.5-1.7x the bf16 one per shape, GPT-2-medium 146.8 ms/step with both against
# 157.0 (dgrad only) / 158.5 (forward only) / 165 (bf16) (profiles/w1_fp8_bwd_r5f.txt,
# profiles/gpt2m_fp8_r5g.txt); 50-step loss trajectory vs bf16: max rel dev 3.2 % in the steep descent
# (steps 9-19), 0.8 % at step 50.  =0 turns either off.
FP8_WGRAD = os.environ.get("REPLICANN_FP8_WGRAD", "1") == "1"
FP8_DGRAD = os.environ.get("REPLICANN_FP8_DGRAD", "1") == "1"
# fp8 MLP backward with both layers' fp8 gradients: the MLP c_proj data gradient on the fp8 GEMM and the
# GELU backward fused into the e5m2 quantisation of dH (ops.linear._MLPFn._fp8_backward).  The unfused
# path (bf16 c_proj dgrad with the multiply in its epilogue + a separate e5m2 pass) still serves the
# shapes the fused one does not take; tests flip this module attribute to compare the two (no env knob:
# the fused path won in round 5, profiles/gpt2m_fp8_r5g.txt).
FP8_MLP_FUSE = True


def pow2_ceil(s):
    """The smallest power of two >= s (float32, exact; 1 for s <= 0): every fp8 scale is one, so the
    one-wave-per-SIMD GEMM can feed the tensors' exponents to the scaled MFMA (csrc/kernels/fp8.hip,
    pow2_ceil)."""
    s = torch.as_tensor(s, dtype=torch.float32)
    if not bool(s > 0):
        return torch.tensor(1.0)
    m, e = torch.frexp(s)  # s = m · 2^e, m in [0.5, 1)
    e = torch.where(m == 0.5, e - 1, e)
    return torch.ldexp(torch.tensor(1.0), e).float()


def _pow2_ceil_pos(s):
    """Element-wise pow2_ceil of the positive entries of a scale tensor (others unchanged)."""
    m, e = torch.frexp(s)
    e = torch.where(m == 0.5, e - 1, e)
    return torch.where(s > 0, torch.ldexp(torch.ones_like(s), e), s)


def quantize_fp8(x):
    """(q uint8 e4m3 storage, state[0] = scale) with x ≈ q·scale (scale a power of two)."""
    if _ext.use_native(x):
        return _ext.ops().fp8_quantize(x.contiguous())
    amax = x.detach().abs().max().float()
    scale = pow2_ceil(amax / E4M3_MAX) if amax > 0 else torch.tensor(1.0)
    q = (x.float() / scale).clamp(-E4M3_MAX, E4M3_MAX).to(torch.float8_e4m3fn)
    return q.view(torch.uint8), torch.stack([scale, amax, scale * 0, scale * 0]).float()


def quantize_bf8(x, state, delayed):
    """e5m2 copy of a gradient with its delayed-scaling slot ``state`` (4 floats: scale, amax,
    previous amax, -): current scaling if not ``delayed``.  Returns q (uint8 storage)."""
    if _ext.use_native(x):
        return _ext.ops().bf8_quantize(x.contiguous(), state, bool(delayed))
    amax = x.detach().abs().max().float()
    if delayed:
        prev = state[1].clone()
        state[2] = prev
        scale = pow2_ceil(2 * prev / E5M2_MAX) if float(prev) > 0 else torch.tensor(1.0)
    else:
        scale = pow2_ceil(amax / E5M2_MAX) if amax > 0 else torch.tensor(1.0)
    state[0] = scale
    state[1] = amax
    q = (x.float() / scale).clamp(-E5M2_MAX, E5M2_MAX).to(torch.float8_e5m2)
    return q.view(torch.uint8)


def dequantize_bf8(q, state):
    if _ext.use_native(q):
        return _ext.ops().bf8_dequantize(q, state)
    return (q.view(torch.float8_e5m2).float() * state[0]).to(torch.bfloat16)


def fp8_wgrad_ok(dy2, x8) -> bool:
    """Shapes the fp8 weight-gradient GEMM takes: tokens % 128, both widths % 16."""
    return dy2.shape[0] % 128 == 0 and dy2.shape[1] % 16 == 0 and x8.shape[1] % 16 == 0 and dy2.shape[0] > 0


def fp8_dgrad_ok(dy2, n_in) -> bool:
    """Shapes the fp8 data-gradient GEMM takes: both widths % 16."""
    return dy2.shape[0] > 0 and dy2.shape[1] % 16 == 0 and n_in % 16 == 0


def fp8_dgrad(dyq, w8, ws):
    """dX = dY·W in fp8: ``dyq`` = (e5m2 dY, its scale slot) from :meth:`Fp8State.gquant`, ``w8`` the
    forward's e4m3 weight [out][in] with scale ``ws`` (read transposed by the kernel: no transposed
    copy).  Returns bf16 [tokens][in].  CPU: quantise → dequantise numerics in fp32."""
    dy8, gs = dyq
    if _ext.use_native(dy8):
        return _ext.ops().gemm_fp8_dgrad(dy8, w8, gs, ws, True)
    return (dequantize_bf8(dy8, gs).float() @ dequantize_fp8(w8, ws).float()).to(torch.bfloat16)


def fp8_wgrad(dy2, x8, xs, state, out=None, accumulate=False, dyq=None):
    """dW = dYᵀ·X in fp8: dY quantised to e5m2 with ``state``'s gradient slot (or ``dyq`` = the
    (e5m2 dY, scale) pair already made for the data gradient), X = the forward's e4m3 copy ``x8``
    with scale slot ``xs``.  Accumulates into ``out`` (the flat gradient view) or returns a new bf16
    tensor.  CPU: the same quantise → dequantise numerics in fp32."""
    dy8, gs = dyq if dyq is not None else state.gquant(dy2)
    if _ext.use_native(dy2):
        if out is None:
            out = torch.zeros(dy2.shape[1], x8.shape[1], device=dy2.device, dtype=torch.bfloat16)
            accumulate = False
        _ext.ops().gemm_fp8_wgrad(dy8, x8, gs, xs, out, accumulate, True)
        return out
    g = dequantize_bf8(dy8, gs).float().t() @ dequantize_fp8(x8, xs).float()
    if out is None:
        return g.to(dy2.dtype)
    if accumulate:
        out.add_(g.to(out.dtype))
    else:
        out.copy_(g)
    return out


def dequantize_fp8(q, state):
    if _ext.use_native(q):
        return _ext.ops().fp8_dequantize(q, state)
    return (q.view(torch.float8_e4m3fn).float() * state[0]).to(torch.bfloat16)


class Fp8State:
    """Scaling state of one fp8 GEMM's two forward operands (activation, weight).

    The first quantisation of each operand uses current scaling (amax pass + quantise
    pass) and records the amax in a persistent device tensor; every later one is a
    single pass with delayed scaling: the scale comes from the previous quantisation's
    amax (x2 headroom, saturating beyond it) and the pass records the new amax
    (``fp8_quantize_delayed``) — the Transformer-Engine recipe with a history of one.
    Everything is on device, so a captured step graph replays it unchanged.

    Persistence: with an ``owner`` module the (2, 4) state tensor is that module's registered
    buffer (``fp8_scales``): it moves with ``.to()``, is saved / loaded with the state_dict (so a
    resumed run continues with the same delayed scales), and is part of ``model.buffers()``, which
    the trainer snapshots around its autotuning pass and graph-capture warm-ups.  The host-side
    ``ready`` flags (whether a slot holds a scale yet) follow the tensor: they are re-derived when a
    state_dict is loaded (:func:`sync_ready_from_tensors`) and snapshotted with it
    (:func:`ready_snapshot` / :func:`ready_restore`)."""

    def __init__(self, owner=None, name="fp8_scales", gname="fp8_gscales"):
        self._owner = owner
        self._name = name
        self._gname = gname
        self._t = None
        self._gt = None
        self.ready = [False, False]
        self.g_ready = False  # gradient slot (fp8 weight gradient's dY) holds a scale
        self.wgrad = FP8_WGRAD
        self.dgrad = FP8_DGRAD
        self.w_cached = False  # the last weight quant() came from the optimizer-refreshed cache
        self._offer = None  # (activation tensor, its e4m3 copy, scale slot) written by the producer kernel
        self.fed = 0  # activations taken from a producer kernel instead of a quantisation pass
        self.wcache = None  # Fp8WeightCache holding this GEMM's e4m3 weight (refreshed by the optimizer)
        self._ti = None  # inference scratch slots (see roll_slot)
        self._goffer = None  # (dY tensor, its e5m2 copy) written by the producing backward kernel (attention)
        # set by the fp8 linear's forward: (fp8 weight gradient, fp8 data gradient) its backward will take —
        # the producer of its dY may then skip the bf16 dY altogether
        self.bwd_plan = (False, False)
        self.grad_mode = True  # grad mode at the op's entry (autograd Functions run forward under no_grad)

    @property
    def t(self):
        return getattr(self._owner, self._name) if self._owner is not None else self._t

    @t.setter
    def t(self, value):
        if self._owner is not None:
            self._owner._buffers[self._name] = value
        else:
            self._t = value

    @property
    def gt(self):
        """(1, 4) gradient slot [scale, amax, previous amax, -] of the fp8 weight gradient's dY."""
        if self._owner is not None and self._gname in self._owner._buffers:
            return self._owner._buffers[self._gname]
        return self._gt

    @gt.setter
    def gt(self, value):
        if self._owner is not None and self._gname in self._owner._buffers:
            self._owner._buffers[self._gname] = value
        else:
            self._gt = value

    def sync_ready(self):
        """ready[i] = slot i holds a scale (host sync: call at load time, never inside a step).

        Loaded scales are also rounded up to powers of two: the one-wave-per-SIMD fp8 GEMM feeds only
        the exponent byte of a scale to the scaled MFMA, so a checkpoint written before every quantiser
        rounded its scale up (2·amax/448, any mantissa) would otherwise run its first resumed step with
        every tensor silently scaled by 2^floor(log2 s)/s.  Power-of-two scales
        (every checkpoint since) are unchanged, so bit-exact resume holds."""
        t = self.t
        if t is not None:
            t[:, 0] = _pow2_ceil_pos(t[:, 0])
        self.ready = [bool(t is not None and float(t[i, 0]) > 0) for i in range(2)]
        g = self.gt
        if g is not None:
            g[:, 0] = _pow2_ceil_pos(g[:, 0])
        self.g_ready = bool(g is not None and float(g[0, 0]) > 0)

    def gslot(self, device):
        """The gradient slot (allocating it on first use) — for a producer kernel that emits dY in e5m2."""
        if self.gt is None or self.gt.device != device:
            self.gt = torch.zeros(1, 4, device=device, dtype=torch.float32)
            self.g_ready = False
        return self.gt[0]

    def goffer(self, dy, q):
        """A producer wrote ``dy``'s e5m2 copy ``q`` with the gradient slot (rolled, amax recorded): the
        next gquant of the same tensor returns it."""
        self._goffer = (dy, q)

    def gquant(self, dy):
        """dY in e5m2 with the gradient slot: current scaling on the first call, delayed after."""
        if self._goffer is not None:
            src, q = self._goffer
            self._goffer = None
            if src.data_ptr() == dy.data_ptr() and src.numel() == dy.numel():
                self.g_ready = True
                return q.view(dy.shape), self.gt[0]
        if self.gt is None or self.gt.device != dy.device:
            self.gt = torch.zeros(1, 4, device=dy.device, dtype=torch.float32)
            self.g_ready = False
        st = self.gt[0]
        q = quantize_bf8(dy, st, self.g_ready)
        self.g_ready = True
        return q, st

    def gquant_mul(self, du, d, bias_grad=None, from_h=False):
        """dH = dU ⊙ d (the MLP's GELU backward against the saved gelu'(h)) straight to e5m2 with the
        gradient slot — dH itself is never written in bf16 — and Σ_rows dH added into ``bias_grad`` (bf16
        [N]) when given.  ``from_h``: ``d`` holds the pre-activation h, gelu'(h) is taken here.  Scaling
        as :meth:`gquant`."""
        if self.gt is None or self.gt.device != du.device:
            self.gt = torch.zeros(1, 4, device=du.device, dtype=torch.float32)
            self.g_ready = False
        st = self.gt[0]
        if _ext.use_native(du):
            q = _ext.ops().act_mul_bf8(du, d, st, self.g_ready, bias_grad, from_h)
        else:
            dd = d.float()
            if from_h:
                from .linear import ACT_GELU, _act_grad_ref
                dd = _act_grad_ref(torch.ones_like(dd), d, ACT_GELU)
            dh = du.float() * dd
            if bias_grad is not None:
                bias_grad.add_(dh.sum(0).to(bias_grad.dtype))
            q = quantize_bf8(dh, st, self.g_ready)
        self.g_ready = True
        return q, st

    def producer_ready(self, device) -> bool:
        """True once the activation slot has a delayed scale, so a producer kernel (LayerNorm)
        can emit the e4m3 activation itself (first call: current scaling in quant())."""
        return self.t is not None and self.t.device == device and self.ready[0] and _ext.use_native(self.t)

    def inference(self) -> bool:
        """Inference (no_grad, or the owning module in eval mode): quantisation must not touch the
        training slots — evaluate() / generate() between training steps would otherwise roll the
        delayed scales and record their own batches' amax, which the next training step quantises
        with."""
        return not self.grad_mode or (self._owner is not None and not self._owner.training)

    def enter(self):
        """Record the caller's grad mode; every op that hands this state to an autograd Function
        calls it before ``apply`` (inside ``forward`` grad mode is always off)."""
        self.grad_mode = torch.is_grad_enabled()
        return self

    def roll_slot(self, i):
        """The scale slot a kernel may ROLL and record an amax into for operand ``i``: the training
        slot, or under inference a scratch copy of it (same delayed scale, amax discarded), so the
        training state is read-only outside training steps."""
        st = self.t[i]
        if not self.inference():
            return st
        if self._ti is None or self._ti.device != st.device:
            self._ti = torch.zeros(2, 4, device=st.device, dtype=torch.float32)
        self._ti[i].copy_(st)
        return self._ti[i]

    def offer(self, x, q, slot=None):
        """A producer quantised ``x`` into ``q`` with scale slot ``slot`` (this state's activation
        slot, or its inference copy; rolled + amax recorded by that kernel); the next quant(x, 0) of
        the same tensor returns it."""
        self._offer = (x, q, self.t[0] if slot is None else slot)

    @property
    def fp8_bwd(self):
        return self.wgrad or self.dgrad

    def quant(self, x, i):
        if i == 1:
            self.w_cached = False
        if i == 1 and self.wcache is not None:
            q = self.wcache.lookup(self, x)
            if q is not None:
                self.w_cached = True
                return q, self.t[1]
        if i == 0 and self._offer is not None:
            src, q, slot = self._offer
            self._offer = None
            if src.data_ptr() == x.data_ptr() and src.shape == x.shape:
                self.fed += 1
                return q, slot
        if self.t is None or self.t.device != x.device:
            self.t = torch.zeros(2, 4, device=x.device, dtype=torch.float32)
            self.ready = [False, False]
        if not self.ready[i] or not _ext.use_native(x):
            q, s = quantize_fp8(x)
            if self.inference():  # current scaling into the scratch slot: the training slot stays unseeded
                st = self.roll_slot(i)
                st.copy_(s)
                return q, st
            st = self.t[i]
            st.copy_(s)
            self.ready[i] = True
            return q, st
        st = self.roll_slot(i)
        return _ext.ops().fp8_quantize_delayed(x, st), st


def fp8_states(model):
    """Every Fp8State of ``model`` (layers with ``fp8_state``), in module order."""
    return [m.fp8_state for m in model.modules() if getattr(m, "fp8_state", None) is not None]


def ready_snapshot(model):
    return [(list(st.ready), st.g_ready) for st in fp8_states(model)]


def ready_restore(model, snap):
    for st, (r, g) in zip(fp8_states(model), snap):
        st.ready = list(r)
        st.g_ready = g


def sync_ready_from_tensors(model):
    for st in fp8_states(model):
        st.sync_ready()


def fp8_forward(x2, weight, bias, res2, act, preact, state: Fp8State, out8: Fp8State | None = None,
                keep=False):
    """act(x2·weightᵀ + bias) + res2 with both operands in e4m3 (GPU: block-scaled MFMA;
    CPU: the same quantise → dequantise numerics in fp32).

    ``out8``: the state of the fp8 GEMM that consumes this output — the epilogue then also writes
    the output in e4m3 with that state's delayed scale and hands it over (no quantisation pass).
    ``keep``: return (y, saved) with saved = (x8, x scale, w8, w scale, state): the e4m3 operands
    the backward's fp8 weight gradient (x8, if ``state.wgrad``) and data gradient (w8, if
    ``state.dgrad``) read.  Scale slots a later quant() may roll are copied; the cached weight's slot
    changes only at the optimizer step, after this backward."""
    xq, xs = state.quant(x2, 0)
    wq, ws = state.quant(weight.contiguous(), 1)
    y = _fp8_forward_q(x2, xq, xs, wq, ws, bias, res2, act, preact, state, out8)
    if keep:
        x_keep = (xq, xs.clone()) if state.wgrad else (None, None)
        w_keep = (wq, ws if state.w_cached else ws.clone()) if state.dgrad else (None, None)
        return y, (*x_keep, *w_keep, state)
    return y


def _fp8_forward_q(x2, xq, xs, wq, ws, bias, res2, act, preact, state, out8):
    if _ext.use_native(x2):
        if (out8 is not None and res2 is None and preact is not None and x2.shape[0] > 0
                and out8.producer_ready(x2.device)):
            slot = out8.roll_slot(0)
            y, q = _ext.ops().gemm_fp8_q8(xq, wq, xs, ws, bias, act, preact, slot)
            out8.offer(y, q, slot)
            return y
        return _ext.ops().gemm_fp8(xq, wq, xs, ws, bias, res2, act, preact)
    h = dequantize_fp8(xq, xs).float() @ dequantize_fp8(wq, ws).float().t()
    if bias is not None:
        h = h + bias.float()
    if preact is not None:
        preact.copy_(_pre_ref(h, act))
    y = _act_ref(h, act)
    if res2 is not None:
        y = y + res2.float()
    return y.to(x2.dtype)


def linear_fp8(x, weight, bias=None, act=None, residual=None, state: Fp8State | None = None):
    """Linear with an fp8 e4m3 forward GEMM; the backward is the bf16 linear's
    (ops.linear: direct flat-buffer gradient accumulation, fused bias reduction)."""
    from .linear import linear
    return linear(x, weight, bias, act=act, residual=residual, fp8=state if state is not None else Fp8State())


class Fp8WeightCache:
    """e4m3 copies of every fp8 weight of a model, written right after each optimizer step.

    The forward then reads the weight operand straight from this cache instead of quantising
    the bf16 weight per GEMM call: the ~3 small launches per fp8 GEMM per step (roll, quantise,
    scale) become 2 launches for the whole model (``fp8_quant_many``: roll every weight slot,
    then quantise every weight from the flat bf16 parameter buffer, delayed scaling with one
    amax per weight).  The optimizer calls :meth:`refresh` at the end of ``step()`` (inside a
    captured step graph as well).  A cached copy is used only while the weight's version
    counter is the one recorded at the refresh, so a weight changed any other way (checkpoint
    load, manual edit) falls back to per-call quantisation until the next refresh."""

    def __init__(self, pairs, flat):
        """``pairs``: [(weight Parameter living in ``flat``, Fp8State)]."""
        self.flat = flat
        off = {id(p): o for p, o, _ in flat.segments()}
        self.entries = []
        qoff = 0
        for w, st in pairs:
            self.entries.append([w, st, off[id(w)], qoff])
            qoff += (w.numel() + 15) // 16 * 16
        dev = flat.data.device
        self.qbuf = torch.empty(max(qoff, 16), dtype=torch.uint8, device=dev)
        self.max_n = max((w.numel() for w, _ in pairs), default=0)
        self.segs = None
        self.version = {}
        self.refreshes = 0
        self.by_state = {}  # id(Fp8State) -> (weight, cached e4m3 view)
        for w, st, _, qo in self.entries:
            st.wcache = self
            self.by_state[id(st)] = (w, self.qbuf[qo:qo + w.numel()].view(w.shape))

    def _ensure_states(self):
        for w, st, _, _ in self.entries:
            if st.t is None or st.t.device != self.flat.data.device:
                st.t = torch.zeros(2, 4, device=self.flat.data.device, dtype=torch.float32)
                st.ready = [False, False]
        rows = [[o, w.numel(), qo, st.t[1].data_ptr()] for w, st, o, qo in self.entries]
        self.segs = torch.tensor(rows, dtype=torch.int64).to(self.flat.data.device)
        self._slot_ptrs = [st.t.data_ptr() for _, st, _, _ in self.entries]

    def refresh(self):
        if not self.entries or not _ext.use_native(self.flat.data):
            return
        # (re)build the device table if a state slot was (re)allocated since: the kernel writes
        # through the addresses in it
        if (self.segs is None or any(st.t is None for _, st, _, _ in self.entries)
                or [st.t.data_ptr() for _, st, _, _ in self.entries] != self._slot_ptrs):
            self._ensure_states()
        for _, st, _, _ in self.entries:
            if not st.ready[1]:  # first quantisation of this weight: current scaling, seeds the amax
                return
        _ext.ops().fp8_quant_many(self.flat.data, self.segs, self.max_n, self.qbuf)
        self.refreshes += 1
        for w, st, _, _ in self.entries:
            self.version[id(st)] = w._version

    def rebuild(self):
        """Re-create every cached e4m3 weight from the current bf16 weights WITHOUT rolling the
        delayed scales: the scales in the slots are the ones the last refresh used, so after a
        checkpoint load (weights and fp8 state slots restored together) the cache holds exactly the
        bytes the saving run's last refresh wrote and a resumed run continues bit for bit."""
        if not self.entries or not _ext.use_native(self.flat.data):
            return
        if (self.segs is None or any(st.t is None for _, st, _, _ in self.entries)
                or [st.t.data_ptr() for _, st, _, _ in self.entries] != self._slot_ptrs):
            self._ensure_states()
        if not all(st.ready[1] for _, st, _, _ in self.entries):
            return  # no scale yet (fresh run): the first forward seeds them, the next step refreshes
        _ext.ops().fp8_quant_many(self.flat.data, self.segs, self.max_n, self.qbuf, False)
        for w, st, _, _ in self.entries:
            self.version[id(st)] = w._version

    def lookup(self, st, w):
        """The cached e4m3 weight of ``st`` if it is current for ``w``, else None."""
        v = self.version.get(id(st))
        if v is None or v != w._version:
            return None
        ww, q = self.by_state[id(st)]
        return q if ww.data_ptr() == w.data_ptr() else None


def attach_weight_cache(model, flat, optimizer):
    """Give every fp8 Linear of ``model`` (``fp8_state`` + ``weight`` in ``flat``) an e4m3 weight
    copy refreshed by ``optimizer`` after each step.  Returns the cache (None if no fp8 layer)."""
    in_flat = {id(p) for p in flat.params}
    pairs = [(m.weight, m.fp8_state) for m in model.modules()
             if getattr(m, "fp8_state", None) is not None and id(getattr(m, "weight", None)) in in_flat]
    if not pairs:
        return None
    cache = Fp8WeightCache(pairs, flat)
    optimizer.post_step_hooks.append(cache.refresh)
    return cache
