"""Pre-LN transformer block shared by GPT-2 and ViT (N19/N20).

Unlike the reference's post-LN blocks (``arch/transformer.py``) this is the
GPT-2/ViT formulation: fused c_attn with bias, scale 1/sqrt(head_dim), GELU
(tanh) MLP, residual adds fused into the output-projection GEMM epilogues:

    h   = LN1(x)                               layernorm kernel
    qkv = h·Wqkvᵀ + b                          GEMM (bias epilogue)
    a   = attention(qkv)  (causal for GPT-2)   flash fwd/bwd kernels
    x   = x + a·Wprojᵀ + b                     GEMM (bias + residual epilogue)
    h   = LN2(x)
    u   = gelu(h·Wfcᵀ + b)                     GEMM (bias + GELU epilogue)
    x   = x + u·Wfc2ᵀ + b                      GEMM (bias + residual epilogue)

Six kernel launches per block forward (plus dropout when enabled).  In the
backward each LayerNorm kernel also adds the residual-branch gradient (x feeds
both the LN and the residual) and reduces Σ_rows dx = the bias gradient of the
c_proj that produced x, so neither needs a pass of its own.
"""

from __future__ import annotations

import math

import torch
import torch.nn as nn

from .. import ops


class Linear(nn.Module):
    """nn.Linear-compatible parameters (weight (out, in), bias (out,)) on the MFMA GEMM.

    ``fp8=True`` runs the forward GEMM in fp8 e4m3 with delayed scaling (ops.fp8.Fp8State);
    the backward is the bf16 one either way."""

    def __init__(self, in_features, out_features, bias=True, std=0.02, fp8=False):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.zeros(out_features)) if bias else None
        self.fp8 = fp8
        self.fp8_state = None
        if fp8:  # delayed-scaling state [activation, weight] x [scale, amax, -, -]: a checkpointed buffer
            self.register_buffer("fp8_scales", torch.zeros(2, 4))
            # and the weight gradient's dY slot (e5m2, ops.fp8.fp8_wgrad)
            self.register_buffer("fp8_gscales", torch.zeros(1, 4))
            self.fp8_state = ops.Fp8State(owner=self)
        nn.init.normal_(self.weight, std=std)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, *args, **kwargs)
        for name in ("fp8_scales", "fp8_gscales"):
            key = prefix + name
            if self.fp8 and key not in state_dict:
                # a checkpoint written before the delayed-scaling buffer existed (or by a bf16 model):
                # start from empty slots (the first call uses current scaling), not a strict-load error
                getattr(self, name).zero_()
                if key in missing_keys:
                    missing_keys.remove(key)
        if self.fp8_state is not None:  # a loaded slot holds a scale: continue with delayed scaling
            self.fp8_state.sync_ready()

    def forward(self, x, act=None, residual=None):
        return ops.linear(x, self.weight, self.bias, act=act, residual=residual, fp8=self.fp8_state)


class Fp8Slots(nn.Module):
    """Delayed-scaling state of an fp8 GEMM whose weight lives elsewhere — the GPT-2 LM head, whose weight is
    the tied token embedding: the activation / weight slots as a checkpointed buffer, as :class:`Linear`'s."""

    def __init__(self):
        super().__init__()
        self.register_buffer("fp8_scales", torch.zeros(2, 4))
        self.fp8_state = ops.Fp8State(owner=self)

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, *args, **kwargs):
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, *args, **kwargs)
        key = prefix + "fp8_scales"
        if key not in state_dict:  # a checkpoint of a model without the fp8 head: empty slots
            self.fp8_scales.zero_()
            if key in missing_keys:
                missing_keys.remove(key)
        self.fp8_state.sync_ready()


class LayerNorm(nn.Module):
    def __init__(self, n, eps=1e-5):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(n))
        self.bias = nn.Parameter(torch.zeros(n))
        self.eps = eps

    def forward(self, x, return_sum=False, producer_bias=None, fp8=None, producer_fp8=None):
        return ops.layer_norm(x, self.weight, self.bias, self.eps, return_sum=return_sum,
                              producer_bias=producer_bias, fp8=fp8, producer_fp8=producer_fp8)


class Attention(nn.Module):
    def __init__(self, n_embd, n_head, causal, attn_dropout=0.0, resid_dropout=0.0, n_layer=12, fp8=False,
                 fp8_proj=True):
        super().__init__()
        self.n_head, self.causal = n_head, causal
        self.c_attn = Linear(n_embd, 3 * n_embd, fp8=fp8)
        self.c_proj = Linear(n_embd, n_embd, std=0.02 / math.sqrt(2 * n_layer), fp8=fp8 and fp8_proj)
        self.attn_dropout, self.resid_dropout = attn_dropout, resid_dropout

    def out_bias(self):
        """Bias whose gradient equals Σ_rows of the block output's gradient (None if dropout intervenes)."""
        return self.c_proj.bias if not (self.resid_dropout > 0 and self.training) else None

    def out_fp8(self):
        """fp8 state of the projection whose output IS the block output (None: bf16, or dropout intervenes)."""
        return self.c_proj.fp8_state if self.out_bias() is not None else None

    def forward(self, h, residual, cache=None, layer=0):
        """``cache``: a :class:`KVCache` (inference) — this call's keys / values are appended at the
        cache position and the queries attend to everything cached so far (causal, bottom-right
        aligned: query i of T new tokens sees keys ≤ pos + i)."""
        B, T, E = h.shape
        if cache is not None and cache.device_pos and T == 1 and self.c_attn.fp8_state is None:
            # captured decode step: the projection's epilogue appends this token's key / value row
            buf = cache.kv[layer]
            qkv = ops.linear_kv_append(h, self.c_attn.weight, self.c_attn.bias, buf, cache.pos_t)
            q = qkv.view(B, T, 3, self.n_head, E // self.n_head)[:, :, 0]
            a = ops.attention_decode(q, buf[:, :, 0], buf[:, :, 1], cache.mask).reshape(B, T, E)
            return self.c_proj(a, residual=residual)
        qkv = self.c_attn(h).view(B, T, 3, self.n_head, E // self.n_head)
        if cache is not None:
            q = qkv[:, :, 0]
            k_all, v_all = cache.update(layer, qkv[:, :, 1:3])
            if cache.device_pos:  # device-position mode: the key mask carries causality
                a = (ops.attention_decode(q, k_all, v_all, cache.mask) if T == 1 else
                     ops.attention(q, k_all, v_all, bias=cache.mask)).reshape(B, T, E)
            else:
                a = ops.attention(q, k_all, v_all, causal=self.causal).reshape(B, T, E)
            return self.c_proj(a, residual=residual)
        a = ops.attention_packed(qkv, causal=self.causal, dropout_p=self.attn_dropout,
                                 training=self.training,
                                 producer_bias=self.c_attn.bias,
                                 consumer8=self.c_attn.fp8_state if torch.is_grad_enabled() else None)
        a = a.reshape(B, T, E)
        if self.resid_dropout > 0 and self.training:
            return residual + ops.dropout(self.c_proj(a), self.resid_dropout, True)
        return self.c_proj(a, residual=residual)


class MLP(nn.Module):
    def __init__(self, n_embd, hidden, dropout=0.0, n_layer=12, fp8=False):
        super().__init__()
        self.c_fc = Linear(n_embd, hidden, fp8=fp8)
        # fp8 c_proj takes its e4m3 input from c_fc's GEMM epilogue (ops.mlp)
        self.c_proj = Linear(hidden, n_embd, std=0.02 / math.sqrt(2 * n_layer), fp8=fp8)
        self.dropout = dropout

    def out_bias(self):
        return self.c_proj.bias if not (self.dropout > 0 and self.training) else None

    def out_fp8(self):
        return self.c_proj.fp8_state if self.out_bias() is not None else None

    def forward(self, h, residual):
        if self.dropout > 0 and self.training:
            u = self.c_fc(h, act="gelu")
            return residual + ops.dropout(self.c_proj(u), self.dropout, True)
        # one autograd node: GELU backward fused into the c_proj dgrad GEMM epilogue
        fp8 = (self.c_fc.fp8_state, self.c_proj.fp8_state) if self.c_fc.fp8 else None
        return ops.mlp(h, self.c_fc.weight, self.c_fc.bias, self.c_proj.weight, self.c_proj.bias, "gelu",
                       residual=residual, fp8=fp8)


class KVCache:
    """Per-layer key / value buffer for incremental decoding, (B, max_len, 2, H, D), allocated on
    first use in the dtype / device of the keys (one HBM allocation per layer for the whole
    generation; an append is one row copy, the attention reads strided key / value views)."""

    def __init__(self, n_layer, max_len):
        self.max_len, self.pos = max_len, 0
        self.kv = [None] * n_layer
        # device-position mode (a captured decode step, GPT2.generate(graph=True)): the write row is
        # the 1-element device tensor pos_t and the attention reads the whole buffer under the additive
        # key mask (1, 1, max_len): 0 for written rows, -inf past them — no host value per step
        self.pos_t = None
        self.mask = None
        self.device_pos = False

    def to_device_position(self):
        """Switch to device-position mode at the current host position (the same pos_t / mask
        tensors are refilled on later calls, so a graph captured on them stays valid)."""
        if self.pos_t is None:
            dev = self.kv[0].device
            self.pos_t = torch.empty(1, dtype=torch.long, device=dev)
            self.mask = torch.empty(1, 1, self.max_len, device=dev)
        self.pos_t.fill_(self.pos)
        self.mask.fill_(float("-inf"))
        self.mask[..., : self.pos] = 0.0
        self.device_pos = True

    def reset(self):
        """Start a new sequence in the same buffers (host-position mode, position 0)."""
        self.pos, self.device_pos = 0, False

    def update(self, layer, kv):
        """Append ``kv`` (B, T, 2, H, D) — the key / value slice of the packed QKV projection — at
        the cache position; returns the (key, value) views the attention reads.  K and V share one
        (B, max_len, 2, H, D) buffer per layer, so an append is ONE copy (one index_copy_ in
        device-position mode)."""
        if self.device_pos:
            buf = self.kv[layer]
            buf.index_copy_(1, self.pos_t, kv)
            return buf[:, :, 0], buf[:, :, 1]
        B, T, _, H, D = kv.shape
        if self.pos + T > self.max_len:
            raise ValueError(f"KV cache full: {self.pos} + {T} > {self.max_len}")
        if self.kv[layer] is None:
            # zeroed, not empty: the device-position step reads the WHOLE buffer under the key mask, and
            # a masked row still enters P·V as 0 · v — a NaN bit pattern in an unwritten row would
            # turn that into NaN
            self.kv[layer] = kv.new_zeros(B, self.max_len, 2, H, D)
        buf = self.kv[layer]
        buf[:, self.pos: self.pos + T].copy_(kv)
        return buf[:, : self.pos + T, 0], buf[:, : self.pos + T, 1]

    def advance(self, T):
        self.pos += T


class PreLNBlock(nn.Module):
    def __init__(self, n_embd, n_head, causal, mlp_ratio=4, dropout=0.0, n_layer=12, eps=1e-5, fp8=False,
                 fp8_proj=True):
        super().__init__()
        self.ln_1 = LayerNorm(n_embd, eps)
        self.attn = Attention(n_embd, n_head, causal, dropout, dropout, n_layer, fp8=fp8, fp8_proj=fp8_proj)
        self.ln_2 = LayerNorm(n_embd, eps)
        self.mlp = MLP(n_embd, mlp_ratio * n_embd, dropout, n_layer, fp8=fp8)

    def out_bias(self):
        return self.mlp.out_bias()

    def out_fp8(self):
        return self.mlp.out_fp8()

    def forward(self, x, prev_bias=None, cache=None, layer=0, prev_fp8=None):
        """``prev_bias`` / ``prev_fp8``: out_bias() / out_fp8() of the block that produced x (its bias gradient is
        then reduced inside ln_1's backward kernel, and an fp8 projection takes its e5m2 dY from there).
        ``cache`` / ``layer``: incremental decoding (see :class:`KVCache`)."""
        # fp8 blocks: the LayerNorms also emit the e4m3 input of c_attn / c_fc
        h, x = self.ln_1(x, return_sum=True, producer_bias=prev_bias, fp8=self.attn.c_attn.fp8_state,
                         producer_fp8=prev_fp8)
        x = self.attn(h, residual=x, cache=cache, layer=layer)
        h, x = self.ln_2(x, return_sum=True, producer_bias=self.attn.out_bias(), fp8=self.mlp.c_fc.fp8_state,
                         producer_fp8=self.attn.out_fp8())
        x = self.mlp(h, residual=x)
        return x
