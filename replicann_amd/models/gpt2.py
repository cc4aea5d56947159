"""GPT-2 (small 124M / medium 355M) — N19, the headline model of BASELINE.json.

Absent from the reference: built here from its standard
definition — learned token + position embeddings, pre-LN blocks with fused
c_attn (bias), true causal attention with scale 1/sqrt(head_dim), tanh-GELU
MLP, final LayerNorm and an LM head tied to the token embedding.

MI355X-specific choices:
  * the token-embedding / LM-head matrix is STORED with 50304 = 393·128 rows
    (MFMA tile multiple); rows ≥ 50257 are zero, never indexed, and masked out
    of the softmax by the fused cross-entropy (``n_valid_cols``), so the model
    is mathematically the 50257-vocab GPT-2;
  * the loss path never materialises fp32 logits: bf16 logits from the GEMM,
    log-sum-exp in the fused CE kernel, gradient written in place.
"""

from __future__ import annotations

import os
import weakref
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .blocks import Fp8Slots, KVCache, LayerNorm, PreLNBlock


@dataclass(frozen=True)
class GPT2Config:
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    block_size: int = 1024
    vocab_size: int = 50257
    vocab_pad: int = 50304
    dropout: float = 0.0
    ln_eps: float = 1e-5
    fp8: bool = False  # fp8 e4m3 forward GEMMs in the transformer blocks ("fp8 weights" config)
    # fp8 also for the attention output projection (its input takes one delayed-scaling quantisation pass; c_attn /
    # c_fc take e4m3 straight from the LayerNorm kernel, the MLP c_proj from the gelu_q8 pass).  On by default since
    # round 5 call V: with the fp8 LM head 131.5 vs 133.6 ms/step, and over steps 40-49 of the 50-step trajectory the
    # loss stays within 0.5 % of bf16 (held-out loss 0.24 % behind, against 1.4 % with this projection in bf16); the
    # early descent (steps 6-9) deviates up to 8 % (profiles/gpt2m_fp8_proj_r5v.txt).  REPLICANN_FP8_PROJ=0: bf16
    # (None: resolved from the environment when the config is built, not at import time)
    fp8_proj: bool | None = None
    # fp8 LM head (fp8 models, training steps only; ops.loss._LinearXentFp8Fn): 1 = logits from e4m3 h · e4m3
    # wte, the loss gradient straight to e5m2 by the cross-entropy kernel, both head gradients on the fp8 GEMMs;
    # 2 = the same gradients with the logits GEMM kept in bf16 (the loss itself unquantised); 0 = bf16 head.
    # Default 1: GPT-2-medium-fp8 132.0 ms/step against 139.9 (bf16 head) and 166.0 (bf16) on one box; the
    # held-out loss after 50 steps is within 1.4 % of the bf16 model's (1.1 % with the bf16 head)
    # (profiles/gpt2m_fp8_head_r5op.txt)
    fp8_head: int | None = None
    # LM head + loss over row chunks of this many tokens (0: the whole batch at once).  Bounds the
    # logits buffer (rows x vocab_pad bf16: 6.6 GB at b64 x 1024) for long sequences / big batches
    ce_chunk: int = 0

    def __post_init__(self):
        if self.fp8_proj is None:
            object.__setattr__(self, "fp8_proj", os.environ.get("REPLICANN_FP8_PROJ", "1") == "1")
        if self.fp8_head is None:
            object.__setattr__(self, "fp8_head", int(os.environ.get("REPLICANN_FP8_HEAD", "1")))

    @staticmethod
    def small(**kw):
        return GPT2Config(**kw)

    @staticmethod
    def medium(**kw):
        return GPT2Config(n_layer=24, n_head=16, n_embd=1024, **kw)

    @staticmethod
    def tiny(**kw):
        """Test-size config (same code paths)."""
        d = dict(n_layer=2, n_head=4, n_embd=128, block_size=128, vocab_size=1000, vocab_pad=1024)
        d.update(kw)
        return GPT2Config(**d)


_DECODE_GRAPHS: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()
# captured decode steps kept per model (least recently used evicted first): each holds a KV cache of
# 2 · n_layer · B · length · n_embd elements (≈ 2.4 GB for GPT-2-small at B = 64, length 1024)
DECODE_GRAPHS_MAX = int(os.environ.get("REPLICANN_DECODE_GRAPHS", "4"))
DECODE_LEN_BUCKET = 64  # cache lengths are rounded up to this (capped at block_size): one graph per bucket


class GPT2(nn.Module):
    def __init__(self, config: GPT2Config | None = None, **kw):
        super().__init__()
        cfg = config or GPT2Config(**kw)
        self.config = cfg
        self.wte = nn.Parameter(torch.empty(cfg.vocab_pad, cfg.n_embd))
        self.wpe = nn.Parameter(torch.empty(cfg.block_size, cfg.n_embd))
        nn.init.normal_(self.wte, std=0.02)
        nn.init.normal_(self.wpe, std=0.01)
        with torch.no_grad():
            self.wte[cfg.vocab_size:].zero_()
        self.wte._rn_shared = True  # tied: embedding + LM head both contribute gradients ...
        self.wte._rn_direct_uses = 2  # ... each accumulated in place into the flat .grad
        self.h = nn.ModuleList(
            PreLNBlock(cfg.n_embd, cfg.n_head, causal=True, dropout=cfg.dropout, n_layer=cfg.n_layer,
                       eps=cfg.ln_eps, fp8=cfg.fp8, fp8_proj=cfg.fp8_proj)
            for _ in range(cfg.n_layer)
        )
        self.ln_f = LayerNorm(cfg.n_embd, cfg.ln_eps)
        # the fp8 LM head's scale slots (the weight is wte); absent unless fp8 and fp8_head
        self.head8 = Fp8Slots() if (cfg.fp8 and cfg.fp8_head > 0) else None

    def _load_from_state_dict(self, state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                              error_msgs):
        # a checkpoint of an fp8-head model loads into a model without the head's slots (fp8_head=0, a bf16
        # model): the slots are simply not needed — not an unexpected-key error
        if self.head8 is None:
            for k in [k for k in state_dict if k.startswith(prefix + "head8.")]:
                state_dict.pop(k)
        super()._load_from_state_dict(state_dict, prefix, local_metadata, strict, missing_keys, unexpected_keys,
                                      error_msgs)

    def num_params(self, non_embedding=False):
        n = sum(p.numel() for p in self.parameters())
        n -= (self.wte.shape[0] - self.config.vocab_size) * self.config.n_embd  # zero pad rows
        if non_embedding:
            n -= self.wpe.numel()
        return n

    def hidden(self, idx, fp8_head=None):
        """Final-LayerNorm output (B, T, n_embd); ``fp8_head``: the fp8 LM head's state, whose e4m3 input the
        LayerNorm kernel then writes as well."""
        x = ops.embedding(idx, self.wte, self.wpe)
        if self.config.dropout > 0 and self.training:
            x = ops.dropout(x, self.config.dropout, True)
        prev = prev8 = None
        for blk in self.h:
            x = blk(x, prev, prev_fp8=prev8)
            prev, prev8 = blk.out_bias(), blk.out_fp8()
        return self.ln_f(x, producer_bias=prev, fp8=fp8_head, producer_fp8=prev8)

    def forward(self, idx, targets=None):
        """idx (B, T) → logits (B, T, vocab_pad) [, mean CE loss when targets given].

        With ``targets`` only the loss is returned (logits are consumed in place).
        """
        fp8h = (self.head8.fp8_state if self.head8 is not None and targets is not None and self.training
                and torch.is_grad_enabled() and self.wte.is_cuda else None)
        if fp8h is not None:
            # decide here whether the fp8 head will run: otherwise ln_f would write (and roll the slot for) an
            # e4m3 copy nobody consumes (chunked head, or shapes the fp8 head does not take)
            rows = idx.numel()
            chunk = self.config.ce_chunk
            if (chunk and chunk < rows) or not ops.loss.fp8_head_ok(idx.new_empty((rows, self.config.n_embd),
                                                                                   device="meta"), self.wte):
                fp8h = None
        h = self.hidden(idx, fp8h)
        if targets is None:
            return ops.linear(h, self.wte)[..., : self.config.vocab_size]
        return ops.linear_cross_entropy(h, self.wte, targets, n_valid_cols=self.config.vocab_size,
                                        chunk_rows=self.config.ce_chunk, fp8=fp8h,
                                        fp8_logits=self.config.fp8_head != 2)

    @torch.no_grad()
    def decode_step(self, idx, cache):
        """Logits (B, vocab) of the LAST position of ``idx`` (B, T) appended at ``cache.pos``:
        prefill (T = prompt length) and one-token decode steps share this path."""
        c = self.config
        T = idx.shape[1]
        x = ops.embedding(idx, self.wte, self.wpe[cache.pos: cache.pos + T])
        prev = None
        for i, blk in enumerate(self.h):
            x = blk(x, prev, cache=cache, layer=i)
            prev = blk.out_bias()
        h = self.ln_f(x, producer_bias=prev)
        cache.advance(T)
        return ops.linear(h[:, -1:].contiguous(), self.wte)[:, 0, : c.vocab_size]

    @torch.no_grad()
    def _device_position_step(self, tok, cache):
        """One-token decode step with every per-step value on the device (``KVCache`` device-position
        mode): capturable as a hipGraph.  Reads ``tok`` (B, 1), returns (B, vocab) logits, advances
        ``cache.pos_t``."""
        c = self.config
        cache.mask.index_fill_(2, cache.pos_t, 0.0)
        x = ops.embedding(tok, self.wte, self.wpe.index_select(0, cache.pos_t))
        prev = None
        for i, blk in enumerate(self.h):
            x = blk(x, prev, cache=cache, layer=i)
            prev = blk.out_bias()
        h = self.ln_f(x, producer_bias=prev)
        logits = ops.linear(h, self.wte)[:, 0, : c.vocab_size]
        cache.pos_t.add_(1)
        return logits

    def _capture_decode(self, cache, B):
        """Record the one-token decode step as a hipGraph (after one eager warm-up that tunes the
        decode GEMM shapes); the caller writes the next token into ``tok`` and replays."""
        dev = self.wte.device
        cache.to_device_position()
        tok = torch.zeros(B, 1, dtype=torch.long, device=dev)
        pos0 = cache.pos

        def reset():  # the warm-up wrote row pos0 and advanced the position: undo
            cache.pos_t.fill_(pos0)
            cache.mask[..., pos0:] = float("-inf")

        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            self._device_position_step(tok, cache)
        torch.cuda.current_stream(dev).wait_stream(side)
        reset()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            out = self._device_position_step(tok, cache)
        reset()
        return graph, tok, out

    @torch.no_grad()
    def generate(self, idx, max_new_tokens, *, temperature=1.0, top_k=None, top_p=None, generator=None, graph=None):
        """Autoregressive sampling with a KV cache: ``idx`` (B, T0) prompt → (B, T0 + max_new_tokens).
        ``temperature`` 0 = greedy; ``top_k`` / ``top_p`` restrict sampling.  One prefill pass over the prompt, then one-token steps whose
        attention reads the cached keys / values (no recomputation of the prefix).  ``graph``
        (default: on for GPU models): the one-token step is captured once as a hipGraph and replayed
        (per-step values live on the device), so a step costs its kernels, not ~130 host launches."""
        c = self.config
        B, T0 = idx.shape
        if T0 + max_new_tokens > c.block_size:
            raise ValueError(f"prompt {T0} + {max_new_tokens} new tokens exceeds block_size {c.block_size}")
        if top_p is not None and not 0.0 < top_p <= 1.0:
            raise ValueError(f"top_p must be in (0, 1], got {top_p}")
        use_graph = (self.wte.is_cuda if graph is None else graph) and max_new_tokens > 2
        was_training = self.training
        self.eval()
        try:
            L = T0 + max_new_tokens
            if use_graph:  # one captured step (and cache) serves every length of a bucket
                L = min(c.block_size, -(-L // DECODE_LEN_BUCKET) * DECODE_LEN_BUCKET)
            # the parameters' storage is part of the key: a graph reads them by address, so one captured
            # before a parameter was re-assigned (p.data = ...) must never be replayed
            sig = tuple(p.data_ptr() for p in self.parameters())
            key = (B, L, self.wte.dtype, self.wte.device, sig)
            graphs = self._decode_graphs()
            for k in [k for k in graphs if k[4] != sig]:
                del graphs[k]
            entry = graphs.pop(key, None) if use_graph else None
            if entry is not None:
                graphs[key] = entry  # most recently used last
            if entry is not None:  # same batch / length as an earlier call: reuse its cache and graph
                cache = entry[0]
                cache.reset()
            else:
                cache = KVCache(c.n_layer, L)
            logits = self.decode_step(idx, cache)
            out = [idx]
            for i in range(max_new_tokens):
                nxt = _sample(logits.float(), temperature, top_k, generator, top_p)
                out.append(nxt)
                if i + 1 == max_new_tokens:
                    break
                if use_graph:
                    if entry is None:
                        while len(graphs) >= max(DECODE_GRAPHS_MAX, 1):  # bounded: evict the least recently used
                            graphs.pop(next(iter(graphs)))
                        entry = (cache, *self._capture_decode(cache, B))
                        graphs[key] = entry
                    elif not cache.device_pos:
                        cache.to_device_position()
                    _, g, tok, g_out = entry
                    tok.copy_(nxt)
                    g.replay()
                    logits = g_out
                else:
                    logits = self.decode_step(nxt, cache)
            return torch.cat(out, 1)
        finally:
            self.train(was_training)

    def _decode_graphs(self):
        """Captured decode steps kept across ``generate`` calls, keyed by (batch, cache length rounded
        up to DECODE_LEN_BUCKET, dtype, device, parameter storage): a serving loop captures once per
        (batch, length bucket).  At most DECODE_GRAPHS_MAX (REPLICANN_DECODE_GRAPHS, default 4) are
        kept, least recently used evicted first.  Each holds its KV cache (2 · n_layer · B · length ·
        n_embd elements); ``clear_decode_graphs`` frees them.  Kept
        outside the module's attributes (a weak-keyed registry), so copying / pickling the model
        never touches graph objects."""
        return _DECODE_GRAPHS.setdefault(self, {})

    def clear_decode_graphs(self):
        _DECODE_GRAPHS.pop(self, None)

    def flops_per_token(self, T=None):
        """Training FLOPs per token (fwd+bwd): 6·N_matmul + attention (causal)."""
        c = self.config
        T = T or c.block_size
        n_mm = c.n_layer * 12 * c.n_embd**2 + c.vocab_size * c.n_embd
        attn = c.n_layer * 2 * 2 * T * c.n_embd * 0.5  # fwd, causal ≈ half
        return 6 * n_mm + 3 * attn


def _sample(logits, temperature, top_k, generator, top_p=None):
    """(B, V) fp32 logits → (B, 1) next-token ids: greedy (temperature 0), else sampling from the
    temperature-scaled softmax restricted to the top-k logits and / or the smallest set of tokens
    whose probability mass reaches top_p (nucleus)."""
    if temperature == 0:
        return logits.argmax(-1, keepdim=True)
    logits = logits / temperature
    if top_k is not None and top_k < logits.shape[-1]:
        kth = torch.topk(logits, top_k, dim=-1).values[:, -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    if top_p is not None and top_p < 1.0:
        srt, idx = torch.sort(logits, dim=-1, descending=True)
        cum = torch.softmax(srt, -1).cumsum(-1)
        drop = cum - torch.softmax(srt, -1) >= top_p  # mass BEFORE a token already reaches top_p
        drop[..., 0] = False  # the most likely token always stays (top_p <= 0 would drop every token)
        srt = srt.masked_fill(drop, float("-inf"))
        logits = torch.full_like(logits, float("-inf")).scatter(-1, idx, srt)
    probs = torch.softmax(logits, -1)
    return torch.multinomial(probs, 1, generator=generator)
