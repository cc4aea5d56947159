"""Bitwise reproducibility of the HIP kernels (race detection row).

Every reduction in the framework runs in a fixed order (split-K slabs, column
sums, LayerNorm partials, attention dK/dV/dQ without atomics, the global grad
norm; odd head sizes included since round 2), so two runs on the same inputs must agree bit for bit.  The one
exception is the token-embedding scatter-add, which uses fp32 atomics (order of
additions varies; bf16 atomics are never used) — it is checked for agreement to
fp32 rounding instead; with REPLICANN_DETERMINISTIC=1 the training path's scatter
accumulates 64-bit fixed point with integer atomics and is bitwise repeatable too.
"""

import pytest
import torch

from replicann_amd import ops

pytestmark = pytest.mark.gpu


def bf(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).bfloat16()


def twice(fn):
    a = fn()
    b = fn()
    return a, b


def same(a, b):
    if isinstance(a, (tuple, list)):
        return all(same(x, y) for x, y in zip(a, b))
    return a is None and b is None or torch.equal(a, b)


@pytest.mark.parametrize("split", [1, 4, 16])
def test_gemm_bitwise(cuda, split):
    torch.manual_seed(0)
    dy, x = bf(4096, 768), bf(4096, 1024)
    a, b = twice(lambda: ops.gemm(dy, x, ta=True, split_k=split, cfg=0))
    assert same(a, b)


@pytest.mark.parametrize("D,drop", [(32, 0.0), (64, 0.0), (128, 0.0), (32, 0.1), (64, 0.1), (128, 0.1)])
def test_attention_fwd_bwd_bitwise(cuda, D, drop):
    """Every MFMA head size, with and without in-kernel dropout (device seed stream reset per run)."""
    from replicann_amd.ops import rng
    torch.manual_seed(1)
    H = 768 // D
    qkv = bf(4, 512, 3, H, D).requires_grad_()
    g = bf(4, 512, H, D)

    def run():
        qkv.grad = None
        rng.manual_seed(5)
        o = ops.attention_packed(qkv, causal=True, dropout_p=drop, training=drop > 0)
        o.backward(g)
        return o.detach().clone(), qkv.grad.clone()

    a, b = twice(run)
    assert same(a, b)


@pytest.mark.parametrize("D,drop,causal", [(48, 0.0, True), (80, 0.0, False), (48, 0.1, True)])
def test_attention_generic_head_bitwise(cuda, D, drop, causal):
    """Odd head sizes (scalar generic kernels): dQ per query row, dK/dV per key row — no atomics,
    so the backward is bitwise repeatable too (it used fp32 atomics for dK/dV until round 2)."""
    from replicann_amd.ops import rng
    torch.manual_seed(3)
    H = 4
    qkv = bf(2, 200, 3, H, D).requires_grad_()
    g = bf(2, 200, H, D)

    def run():
        qkv.grad = None
        rng.manual_seed(6)
        o = ops.attention_packed(qkv, causal=causal, dropout_p=drop, training=drop > 0)
        o.backward(g)
        return o.detach().clone(), qkv.grad.clone()

    a, b = twice(run)
    assert same(a, b)


def test_layernorm_bwd_bitwise(cuda):
    torch.manual_seed(2)
    x = bf(8192, 768).requires_grad_()
    w, bb = bf(768).requires_grad_(), bf(768).requires_grad_()
    g = bf(8192, 768)

    def run():
        for t in (x, w, bb):
            t.grad = None
        ops.layer_norm(x, w, bb).backward(g)
        return x.grad.clone(), w.grad.clone(), bb.grad.clone()

    a, b = twice(run)
    assert same(a, b)


def test_cross_entropy_bitwise(cuda):
    torch.manual_seed(3)
    h = bf(2048, 768).requires_grad_()
    w = bf(50304, 768, scale=0.02).requires_grad_()
    t = torch.randint(0, 50257, (2048,), device="cuda")

    def run():
        h.grad = w.grad = None
        loss = ops.linear_cross_entropy(h, w, t, n_valid_cols=50257)
        loss.backward()
        return loss.detach().clone(), h.grad.clone(), w.grad.clone()

    a, b = twice(run)
    assert same(a, b)


def test_optimizer_step_bitwise(cuda):
    from replicann_amd.optim import FusedAdamW
    from replicann_amd.utils.flat import FlatParams

    def run():
        torch.manual_seed(4)
        m = torch.nn.Linear(512, 512).cuda().bfloat16()
        flat = FlatParams(m)
        opt = FusedAdamW(flat, lr=1e-3)
        for _ in range(3):
            flat.grad.copy_(torch.randn_like(flat.grad.float()).bfloat16())
            opt.step()
        return flat.data.clone(), opt.m.clone(), opt.v.clone(), opt.norm_buf.clone()

    a, b = twice(run)
    assert same(a, b)


def test_embedding_scatter_close(cuda):
    torch.manual_seed(5)
    V, E = 1000, 256
    wte = bf(V, E).requires_grad_()
    ids = torch.randint(0, 50, (8, 128), device="cuda")  # many repeats → contended atomics
    g = bf(8, 128, E)

    def run():
        wte.grad = None
        ops.embedding(ids, wte).backward(g)
        return wte.grad.float().clone()

    a, b = twice(run)
    ref = torch.zeros(V, E, device="cuda").index_add_(0, ids.reshape(-1), g.reshape(-1, E).float())
    assert ((a - b).abs().max() <= 1e-2 * ref.abs().max())
    assert ((a - ref).norm() / ref.norm()) < 1e-2


def test_embedding_scatter_deterministic_mode(cuda, monkeypatch):
    """REPLICANN_DETERMINISTIC=1: the flat-buffer (training) embedding backward is bitwise repeatable
    under heavy id repetition and matches the fp32 index_add reference."""
    from replicann_amd.utils.flat import FlatParams

    monkeypatch.setenv("REPLICANN_DETERMINISTIC", "1")
    torch.manual_seed(7)
    V, E = 1000, 256
    mod = torch.nn.Module()
    mod.wte = torch.nn.Parameter(bf(V, E))
    flat = FlatParams(mod)
    ids = torch.randint(0, 50, (8, 128), device="cuda")  # many repeats per row
    g = bf(8, 128, E)

    def run():
        flat.zero_grad()
        ops.embedding(ids, mod.wte).backward(g)
        return mod.wte.grad.float().clone()

    a, b = twice(run)
    assert torch.equal(a, b)
    ref = torch.zeros(V, E, device="cuda").index_add_(0, ids.reshape(-1), g.reshape(-1, E).float())
    assert ((a - ref).norm() / ref.norm()) < 1e-2


def test_embedding_scatter_deterministic_tiny_gradients(cuda, monkeypatch):
    """The fixed-point deterministic scatter keeps gradients of a small loss scale (1e-9 .. 1e-7 per
    token, e.g. 1/(B·T·grad_accum)) as accurately as the fp32-atomic path (a 2^-32
    resolution rounded them to a few bits)."""
    from replicann_amd.utils.flat import FlatParams

    torch.manual_seed(8)
    V, E = 512, 128
    ids = torch.randint(0, 40, (4, 256), device="cuda")
    g = (torch.randn(4, 256, E, device="cuda") * 1e-8).bfloat16()
    ref = torch.zeros(V, E, device="cuda").index_add_(0, ids.reshape(-1), g.reshape(-1, E).float())
    out = {}
    for det in ("0", "1"):
        monkeypatch.setenv("REPLICANN_DETERMINISTIC", det)
        mod = torch.nn.Module()
        mod.wte = torch.nn.Parameter(torch.zeros(V, E, device="cuda", dtype=torch.bfloat16))
        flat = FlatParams(mod)
        flat.zero_grad()
        ops.embedding(ids, mod.wte).backward(g)
        out[det] = mod.wte.grad.float().clone()
    err = {k: float((v - ref).norm() / ref.norm()) for k, v in out.items()}
    assert err["1"] < 1e-2 and err["1"] <= 2 * err["0"] + 1e-3, err


def test_training_step_bitwise_deterministic_mode(cuda, monkeypatch):
    """With REPLICANN_DETERMINISTIC=1 a whole GPT-2 training run (embedding scatter, GEMMs incl.
    split-K, attention, LayerNorm, CE, grad-norm, AdamW with stochastic rounding) repeats bit for bit."""
    from replicann_amd.training import TrainConfig, Trainer

    monkeypatch.setenv("REPLICANN_DETERMINISTIC", "1")

    def run():
        cfg = TrainConfig(model="gpt2-tiny", batch_size=4, seq_len=128, steps=100, warmup_steps=1, lr=1e-3,
                          log_every=10**9, seed=11, graph="off")
        tr = Trainer(cfg)
        losses = [float(tr.step()) for _ in range(4)]
        return losses, tr.flat.data.clone()

    (la, wa), (lb, wb) = run(), run()
    assert la == lb and torch.equal(wa, wb)
