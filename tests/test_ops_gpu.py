"""T2: every HIP kernel vs a plain PyTorch fp32 reference of the same op (gfx950 only)."""

import math

import pytest
import torch
import torch.nn.functional as F

from replicann_amd import _ext, ops

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def bf(*shape, scale=1.0, dev="cuda"):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def test_native_loaded(cuda):
    assert _ext.available()
    assert torch.ops.replicann.native_version() == 1


# ----------------------------------------------------------------- GEMM
@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 4, 5, 6, 8, 9])
@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (200, 72, 96), (1000, 384, 520), (64, 24, 8), (520, 776, 1088)])
def test_gemm_layouts(cuda, ta, tb, M, N, K, cfg):
    torch.manual_seed(0)
    a = bf(K, M) if ta else bf(M, K)
    b = bf(N, K) if tb else bf(K, N)
    ref = (a.float().t() if ta else a.float()) @ (b.float().t() if tb else b.float())
    out = ops.gemm(a, b, ta=ta, tb=tb, cfg=cfg)
    assert out.shape == (M, N)
    assert rel_err(out, ref) < 1e-2


@pytest.mark.parametrize("ta,tb", [(False, True), (False, False), (True, False), (True, True)])
@pytest.mark.parametrize("M,N,K", [(8192, 2304, 768), (4352, 4200, 200), (8200, 1032, 72), (2048, 512, 64)])
def test_gemm_persistent_multi_tile(cuda, ta, tb, M, N, K):
    """cfg 9 walks several output tiles per workgroup with the operand stream running across tile
    boundaries (epilogue while the next tile's half-tiles are in flight); ragged M/N/K tails."""
    torch.manual_seed(11)
    a = bf(K, M) if ta else bf(M, K)
    b = bf(N, K) if tb else bf(K, N)
    bias, res = bf(N), bf(M, N)
    af = a.float().t() if ta else a.float()
    bf_ = b.float().t() if tb else b.float()
    ref = af @ bf_
    out = ops.gemm(a, b, ta=ta, tb=tb, cfg=9)
    assert rel_err(out, ref) < 1e-2
    out = ops.gemm(a, b, ta=ta, tb=tb, cfg=9, bias=bias, residual=res)
    assert rel_err(out, ref + bias.float() + res.float()) < 1e-2
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out = ops.gemm(a, b, ta=ta, tb=tb, cfg=9, bias=bias, act=2, preact=pre)
    h = ref + bias.float()
    assert rel_err(pre, h) < 1e-2 and rel_err(out, F.gelu(h, approximate="tanh")) < 1e-2
    o32 = ops.gemm(a, b, ta=ta, tb=tb, cfg=9, out_dtype=torch.float32)
    assert o32.dtype == torch.float32 and rel_err(o32, ref) < 5e-3


def test_gemm_persistent_act_backward_multi_tile(cuda):
    torch.manual_seed(12)
    M, N, K = 4600, 3072, 768
    dy, w, pre = bf(M, K), bf(K, N, scale=0.05), bf(M, N)
    bg = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    out = torch.ops.replicann.gemm(dy, w, False, False, None, None, 4, pre, None, False, 0, False, None, 9, bg)
    du = (dy.float() @ w.float()).bfloat16().float()
    pf = pre.float().requires_grad_()
    (g,) = torch.autograd.grad(F.gelu(pf, approximate="tanh"), pf, du)
    assert rel_err(out, g) < 1e-2
    assert rel_err(bg.float(), out.float().sum(0)) < 2e-2


@pytest.mark.parametrize("act", [3, 4, 6])
@pytest.mark.parametrize("M,N,K", [(9000, 3000, 768), (9000, 3000, 128), (600, 5000, 320)])
def test_gemm_persistent_act_backward_prefetch(cuda, act, M, N, K):
    """Act-backward epilogues with the saved-activation L2 prefetch (gemm_pk.h, PF): several items
    per workgroup, ragged M/N edges, K slices shorter than the 4-K-tile prefetch window."""
    torch.manual_seed(13)
    dy, w, pre = bf(M, K), bf(K, N, scale=0.05), bf(M, N)
    bg = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    out = torch.ops.replicann.gemm(dy, w, False, False, None, None, act, pre, None, False, 0, False, None, 9, bg)
    du = (dy.float() @ w.float()).bfloat16().float()
    if act == 6:
        ref = du * pre.float()
    else:
        pf = pre.float().requires_grad_()
        y = F.relu(pf) if act == 3 else F.gelu(pf, approximate="tanh")
        (ref,) = torch.autograd.grad(y, pf, du)
    assert rel_err(out, ref) < 1e-2
    assert rel_err(bg.float(), out.float().sum(0)) < 2e-2


def test_gemm_alpha(cuda):
    a, b = bf(300, 128), bf(200, 128)
    alpha = torch.tensor([0.25], device="cuda")
    out = ops.gemm(a, b, tb=True, alpha=alpha)
    assert rel_err(out, 0.25 * (a.float() @ b.float().t())) < 1e-2


def test_gemm_identity_asymmetric(cuda):
    # A = I with an asymmetric B catches a transposed C-write
    M = 128
    a = torch.eye(M, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(M * 64, device="cuda").reshape(64, M) % 61).to(torch.bfloat16)  # [N=64][K=M]
    out = ops.gemm(a, b, tb=True)
    torch.testing.assert_close(out.float(), b.float().t(), atol=0, rtol=0)


@pytest.mark.parametrize("cfg", [-1, 1, 9])
@pytest.mark.parametrize("act", [0, 1, 2])
def test_gemm_epilogue(cuda, act, cfg):
    torch.manual_seed(1)
    M, N, K = 300, 264, 192
    a, w = bf(M, K), bf(N, K, scale=0.1)
    bias, res = bf(N), bf(M, N)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out = ops.gemm(a, w, tb=True, bias=bias, residual=res, act=act, preact=pre if act else None, cfg=cfg)
    h = a.float() @ w.float().t() + bias.float()
    y = {0: h, 1: F.relu(h), 2: F.gelu(h, approximate="tanh")}[act] + res.float()
    assert rel_err(out, y) < 1e-2
    if act:
        assert rel_err(pre, h) < 1e-2


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64])
@pytest.mark.parametrize("N,K,split", [(24, 8, 0), (768, 768, 0), (1000, 1000, 3), (2304, 96, 2), (200, 3072, 12)])
def test_gemm_skinny_decode(cuda, M, N, K, split):
    """Config 10 (decode-size x·Wᵀ, gemm_skinny.hip) against fp32 math: bias + residual, the GELU
    saved-derivative epilogue, split-K partials; bitwise repeatable."""
    torch.manual_seed(M * 7 + N)
    a, w = bf(M, K), bf(N, K, scale=0.1)
    bias, res = bf(N), bf(M, N)
    out = ops.gemm(a, w, tb=True, bias=bias, residual=res, split_k=split, cfg=10)
    h = a.float() @ w.float().t() + bias.float()
    assert rel_err(out, h + res.float()) < 1e-2
    assert torch.equal(out, ops.gemm(a, w, tb=True, bias=bias, residual=res, split_k=split, cfg=10))
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    y = ops.gemm(a, w, tb=True, bias=bias, act=5, preact=pre, split_k=split, cfg=10)
    assert rel_err(y, F.gelu(h, approximate="tanh")) < 1e-2
    assert rel_err(pre, _gelu_grad(h.bfloat16())) < 1e-2
    r = ops.gemm(a, w, tb=True, act=1, split_k=split, cfg=10)
    assert rel_err(r, F.relu(a.float() @ w.float().t())) < 1e-2
    o32 = ops.gemm(a, w, tb=True, split_k=split, cfg=10, out_dtype=torch.float32)
    assert o32.dtype == torch.float32 and rel_err(o32, a.float() @ w.float().t()) < 5e-3


@pytest.mark.parametrize("B,H,Tk", [(1, 12, 256), (3, 2, 19), (64, 12, 129), (2, 4, 1024)])
def test_attention_decode_one_query(cuda, B, H, Tk):
    """One-query attention over a strided K|V cache view with an additive key mask (the captured
    decode step's form) against fp32 math."""
    torch.manual_seed(B * H + Tk)
    qkv = bf(B, 1, 3, H, 64)
    kv = bf(B, Tk + 5, 2, H, 64)  # a longer buffer: the kernel reads the first Tk rows of strided views
    q, k, v = qkv[:, :, 0], kv[:, :Tk, 0], kv[:, :Tk, 1]
    mask = torch.zeros(1, 1, Tk, device="cuda")
    mask[..., Tk * 2 // 3:] = float("-inf")
    with torch.no_grad():
        o = ops.attention_decode(q, k, v, mask)
    ref = ops.attention_reference(q, k, v, 64 ** -0.5, bias=mask)
    assert o.shape == (B, 1, H, 64) and rel_err(o, ref) < 1e-2
    with torch.no_grad():
        o2 = ops.attention_decode(q, k, v, None)
    assert rel_err(o2, ops.attention_reference(q, k, v, 64 ** -0.5)) < 1e-2


@pytest.mark.parametrize("B,H", [(1, 12), (5, 2), (64, 12)])
def test_linear_kv_append(cuda, B, H):
    """Decode QKV projection with the K|V cache append in the epilogue: the output equals the plain
    GEMM, cache row pos holds its key / value columns, every other row is untouched."""
    torch.manual_seed(B + H)
    E, L = 64 * H, 40
    x, w, bias = bf(B, 1, E), bf(3 * E, E, scale=0.05), bf(3 * E, scale=0.1)
    kv = bf(B, L, 2, H, 64)
    before = kv.clone()
    pos = torch.tensor([17], device="cuda")
    with torch.no_grad():
        y = ops.linear_kv_append(x, w, bias, kv, pos)
    ref = ops.gemm(x.reshape(B, E), w, tb=True, bias=bias)
    assert y.shape == (B, 1, 3 * E) and rel_err(y.reshape(B, -1), ref) < 1e-2
    assert torch.equal(kv[:, 17].reshape(B, -1), y.reshape(B, -1)[:, E:])
    keep = torch.ones(L, dtype=torch.bool)
    keep[17] = False
    assert torch.equal(kv[:, keep], before[:, keep])


def test_gemm_skinny_rejects_other_layouts(cuda):
    a, w = bf(16, 64), bf(64, 32)
    with pytest.raises(RuntimeError):
        ops.gemm(a, w, cfg=10)  # B not K-contiguous: config 10 takes the Linear forward layout only
    with pytest.raises(RuntimeError):
        ops.gemm(bf(128, 64), bf(32, 64), tb=True, cfg=10)  # M > 64


def _gelu_grad(h):
    hf = h.float().requires_grad_()
    (g,) = torch.autograd.grad(F.gelu(hf, approximate="tanh"), hf, torch.ones_like(hf))
    return g


@pytest.mark.parametrize("cfg,split", [(-1, 0), (0, 0), (1, 0), (6, 0), (9, 0), (9, 3), (0, 4)])
def test_gemm_gelu_saved_derivative(cuda, cfg, split):
    """Epilogue code 5 (forward: y = gelu(h), pre = gelu'(h)) and code 6 (dgrad: out = (dY·W) ⊙ pre),
    the pair the fused MLP uses; against fp32 math."""
    torch.manual_seed(21)
    M, N, K = 520, 776, 384
    a, w, bias = bf(M, K), bf(N, K, scale=0.1), bf(N)
    pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    out = torch.ops.replicann.gemm(a, w, False, True, bias, None, 5, pre, None, False, split, False, None, cfg, None)
    h = a.float() @ w.float().t() + bias.float()
    assert rel_err(out, F.gelu(h, approximate="tanh")) < 1e-2
    assert rel_err(pre, _gelu_grad(h)) < 1e-2
    dy, w2 = bf(M, K), bf(K, N, scale=0.1)
    bg = torch.zeros(N, device="cuda", dtype=torch.bfloat16)
    dh = torch.ops.replicann.gemm(dy, w2, False, False, None, None, 6, pre, None, False, split, False, None, cfg, bg)
    ref = (dy.float() @ w2.float()).bfloat16().float() * pre.float()
    assert rel_err(dh, ref) < 1e-2
    assert rel_err(bg.float(), dh.float().sum(0)) < 2e-2


@pytest.mark.parametrize("split,cfg", [(2, 0), (4, 1), (8, -1), (3, 2), (4, 9), (7, 9)])
def test_gemm_splitk_fp32_accumulate(cuda, split, cfg):
    torch.manual_seed(2)
    M, N, K = 192, 320, 4096
    a, b = bf(K, M), bf(K, N)
    ref = a.float().t() @ b.float()
    out = ops.gemm(a, b, ta=True, split_k=split, out_dtype=torch.float32, cfg=cfg)
    assert out.dtype == torch.float32 and rel_err(out, ref) < 5e-3
    acc = torch.ones(M, N, device="cuda")
    ops.gemm(a, b, ta=True, split_k=split, out=acc, accumulate=True)
    assert rel_err(acc, ref + 1) < 5e-3


def test_linear_autograd(cuda):
    torch.manual_seed(3)
    x = bf(4, 33, 96).requires_grad_()
    w = bf(160, 96, scale=0.1).requires_grad_()
    b = bf(160).requires_grad_()
    r = bf(4, 33, 160).requires_grad_()
    y = ops.linear(x, w, b, act="gelu", residual=r)
    g = bf(4, 33, 160)
    y.backward(g)
    xf, wf, bf_, rf = [t.detach().float().requires_grad_() for t in (x, w, b, r)]
    yf = F.gelu(xf @ wf.t() + bf_, approximate="tanh") + rf
    yf.backward(g.float())
    assert rel_err(y, yf) < 1e-2
    for t, tf in ((x, xf), (w, wf), (b, bf_), (r, rf)):
        assert rel_err(t.grad, tf.grad) < 2e-2


@pytest.mark.parametrize("act", [3, 4])
@pytest.mark.parametrize("cfg,split", [(0, 0), (1, 0), (6, 0), (2, 0), (0, 4), (-1, 0), (9, 0), (9, 3)])
def test_gemm_act_backward_epilogue(cuda, act, cfg, split):
    """dH = (dY·W) ⊙ act'(pre) fused into the dgrad GEMM epilogue (3 = ReLU', 4 = GELU')."""
    torch.manual_seed(7)
    M, N, K = 520, 776, 384
    dy, w, pre = bf(M, K), bf(K, N, scale=0.1), bf(M, N)
    bg = bf(N)
    bg0 = bg.float().clone()
    out = torch.ops.replicann.gemm(dy, w, False, False, None, None, act, pre, None, False, split, False, None, cfg, bg)
    du = (dy.float() @ w.float()).bfloat16().float()
    pf = pre.float().requires_grad_()
    y = F.relu(pf) if act == 3 else F.gelu(pf, approximate="tanh")
    (g,) = torch.autograd.grad(y, pf, du)
    assert rel_err(out, g) < 1e-2
    # fused bias gradient (column partials in the epilogue, or the fallback pass) accumulates Σ_rows out
    assert rel_err(bg.float() - bg0, out.float().sum(0)) < 2e-2


def test_mlp_fused_matches_unfused(cuda):
    torch.manual_seed(8)
    E, H, M = 256, 1024, 300
    x = bf(M, E).requires_grad_()
    r = bf(M, E).requires_grad_()
    w1, b1 = bf(H, E, scale=0.05).requires_grad_(), bf(H, scale=0.1).requires_grad_()
    w2, b2 = bf(E, H, scale=0.05).requires_grad_(), bf(E, scale=0.1).requires_grad_()
    g = bf(M, E)
    y = ops.mlp(x, w1, b1, w2, b2, "gelu", residual=r)
    y.backward(g)
    got = [t.grad.clone() for t in (x, r, w1, b1, w2, b2)]
    ts = [t.detach().float().requires_grad_() for t in (x, r, w1, b1, w2, b2)]
    xf, rf, w1f, b1f, w2f, b2f = ts
    yf = F.linear(F.gelu(F.linear(xf, w1f, b1f), approximate="tanh"), w2f, b2f) + rf
    yf.backward(g.float())
    assert rel_err(y, yf) < 1e-2
    for a, t in zip(got, ts):
        assert rel_err(a, t.grad) < 2e-2


def test_gemm_library_candidate_plain_only(cuda):
    """cfg 7 (vendor library) serves plain GEMMs only; the autotuner cache is keyed by the epilogue,
    so a shape tuned plain never sends a biased call to the library."""
    torch.manual_seed(9)
    a, w, bias = bf(640, 256), bf(384, 256), bf(384)
    ref = a.float() @ w.float().t()
    assert rel_err(torch.ops.replicann.gemm(a, w, False, True, None, None, 0, None, None, False, 0, False, None, 7),
                   ref) < 1e-2
    with pytest.raises(RuntimeError):
        torch.ops.replicann.gemm(a, w, False, True, bias, None, 0, None, None, False, 0, False, None, 7)
    plain = ops.gemm(a, w, tb=True)        # tunes the plain key (library is a candidate)
    biased = ops.gemm(a, w, tb=True, bias=bias)
    assert rel_err(plain, ref) < 1e-2
    assert rel_err(biased, ref + bias.float()) < 1e-2


# ----------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("E", [768, 1024, 96])
def test_layernorm(cuda, E):
    torch.manual_seed(4)
    x, r = bf(37, E), bf(37, E)
    w, b = bf(E).requires_grad_(), bf(E).requires_grad_()
    xg, rg = x.clone().requires_grad_(), r.clone().requires_grad_()
    y, h = ops.layer_norm(xg, w, b, 1e-5, residual=rg, return_sum=True)
    gy = bf(37, E)
    (y.float() * gy.float()).sum().backward()
    xf, rf, wf, bf_ = [t.detach().float().requires_grad_() for t in (x, r, w, b)]
    yf = F.layer_norm(xf + rf, (E,), wf, bf_, 1e-5)
    (yf * gy.float()).sum().backward()
    assert rel_err(y, yf) < 1e-2
    assert rel_err(h, xf + rf) < 1e-2
    for t, tf in ((xg, xf), (rg, rf), (w, wf), (b, bf_)):
        assert rel_err(t.grad, tf.grad) < 2e-2


@pytest.mark.parametrize("M,E", [(37, 768), (5000, 96), (16384, 768), (300, 4096)])
def test_layernorm_passthrough_producer_bias(cuda, M, E):
    """Pre-LN block form: (y, x) = LN(x) with x also the residual; the kernel fuses the
    residual-gradient add and reduces Σ_rows dx into the producer's bias grad."""
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(5)
    mod = torch.nn.Module()
    mod.w = torch.nn.Parameter(torch.randn(E, device="cuda").bfloat16())
    mod.b = torch.nn.Parameter(torch.randn(E, device="cuda").bfloat16())
    mod.pb = torch.nn.Parameter(torch.zeros(E, device="cuda").bfloat16())
    flat = FlatParams(mod)
    flat.zero_grad()
    x = bf(M, E).requires_grad_()
    gy, gr = bf(M, E), bf(M, E)
    y, xp = ops.layer_norm(x, mod.w, mod.b, 1e-5, return_sum=True, producer_bias=mod.pb)
    ((y.float() * gy.float()).sum() + (xp.float() * gr.float()).sum()).backward()
    assert mod.pb._rn_bias_done
    xf, wf, bf_ = [t.detach().float().requires_grad_() for t in (x, mod.w, mod.b)]
    yf = F.layer_norm(xf, (E,), wf, bf_, 1e-5)
    ((yf * gy.float()).sum() + (xf * gr.float()).sum()).backward()
    assert rel_err(y, yf) < 1e-2
    assert rel_err(x.grad, xf.grad) < 2e-2
    assert rel_err(mod.w.grad, wf.grad) < 2e-2 and rel_err(mod.b.grad, bf_.grad) < 2e-2
    assert rel_err(mod.pb.grad, x.grad.float().sum(0)) < 1e-2


@pytest.mark.parametrize("C,M", [(64, 3000), (200, 3000), (2304, 3000), (50304, 3000), (64, 40000), (96, 20000)])
def test_bias_grad_column_reduction(cuda, C, M):
    """Deterministic column sums of the row-split partials (the splitter makes <= 512 of them, so the
    one-pass kernel; up to 512 rows at M=40000, C=64) — bitwise repeatable.  The two-stage last-block
    kernel (> 512 partial rows) is exercised by the LayerNorm-backward tests."""
    torch.manual_seed(6)
    dy = bf(M, C)
    _, db1 = torch.ops.replicann.bias_act_grad(dy, None, 0, True, None)
    _, db2 = torch.ops.replicann.bias_act_grad(dy, None, 0, True, None)
    assert rel_err(db1, dy.float().sum(0)) < 1e-2
    assert torch.equal(db1, db2)


# ----------------------------------------------------------------- cross entropy
def test_cross_entropy_padded(cuda):
    torch.manual_seed(5)
    N, V, nv = 64, 1024, 1000
    logits = bf(N, V, scale=3.0)
    tgt = torch.randint(0, nv, (N,), device="cuda")
    tgt[3] = -100
    lg = logits.clone().requires_grad_()
    loss = ops.cross_entropy(lg, tgt, n_valid_cols=nv)
    loss.backward()
    lf = logits.float()[:, :nv].requires_grad_()
    lref = F.cross_entropy(lf, tgt, ignore_index=-100)
    lref.backward()
    assert abs(loss.item() - lref.item()) < 1e-2
    assert rel_err(lg.grad[:, :nv], lf.grad) < 2e-2
    assert lg.grad[:, nv:].abs().max().item() == 0


@pytest.mark.parametrize("chunk", [256, 384])
def test_linear_cross_entropy_chunked(cuda, chunk):
    """LM head + CE over row chunks (gradients formed in the forward, scaled by g in the
    backward) vs the whole-batch fused path and fp32 math; a partial last chunk (1000 rows,
    384-row chunks), ignore_index rows and a non-unit upstream gradient."""
    torch.manual_seed(11)
    R, E, V, nv = 1000, 128, 2048, 2000
    h = bf(R, E)
    w = bf(V, E, scale=0.5)
    w[nv:] = 0
    t = torch.randint(0, nv, (R,), device="cuda")
    t[::37] = -100
    outs = []
    for c in (0, chunk):
        hh = h.clone().requires_grad_()
        ww = w.clone().requires_grad_()
        loss = ops.linear_cross_entropy(hh, ww, t, n_valid_cols=nv, chunk_rows=c)
        (loss * 0.75).backward()
        outs.append((loss.detach(), hh.grad.float(), ww.grad.float()))
    hf = h.float().requires_grad_()
    wf = w.float().requires_grad_()
    lref = F.cross_entropy((hf @ wf.t())[:, :nv], t, ignore_index=-100)
    (lref * 0.75).backward()
    (l0, gh0, gw0), (l1, gh1, gw1) = outs
    assert abs(l1.item() - lref.item()) < 1e-2 and abs(l1.item() - l0.item()) < 2e-3
    assert rel_err(gh1, hf.grad) < 2e-2 and rel_err(gw1, wf.grad) < 2e-2
    assert rel_err(gh1, gh0) < 1e-2 and rel_err(gw1, gw0) < 1e-2
    assert gw1[nv:].abs().max().item() == 0


def test_fused_lm_xent_rows_gpt2_vocab(cuda):
    """The in-place gradient row kernel at GPT-2's padded vocab (50304 columns, 50257 valid):
    one block reduction, one exp per element."""
    torch.manual_seed(8)
    N, V, nv = 96, 50304, 50257
    logits = bf(N, V, scale=4.0)
    tgt = torch.randint(0, nv, (N,), device="cuda")
    tgt[5] = -100
    tgt[7] = nv - 1
    tgt[9] = 0
    g = logits.clone()
    loss_rows, lse = torch.ops.replicann.xent_fwd(g, tgt, nv, -100, True)
    lf = logits.float()[:, :nv]
    ref_lse = torch.logsumexp(lf, 1)
    ref_rows = F.cross_entropy(lf, tgt.clamp(min=0), reduction="none")
    ref_rows[5] = 0
    ref_g = torch.softmax(lf, 1)
    ref_g[torch.arange(N), tgt.clamp(min=0)] -= 1
    ref_g[5] = 0
    torch.cuda.synchronize()
    assert (lse - ref_lse).abs().max().item() < 1e-3
    assert (loss_rows - ref_rows).abs().max().item() < 2e-2
    assert (g[:, :nv].float() - ref_g).abs().max().item() < 4e-3
    assert rel_err(g[:, :nv], ref_g) < 1e-2
    assert g[:, nv:].abs().max().item() == 0 and g[5].abs().max().item() == 0


# ----------------------------------------------------------------- attention
def _attn_check(B, T, H, D, causal, bias=None, Tk=None, tol=2e-2):
    Tk = Tk or T
    q, k, v = bf(B, T, H, D), bf(B, Tk, H, D), bf(B, Tk, H, D)
    qg, kg, vg = [t.clone().requires_grad_() for t in (q, k, v)]
    scale = 1 / math.sqrt(D) if D != 64 else 0.125
    o = ops.attention(qg, kg, vg, scale=scale, causal=causal, bias=bias)
    go = bf(B, T, H, D)
    o.backward(go)
    qf, kf, vf = [t.detach().float().requires_grad_() for t in (q, k, v)]
    of = ops.attention_reference(qf, kf, vf, scale, causal, bias)
    of.backward(go.float())
    assert rel_err(o, of) < tol
    for t, tf in ((qg, qf), (kg, kf), (vg, vf)):
        assert rel_err(t.grad, tf.grad) < 2 * tol


@pytest.mark.parametrize("causal", [True, False])
@pytest.mark.parametrize("T", [256, 197, 64])
def test_attention_d64(cuda, causal, T):
    torch.manual_seed(6)
    _attn_check(2, T, 3, 64, causal)


def test_attention_d64_long(cuda):
    torch.manual_seed(7)
    _attn_check(1, 1024, 2, 64, True)


def test_attention_d64_causal_offsets(cuda):
    """The causal D=64 kernels (forward, dQ, dK/dV) against the fp32 reference: full, diagonal and
    ragged tiles, Tq != Tk (causal offset), partial last blocks; a non-causal ragged case.
    (The round-4 arms — 64 queries per wave, a software-pipelined forward / dK-dV, 4 query / key
    groups per wave — measured slower and were removed: profiles/attention_arms_r4e.txt.)"""
    torch.manual_seed(70)
    _attn_check(2, 320, 3, 64, True)
    _attn_check(1, 100, 2, 64, True, Tk=260)
    _attn_check(1, 1024, 2, 64, True)
    _attn_check(1, 130, 2, 64, False, Tk=70)


def test_attention_bias_additive(cuda):
    torch.manual_seed(8)
    T = 96
    bias = torch.tril(torch.ones(T, T, device="cuda")).unsqueeze(0)  # the reference's 0/1 mask, added
    _attn_check(2, T, 2, 64, False, bias=bias)


@pytest.mark.parametrize("D", [32, 128])
@pytest.mark.parametrize("causal", [True, False])
def test_attention_mfma_d(cuda, D, causal):
    """Head sizes 32 / 128 on the MFMA kernels (templated on D; no fp32 atomics): several key tiles,
    ragged T, Tq != Tk (causal offset / ragged key blocks), additive bias."""
    assert ops.attention_is_mfma(D)
    torch.manual_seed(90 + D)
    _attn_check(2, 320, 3, D, causal)
    _attn_check(1, 100, 2, D, causal, Tk=260)
    if not causal:
        _attn_check(1, 130, 2, D, False, Tk=70)
        T = 96
        _attn_check(2, T, 2, D, False, bias=torch.tril(torch.ones(T, T, device="cuda")).unsqueeze(0))


@pytest.mark.parametrize("T,Tk", [(197, None), (33, None), (256, None), (150, 230), (230, 96), (5, 3)])
def test_attention_resident_head(cuda, T, Tk):
    """Whole-head-resident D = 64 kernels (Tq, Tk <= 256): the forward (8 waves, K / V staged once) and the
    persistent backward (one workgroup per CU walking B·H heads, next head's tiles streamed during the
    current head's phases) — B·H = 384 heads > the CU count, so workgroups carry several heads and the
    cross-head pipelining (prefetched registers, tiles refilled between barriers) is exercised."""
    torch.manual_seed(14)
    _attn_check(32, T, 12, 64, False, Tk=Tk)


def test_attention_resident_single_token(cuda):
    """T = 1 through the resident kernels: softmax over one key is exactly 1, so O = V, dV = dO and dQ = dK = 0
    in exact arithmetic (a relative error against that zero reference is meaningless: absolute bounds)."""
    torch.manual_seed(17)
    B, H = 8, 12
    q, k, v, go = (bf(B, 1, H, 64) for _ in range(4))
    qg, kg, vg = [t.clone().requires_grad_() for t in (q, k, v)]
    o = ops.attention(qg, kg, vg, scale=0.125, causal=False)
    o.backward(go)
    assert rel_err(o, v) < 1e-2 and rel_err(vg.grad, go) < 1e-2
    assert qg.grad.float().abs().max() < 1e-4 and kg.grad.float().abs().max() < 1e-4


@pytest.mark.parametrize("T,Tk", [(100, 200), (64, 64), (250, 256)])
def test_attention_resident_forward_causal(cuda, T, Tk):
    """The resident forward's causal form (Tq, Tk <= 256, incl. Tq < Tk: the causal offset) against the fp32
    reference; its backward is the streaming pair."""
    torch.manual_seed(16)
    _attn_check(4, T, 6, 64, True, Tk=Tk)


def test_attention_resident_head_bias_grad(cuda):
    """The resident backward's Σ_rows dQKV: Σ dV = Σ dO, Σ dK = 0, Σ dQ from the MFMA column sums of dS —
    against Σ_rows of the returned dQKV over 384 heads (several per workgroup)."""
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(15)
    B, H, D, T = 32, 12, 64, 197
    mod = torch.nn.Module()
    mod.pb = torch.nn.Parameter(torch.zeros(3 * H * D, device="cuda").bfloat16())
    flat = FlatParams(mod)
    flat.zero_grad()
    qkv = bf(B, T, 3, H, D).requires_grad_()
    o = ops.attention_packed(qkv, causal=False, producer_bias=mod.pb)
    o.backward(bf(B, T, H, D))
    assert mod.pb._rn_bias_done
    ref = qkv.grad.float().reshape(B * T, 3, H * D).sum(0)
    got = mod.pb.grad.float().reshape(3, H * D)
    assert rel_err(got[0], ref[0]) < 1e-2 and rel_err(got[2], ref[2]) < 1e-2
    assert got[1].abs().max() < 1e-2 * ref[0].abs().max()  # Σ dK: zero in exact arithmetic


@pytest.mark.parametrize("D", [32, 128])
def test_attention_packed_qkv_bias_grad_d(cuda, D):
    """The in-kernel Σ_rows dQKV partials at head sizes 32 / 128."""
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(12)
    B, H, T = 2, 2, 200
    mod = torch.nn.Module()
    mod.pb = torch.nn.Parameter(torch.zeros(3 * H * D, device="cuda").bfloat16())
    flat = FlatParams(mod)
    flat.zero_grad()
    qkv = bf(B, T, 3, H, D).requires_grad_()
    o = ops.attention_packed(qkv, causal=True, producer_bias=mod.pb)
    o.backward(bf(B, T, H, D))
    assert mod.pb._rn_bias_done
    assert rel_err(mod.pb.grad, qkv.grad.float().reshape(B * T, 3 * H * D).sum(0)) < 1e-2


@pytest.mark.parametrize("D", [4, 48, 80])
@pytest.mark.parametrize("causal,Tk", [(True, None), (False, None), (True, 56), (False, 33)])
def test_attention_generic_d(cuda, D, causal, Tk):
    """Odd head sizes: generic forward, dQ per query row + deterministic dK/dV per key row."""
    torch.manual_seed(9)
    _attn_check(2, 40, 3, D, causal, Tk=Tk)


@pytest.mark.parametrize("D", [48])
def test_attention_generic_d_bias(cuda, D):
    torch.manual_seed(11)
    bias = torch.randn(1, 40, 40, device="cuda") * 0.5
    _attn_check(2, 40, 3, D, False, bias=bias)


def test_attention_packed_grad(cuda):
    torch.manual_seed(10)
    B, T, H, D = 2, 128, 4, 64
    qkv = bf(B, T, 3, H, D).requires_grad_()
    o = ops.attention_packed(qkv, causal=True)
    go = bf(B, T, H, D)
    o.backward(go)
    qf = qkv.detach().float().requires_grad_()
    q, k, v = qf.unbind(2)
    of = ops.attention_reference(q, k, v, 0.125, True)
    of.backward(go.float())
    assert rel_err(o, of) < 2e-2 and rel_err(qkv.grad, qf.grad) < 4e-2


@pytest.mark.parametrize("causal,T", [(True, 256), (False, 200), (True, 320), (True, 200)])
def test_attention_packed_qkv_bias_grad(cuda, causal, T):
    """Σ_rows dQKV (the c_attn bias gradient) reduced inside the attention backward kernels
    (incl. an odd number of 64-row blocks: a partial last two-group block)."""
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(11)
    B, H, D = 3, 4, 64
    mod = torch.nn.Module()
    mod.pb = torch.nn.Parameter(torch.zeros(3 * H * D, device="cuda").bfloat16())
    flat = FlatParams(mod)
    flat.zero_grad()
    qkv = bf(B, T, 3, H, D).requires_grad_()
    g = bf(B, T, H, D)
    o = ops.attention_packed(qkv, causal=causal, producer_bias=mod.pb)
    o.backward(g)
    assert mod.pb._rn_bias_done
    ref = qkv.grad.float().reshape(B * T, 3 * H * D).sum(0)
    assert rel_err(mod.pb.grad, ref) < 1e-2


@pytest.mark.parametrize("D", [32, 64, 128])
def test_attention_dropout_unbiased(cuda, D):
    torch.manual_seed(11)
    B, T, H = 4, 128, 4
    q, k, v = bf(B, T, H, D), bf(B, T, H, D), bf(B, T, H, D)
    o0 = ops.attention(q, k, v, causal=True)
    outs = torch.stack([ops.attention(q, k, v, causal=True, dropout_p=0.1, training=True).float() for _ in range(16)])
    assert rel_err(outs.mean(0), o0) < 0.1
    assert not torch.equal(outs[0], outs[1])


# ----------------------------------------------------------------- misc kernels
def test_softmax_act_dropout(cuda):
    torch.manual_seed(12)
    x = bf(50, 300).requires_grad_()
    y = ops.softmax(x, scale=0.5)
    g = bf(50, 300)
    y.backward(g)
    xf = x.detach().float().requires_grad_()
    yf = torch.softmax(xf * 0.5, -1)
    yf.backward(g.float())
    assert rel_err(y, yf) < 1e-2 and rel_err(x.grad, xf.grad) < 2e-2
    z = bf(1000, 8).requires_grad_()
    for fn, rf in ((ops.gelu, lambda t: F.gelu(t, approximate="tanh")), (ops.relu, F.relu)):
        zz = z.detach().clone().requires_grad_()
        out = fn(zz)
        out.sum().backward()
        zf = z.detach().float().requires_grad_()
        rf(zf).sum().backward()
        assert rel_err(out, rf(z.float())) < 1e-2 and rel_err(zz.grad, zf.grad) < 2e-2
    d = ops.dropout(torch.ones(100000, device="cuda", dtype=torch.bfloat16), 0.25, True)
    keep = (d != 0).float().mean().item()
    assert abs(keep - 0.75) < 0.01 and abs(d.float().mean().item() - 1.0) < 0.02


@pytest.mark.parametrize("flat", [False, True])
def test_vit_join(cuda, flat):
    """ViT token join ([cls; patches] + pos, fused kernel both ways) against the fp32 reference, with
    the cls / pos gradients returned (autograd) or accumulated into the flat-buffer views."""
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(21)
    B, P, E = 5, 196, 768
    mod = torch.nn.Module()
    mod.cls = torch.nn.Parameter(bf(1, 1, E))
    mod.pos = torch.nn.Parameter(bf(1, P + 1, E))
    if flat:
        fp = FlatParams(mod)
        fp.zero_grad()
    patches = bf(B, P, E).requires_grad_()
    x = ops.vit_join(patches, mod.cls, mod.pos)
    g = bf(B, P + 1, E)
    x.backward(g)
    pf, cf, qf = [t.detach().float().requires_grad_() for t in (patches, mod.cls, mod.pos)]
    xr = torch.cat([cf.expand(B, -1, -1), pf], dim=1) + qf
    xr.backward(g.float())
    assert rel_err(x, xr) < 1e-2
    assert torch.equal(patches.grad, g[:, 1:])  # a copy: exact
    assert rel_err(mod.cls.grad, cf.grad) < 1e-2 and rel_err(mod.pos.grad, qf.grad) < 1e-2


def test_embedding(cuda):
    torch.manual_seed(13)
    V, E, B, T = 500, 128, 3, 40
    wte = bf(V, E).requires_grad_()
    wpe = bf(64, E).requires_grad_()
    ids = torch.randint(0, V, (B, T), device="cuda")
    ids[0, :5] = 7  # repeated ids exercise the scatter-add
    x = ops.embedding(ids, wte, wpe)
    g = bf(B, T, E)
    x.backward(g)
    wf, pf = wte.detach().float().requires_grad_(), wpe.detach().float().requires_grad_()
    xf = F.embedding(ids, wf) + pf[:T]
    xf.backward(g.float())
    assert rel_err(x, xf) < 1e-2 and rel_err(wte.grad, wf.grad) < 1e-2 and rel_err(wpe.grad, pf.grad) < 1e-2


def test_fused_adamw_matches_cpu(cuda):
    from replicann_amd.optim import FusedAdamW
    from replicann_amd.utils.flat import FlatParams

    torch.manual_seed(14)
    m_gpu = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 8)).cuda().to(torch.bfloat16)
    m_cpu = torch.nn.Sequential(torch.nn.Linear(64, 128), torch.nn.Linear(128, 8))
    m_cpu.load_state_dict({k: v.float().cpu() for k, v in m_gpu.state_dict().items()})
    fg, fc = FlatParams(m_gpu), FlatParams(m_cpu)
    og = FusedAdamW(fg, lr=1e-2, max_grad_norm=0.5, grad_scale=0.5)
    oc = FusedAdamW(fc, lr=1e-2, max_grad_norm=0.5, grad_scale=0.5)
    for _ in range(3):
        g = torch.randn(fc.numel)
        fg.grad.copy_(g.to(torch.bfloat16))
        fc.grad.copy_(g.to(torch.bfloat16).float())
        og.step()
        oc.step()
    assert rel_err(og.master.cpu(), oc.master) < 1e-4
    # non-finite gradient -> step skipped in-kernel
    before = og.master.clone()
    fg.grad[5] = float("nan")
    og.step()
    assert torch.equal(before, og.master) and og.norm_buf[1].item() == 1.0


def test_adamw_stochastic_rounding_unbiased(cuda):
    """The bf16 weight copy under stochastic rounding: a master value a quarter bf16 ulp above 1.0
    rounds up for ~1/4 of the elements (nearest rounding: never), deterministically per step."""
    from replicann_amd.optim import FusedAdamW
    from replicann_amd.utils.flat import FlatParams
    lin = torch.nn.Linear(1024, 1024, bias=False).cuda().to(torch.bfloat16)
    flat = FlatParams(lin)
    outs = []
    for sr in (True, True, False):
        opt = FusedAdamW(flat, lr=0.0, weight_decay=0.0, max_grad_norm=0.0, stochastic_round=sr)
        opt.master.fill_(1.0 + 2.0 ** -9)
        flat.grad.zero_()
        opt.step()
        outs.append(flat.data.float().clone())
    up = (outs[0] > 1.0).float().mean().item()
    assert 0.24 < up < 0.26, up
    assert abs(outs[0].mean().item() - (1.0 + 2.0 ** -9)) < 2e-4
    assert torch.equal(outs[0], outs[1])  # same step count -> same bits
    assert (outs[2] == 1.0).all()


# ----------------------------------------------------------------- conv / bn / pool
@pytest.mark.parametrize("cfg", [(3, 7, 2, 3), (16, 3, 1, 1), (16, 1, 2, 0), (8, 3, 2, 1), (3, 16, 16, 0)])
def test_conv2d(cuda, cfg):
    torch.manual_seed(15)
    C, Kk, S, P = cfg
    x = bf(2, 32, 32, C).requires_grad_()
    w = bf(24, Kk, Kk, C, scale=0.1).requires_grad_()
    b = bf(24).requires_grad_()
    y = ops.conv2d_nhwc(x, w, b, S, P)
    g = bf(*y.shape)
    y.backward(g)
    torch.cuda.synchronize()  # a fault in the native kernels surfaces here, not in the reference
    xf, wf, bf_ = [t.detach().float().cpu().requires_grad_() for t in (x, w, b)]
    yf = F.conv2d(xf.permute(0, 3, 1, 2), wf.permute(0, 3, 1, 2), bf_, S, P).permute(0, 2, 3, 1)
    yf.backward(g.float().cpu())
    assert rel_err(y, yf) < 1e-2
    for t, tf in ((x, xf), (w, wf), (b, bf_)):
        assert rel_err(t.grad, tf.grad) < 2e-2


def test_conv3x3_halo_dgrad_accumulate_and_fallback(cuda):
    """The halo-tile 3×3 kernel (conv3x3.hip) against the implicit GEMM it replaces, both vs fp32: forward, the
    data gradient with and without accumulation into an existing gradient (the residual-block join), and
    the statistics partials ([tiles][128], one row per tile of whole image rows)."""
    from replicann_amd import _ext
    torch.manual_seed(31)
    N, H = 3, 56
    x = bf(N, H, H, 64)
    w = bf(64, 3, 3, 64, scale=0.05)
    dy = bf(N, H, H, 64)
    base = bf(N, H, H, 64)
    o = _ext.ops()
    y, part = o.conv_fwd_implicit_stats(x, w, None, 1, 1)
    dx = o.conv_dgrad_implicit(dy, w, H, H, 1)
    acc = base.clone()
    o.conv_dgrad_implicit(dy, w, H, H, 1, acc, True)
    torch.cuda.synchronize()
    assert part.shape == (N * H // 8, 128)  # TR = 8 rows of 56: 448 pixels per tile (7 waves x 64)
    xf, wf, dyf = x.float().cpu(), w.float().cpu(), dy.float().cpu()
    yf = F.conv2d(xf.permute(0, 3, 1, 2), wf.permute(0, 3, 1, 2), None, 1, 1).permute(0, 2, 3, 1)
    dxf = torch.nn.grad.conv2d_input(xf.permute(0, 3, 1, 2).shape, wf.permute(0, 3, 1, 2), dyf.permute(0, 3, 1, 2),
                                     1, 1).permute(0, 2, 3, 1)
    assert rel_err(y, yf) < 1e-2 and rel_err(dx, dxf) < 1e-2
    assert rel_err(acc, base.float().cpu() + dxf) < 1e-2
    yb = y.float().cpu().reshape(-1, 64)
    assert rel_err(part.sum(0)[:64], yb.sum(0)) < 1e-3 and rel_err(part.sum(0)[64:], yb.square().sum(0)) < 1e-3
    # the implicit GEMM for the same shapes (REPLICANN_CONV3X3 read once per process: compare through the
    # generic geometry it also serves, a 64-channel 3x3 on 14 x 14 images, which the halo kernel does not take)
    assert o.conv_fwd_implicit_stats(bf(2, 14, 14, 64), w, None, 1, 1)[1].shape[0] == (2 * 14 * 14 + 255) // 256


@pytest.mark.parametrize("N,H,W,C,K,S,P", [(2, 224, 224, 3, 7, 2, 3), (3, 37, 29, 3, 7, 2, 3), (2, 20, 18, 5, 3, 1, 1),
                                           (1, 9, 2200, 3, 5, 3, 2)])
def test_im2col_small_channels(cuda, N, H, W, C, K, S, P):
    """The small-C im2col (LDS-staged rows; the last case exceeds the LDS budget and takes the
    per-chunk gather) is a pure copy: bitwise equal to F.unfold's layout ((kh, kw, c) per row)."""
    from replicann_amd import _ext
    torch.manual_seed(3)
    x = bf(N, H, W, C)
    OH, OW = (H + 2 * P - K) // S + 1, (W + 2 * P - K) // S + 1
    Kd = K * K * C
    Kp = (Kd + 7) // 8 * 8
    cols = _ext.ops().im2col(x.contiguous(), K, K, S, P, Kp)
    u = F.unfold(x.permute(0, 3, 1, 2).float(), K, padding=P, stride=S)  # [N, C*K*K (c, kh, kw)], L
    u = u.view(N, C, K, K, OH * OW).permute(0, 4, 2, 3, 1).reshape(N * OH * OW, Kd)
    ref = torch.zeros(N * OH * OW, Kp, device=x.device, dtype=torch.bfloat16)
    ref[:, :Kd] = u.to(torch.bfloat16)
    assert torch.equal(cols.view(N * OH * OW, Kp), ref)


@pytest.mark.parametrize("C,OC,Kk,S,P,HW", [(64, 64, 3, 1, 1, 14), (64, 128, 3, 2, 1, 15), (128, 64, 3, 1, 1, 9),
                                           (64, 128, 1, 2, 0, 16), (128, 128, 3, 1, 1, 7), (64, 64, 3, 1, 0, 10),
                                           (64, 256, 3, 1, 1, 8),
                                           # the halo-tile kernel (conv3x3.hip): 4 / 8 / 7 waves per tile
                                           (64, 64, 3, 1, 1, 16), (64, 64, 3, 1, 1, 32), (64, 64, 3, 1, 1, 56)])
def test_conv2d_implicit_gemm(cuda, C, OC, Kk, S, P, HW):
    """Implicit-GEMM path (channels % 64 == 0): fwd, dgrad (stride 1 implicit / stride 2 col2im), wgrad."""
    from replicann_amd.ops.conv import implicit_ok
    assert implicit_ok(C, OC, Kk, Kk, S, P)
    torch.manual_seed(17)
    x = bf(3, HW, HW, C).requires_grad_()
    w = bf(OC, Kk, Kk, C, scale=0.05).requires_grad_()
    y = ops.conv2d_nhwc(x, w, None, S, P)
    g = bf(*y.shape)
    y.backward(g)
    torch.cuda.synchronize()  # a fault in the native kernels surfaces here, not in the reference
    xf, wf = [t.detach().float().cpu().requires_grad_() for t in (x, w)]
    yf = F.conv2d(xf.permute(0, 3, 1, 2), wf.permute(0, 3, 1, 2), None, S, P).permute(0, 2, 3, 1)
    yf.backward(g.float().cpu())
    assert y.shape == yf.shape
    assert rel_err(y, yf) < 1e-2
    assert rel_err(x.grad, xf.grad) < 2e-2
    assert rel_err(w.grad, wf.grad) < 2e-2


@pytest.mark.parametrize("relu", [False, True])
def test_batchnorm(cuda, relu):
    torch.manual_seed(16)
    x = bf(4, 9, 9, 40).requires_grad_()
    w, b = bf(40).requires_grad_(), bf(40).requires_grad_()
    rm, rv = torch.zeros(40, device="cuda"), torch.ones(40, device="cuda")
    y = ops.batch_norm_nhwc(x, w, b, rm, rv, True, 0.1, 1e-5, relu)
    g = bf(*y.shape)
    y.backward(g)
    torch.cuda.synchronize()  # a fault in the native kernels surfaces here, not in the reference
    xf, wf, bf_ = [t.detach().float().cpu().requires_grad_() for t in (x, w, b)]
    rm2, rv2 = torch.zeros(40), torch.ones(40)
    yf = F.batch_norm(xf.permute(0, 3, 1, 2), rm2, rv2, wf, bf_, True, 0.1, 1e-5).permute(0, 2, 3, 1)
    if relu:
        yf = F.relu(yf)
    yf.backward(g.float().cpu())
    assert rel_err(y, yf) < 1e-2
    assert rel_err(rm, rm2) < 1e-3 and rel_err(rv, rv2) < 1e-3
    for t, tf in ((x, xf), (w, wf), (b, bf_)):
        assert rel_err(t.grad, tf.grad) < 3e-2


@pytest.mark.parametrize("C", [64, 512])
def test_batchnorm_residual_relu(cuda, C):
    """ResNet block output in one pass: y = relu(BN(x) + r); grads of x, w, b and the residual r
    (several row splits → the deterministic two-level statistics reduction)."""
    torch.manual_seed(18)
    N, H = 8, 28 if C == 64 else 7
    x, r = bf(N, H, H, C).requires_grad_(), bf(N, H, H, C).requires_grad_()
    w, b = bf(C).requires_grad_(), bf(C).requires_grad_()
    rm, rv = torch.zeros(C, device="cuda"), torch.ones(C, device="cuda")
    y = ops.batch_norm_nhwc(x, w, b, rm, rv, True, 0.1, 1e-5, True, residual=r)
    g = bf(*y.shape)
    y.backward(g)
    torch.cuda.synchronize()  # a fault in the native kernels surfaces here, not in the reference
    xf, rf, wf, bf_ = [t.detach().float().cpu().requires_grad_() for t in (x, r, w, b)]
    rm2, rv2 = torch.zeros(C), torch.ones(C)
    yf = F.relu(F.batch_norm(xf.permute(0, 3, 1, 2), rm2, rv2, wf, bf_, True, 0.1, 1e-5).permute(0, 2, 3, 1) + rf)
    yf.backward(g.float().cpu())
    assert rel_err(y, yf) < 1e-2
    assert rel_err(rm, rm2) < 1e-3 and rel_err(rv, rv2) < 1e-3
    for t, tf in ((x, xf), (r, rf), (w, wf), (b, bf_)):
        assert rel_err(t.grad, tf.grad) < 3e-2
    # eval mode (running statistics) with the residual
    ye = ops.batch_norm_nhwc(x.detach(), w.detach(), b.detach(), rm, rv, False, 0.1, 1e-5, True, residual=r.detach())
    yef = F.relu(F.batch_norm(xf.detach().permute(0, 3, 1, 2), rm.cpu(), rv.cpu(), wf.detach(), bf_.detach(), False, 0.1,
                              1e-5).permute(0, 2, 3, 1) + rf.detach())
    assert rel_err(ye, yef) < 1e-2


@pytest.mark.parametrize("C", [3, 16, 64])
def test_maxpool_ties(cuda, C):
    """Saved window indices: the gradient goes to the FIRST maximum of each window (ATen's rule),
    also with many ties (small-integer inputs) and on the scalar path (C % 8 != 0)."""
    torch.manual_seed(19)
    x = torch.randint(0, 3, (2, 15, 15, C), device="cuda").to(torch.bfloat16).requires_grad_()
    y = ops.maxpool_nhwc(x, 3, 2, 1)
    g = bf(*y.shape)
    y.backward(g)
    torch.cuda.synchronize()  # a fault in the native kernels surfaces here, not in the reference
    xf = x.detach().float().cpu().requires_grad_()
    yf = F.max_pool2d(xf.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    yf.backward(g.float().cpu())
    assert torch.equal(y.float().cpu(), yf)
    assert rel_err(x.grad, xf.grad) < 1e-2


def test_pools(cuda):
    torch.manual_seed(17)
    x = bf(2, 17, 17, 16).requires_grad_()
    y = ops.maxpool_nhwc(x, 3, 2, 1)
    g = bf(*y.shape)
    y.backward(g)
    torch.cuda.synchronize()
    xf = x.detach().float().cpu().requires_grad_()
    yf = F.max_pool2d(xf.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    yf.backward(g.float().cpu())
    assert rel_err(y, yf) < 1e-2 and rel_err(x.grad, xf.grad) < 1e-2
    x2 = bf(3, 7, 7, 32).requires_grad_()
    a = ops.avgpool_nhwc(x2)
    a.sum().backward()
    assert rel_err(a, x2.detach().float().mean((1, 2))) < 1e-2
    assert torch.allclose(x2.grad.float(), torch.full_like(x2.grad.float(), 1 / 49), rtol=1e-2)


# ----------------------------------------------------------------- fp8
def test_fp8_quantize_roundtrip(cuda):
    torch.manual_seed(20)
    x = bf(300, 264, scale=3.0)
    q, st = ops.quantize_fp8(x)
    # the scale: amax / 448 rounded UP to a power of two (the scaled MFMA's E8M0 operand, ops/fp8.py)
    from replicann_amd.ops.fp8 import pow2_ceil
    want = pow2_ceil(x.float().abs().max().cpu() / 448).item()
    assert q.dtype == torch.uint8 and st[0].item() == want
    y = ops.dequantize_fp8(q, st)
    assert rel_err(y, x) < 0.05
    # bit-compatible with torch's OCP e4m3fn
    ref = (x.float() / st[0]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    assert (q == ref).float().mean().item() > 0.99


@pytest.mark.parametrize("M,N,K", [(512, 384, 256), (300, 200, 528), (1024, 768, 1024)])
def test_gemm_fp8_matches_dequantized_reference(cuda, M, N, K):
    torch.manual_seed(21)
    a, b = bf(M, K), bf(N, K, scale=0.2)
    qa, sa = ops.quantize_fp8(a)
    qb, sb = ops.quantize_fp8(b)
    out = torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, None, None, 0, None)
    ref = ops.dequantize_fp8(qa, sa).float() @ ops.dequantize_fp8(qb, sb).float().t()
    assert rel_err(out, ref) < 1e-2  # exact products; only accumulation order + bf16 output differ
    assert rel_err(out, a.float() @ b.float().t()) < 0.08  # vs the unquantised product


@pytest.mark.parametrize("act", [0, 2, 5])
@pytest.mark.parametrize("M,N,K", [(1000, 1100, 1040), (4096, 3072, 1024)])
def test_gemm_fp8_persistent_vs_tile_kernel(cuda, monkeypatch, M, N, K, act):
    """The persistent 256x256 fp8 kernel (default) against the one-tile-per-block 256x192 one:
    same operands, same epilogue (bias + GELU / GELU with saved derivative); tails in M, N, K."""
    torch.manual_seed(23)
    a, b = bf(M, K), bf(N, K, scale=0.2)
    bias = bf(N, scale=0.1)
    qa, sa = ops.quantize_fp8(a)
    qb, sb = ops.quantize_fp8(b)
    outs = []
    for kern in ("9", "0"):
        monkeypatch.setenv("REPLICANN_FP8_GEMM", kern)
        pre = torch.empty(M, N, device="cuda", dtype=torch.bfloat16) if act == 5 else None
        o = torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, None, act, pre)
        outs.append((o, pre))
    torch.cuda.synchronize()
    ref = ops.dequantize_fp8(qa, sa).float() @ ops.dequantize_fp8(qb, sb).float().t() + bias.float()
    if act:
        ref = torch.nn.functional.gelu(ref, approximate="tanh")
    assert rel_err(outs[0][0], ref) < 1e-2
    assert rel_err(outs[0][0], outs[1][0]) < 5e-3
    if act == 5:
        assert rel_err(outs[0][1], outs[1][1]) < 5e-3


def test_layernorm_fused_fp8_output(cuda):
    """LayerNorm emitting its output in e4m3 for an fp8 consumer (delayed scaling): the bytes match
    a separate delayed quantisation of y with the same rolled scale, and the recorded amax is |y|max."""
    torch.manual_seed(24)
    M, E = 3000, 1024
    x, r = bf(M, E), bf(M, E)
    w, b = bf(E, scale=0.5) + 1.0, bf(E, scale=0.1)
    st_a = torch.tensor([0.0, 3.0, 0.0, 0.0], device="cuda")  # previous amax 3 -> scale 2*3/448
    st_b = st_a.clone()
    y, h, mean, rstd, q8 = torch.ops.replicann.layernorm_fwd_q8(x, r, w, b, 1e-5, st_a)
    y_ref, h_ref, _, _ = torch.ops.replicann.layernorm_fwd(x, r, w, b, 1e-5)
    q_ref = torch.ops.replicann.fp8_quantize_delayed(y_ref, st_b)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref) and torch.equal(h, h_ref)
    from replicann_amd.ops.fp8 import pow2_ceil
    assert st_a[0].item() == pow2_ceil(2 * 3.0 / 448).item() and st_a[2].item() == 3.0
    assert st_a[1].item() == y.float().abs().max().item()
    assert torch.equal(q8, q_ref)


@pytest.mark.parametrize("act", [2, 5])
def test_gemm_fp8_with_e4m3_output(cuda, act):
    """The fp8 GEMM whose GELU output also comes out in e4m3 for the next fp8 GEMM: same bf16
    output as the plain call, e4m3 bytes equal to a separate delayed quantisation with the same
    rolled scale, amax recorded."""
    torch.manual_seed(25)
    M, N, K = 1500, 4096, 1024
    a, b, bias = bf(M, K), bf(N, K, scale=0.05), bf(N, scale=0.1)
    qa, sa = ops.quantize_fp8(a)
    qb, sb = ops.quantize_fp8(b)
    pre1 = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    pre2 = torch.empty_like(pre1)
    st = torch.tensor([0.0, 2.0, 0.0, 0.0], device="cuda")
    st_ref = st.clone()
    y, q = torch.ops.replicann.gemm_fp8_q8(qa, qb, sa, sb, bias, act, pre1, st)
    y_ref = torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, None, act, pre2)
    q_ref = torch.ops.replicann.fp8_quantize_delayed(y_ref, st_ref)
    torch.cuda.synchronize()
    assert torch.equal(y, y_ref) and torch.equal(pre1, pre2)
    assert torch.equal(q, q_ref)
    assert st[1].item() == y.float().abs().max().item() and st[2].item() == 2.0


def test_fp8_weight_cache_matches_per_call_quantisation(cuda):
    """Fp8WeightCache: after an optimizer step the cached e4m3 weight equals a delayed quantisation
    of the updated bf16 weight with the same rolled scale; a weight changed outside the optimizer
    is not served from the cache."""
    from replicann_amd.ops.fp8 import Fp8State, attach_weight_cache
    from replicann_amd.optim import FusedAdamW
    from replicann_amd.utils.flat import FlatParams

    torch.manual_seed(26)

    class L(torch.nn.Module):
        def __init__(self, n, k):
            super().__init__()
            self.weight = torch.nn.Parameter(torch.randn(n, k) * 0.05)
            self.fp8_state = Fp8State()

    m = torch.nn.Sequential(L(384, 256), L(1000, 384)).cuda()
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    flat = FlatParams(m)
    opt = FusedAdamW(flat, lr=1e-2)
    cache = attach_weight_cache(m, flat, opt)
    assert cache is not None and len(cache.entries) == 2
    for layer in m:  # first use: current scaling (seeds the amax)
        layer.fp8_state.quant(layer.weight, 1)
    flat.grad.normal_()
    opt.step()
    assert cache.refreshes == 1
    for layer in m:
        st = layer.fp8_state
        q, s_ = st.quant(layer.weight, 1)
        assert q.data_ptr() >= cache.qbuf.data_ptr()  # served from the cache
        ref_state = st.t[1].clone()
        ref_state[1] = ref_state[2]  # replay the roll from the amax the cache's roll consumed
        q_ref = torch.ops.replicann.fp8_quantize_delayed(layer.weight.contiguous(), ref_state)
        torch.cuda.synchronize()
        assert torch.equal(q, q_ref)
        assert st.t[1][1].item() == layer.weight.float().abs().max().item()
    with torch.no_grad():
        m[0].weight.mul_(2.0)  # outside the optimizer: version changes, cache not used
    q2, _ = m[0].fp8_state.quant(m[0].weight, 1)
    assert not (cache.qbuf.data_ptr() <= q2.data_ptr() < cache.qbuf.data_ptr() + cache.qbuf.numel())


def test_linear_fp8_autograd(cuda):
    torch.manual_seed(22)
    x = bf(4, 64, 256).requires_grad_()
    w = bf(512, 256, scale=0.05).requires_grad_()
    b = bf(512).requires_grad_()
    r = bf(4, 64, 512)
    y = ops.linear_fp8(x, w, b, act="gelu", residual=r)
    yref = ops.linear(x.detach(), w.detach(), b.detach(), act="gelu", residual=r)
    assert rel_err(y, yref) < 0.05
    y.float().pow(2).mean().backward()
    assert all(torch.isfinite(t.grad.float()).all() for t in (x, w, b))


def test_fp8_delayed_scaling(cuda):
    """One-pass delayed scaling: scale = 2·amax(previous quantisation)/448 rounded up to a power of two, the pass records the new
    amax; values beyond the headroom saturate at ±448·scale."""
    torch.manual_seed(23)
    st = ops.Fp8State()
    x0 = bf(256, 512, scale=2.0)
    q0, s0 = st.quant(x0, 0)  # first call: current scaling
    amax0 = x0.float().abs().max().item()
    assert abs(s0[1].item() - amax0) < 1e-3 * amax0
    x1 = bf(256, 512, scale=2.5)
    q1, s1 = st.quant(x1, 0)  # delayed: scale from amax0
    from replicann_amd.ops.fp8 import pow2_ceil
    assert s1[0].item() == pow2_ceil(torch.tensor(2 * amax0, dtype=torch.float32) / 448).item()
    assert abs(s1[1].item() - x1.float().abs().max().item()) < 1e-3 * amax0  # new amax recorded
    y1 = ops.dequantize_fp8(q1, s1)
    assert rel_err(y1, x1) < 0.06
    x2 = bf(256, 512, scale=40.0)  # far beyond the headroom: saturates, stays finite
    q2, s2 = st.quant(x2, 0)
    y2 = ops.dequantize_fp8(q2, s2)
    assert torch.isfinite(y2.float()).all() and y2.float().abs().max().item() <= 448 * s2[0].item() * 1.001


def test_mlp_fp8_matches_bf16(cuda):
    """Fused MLP node with e4m3 forward GEMMs (delayed scaling after the first call) vs bf16."""
    torch.manual_seed(24)
    x = bf(2, 128, 256)
    w1, b1 = bf(1024, 256, scale=0.05), bf(1024, scale=0.1)
    w2, b2 = bf(256, 1024, scale=0.05), bf(256, scale=0.1)
    r = bf(2, 128, 256)
    states = (ops.Fp8State(), ops.Fp8State())
    ref = ops.mlp(x, w1, b1, w2, b2, "gelu", residual=r)
    for _ in range(3):  # first call current scaling, then delayed
        xs = x.clone().requires_grad_()
        y = ops.mlp(xs, w1, b1, w2, b2, "gelu", residual=r, fp8=states)
        assert rel_err(y, ref) < 0.05
    y.float().pow(2).mean().backward()
    assert torch.isfinite(xs.grad.float()).all()


def test_conv_bn_direct_grad_accumulation(cuda):
    """Implicit-conv weight and BatchNorm weight/bias gradients added by the kernels straight into
    the flat gradient buffer (no AccumulateGrad) equal autograd's, accumulated over two backwards."""
    from replicann_amd.models.resnet import BasicBlock
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(23)
    ref, blk = BasicBlock(64, 128, 2).cuda(), BasicBlock(64, 128, 2).cuda()
    for m in (ref, blk):
        for p in m.parameters():  # bf16 parameters, fp32 BN running statistics (as the Trainer does)
            p.data = p.data.bfloat16()
    blk.load_state_dict(ref.state_dict())
    flat = FlatParams(blk, dtype=torch.bfloat16, device="cuda", grad_dtype=torch.bfloat16)
    seen = []
    flat.ready_hooks.append(lambda p: seen.append(id(p)))
    xs = [bf(4, 16, 16, 64) for _ in range(2)]
    for x in xs:
        ref(x).float().square().mean().backward()
        blk(x).float().square().mean().backward()
    n_direct = 0
    for (name, p), (_, q) in zip(ref.named_parameters(), blk.named_parameters()):
        assert rel_err(q.grad, p.grad) < 2e-2, name
        n_direct += id(q) in seen
    assert n_direct >= 5  # conv1/conv2/shortcut weights + BN params took the direct path


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("N,HW,C,OC", [(3, 15, 64, 128), (2, 9, 128, 64), (3, 16, 64, 64), (2, 56, 64, 64)])
def test_conv_bn_fused_statistics(cuda, monkeypatch, fused, N, HW, C, OC):
    """Implicit-conv forward emitting the BatchNorm batch statistics from its GEMM epilogue
    (ops.conv.BN_FUSED_STATS, M % 256 != 0 here) vs the BN's own statistics pass, both
    against fp32 conv + batch_norm (outputs, running statistics, input / weight gradients)."""
    from replicann_amd.ops import conv as conv_mod
    monkeypatch.setattr(conv_mod, "BN_FUSED_STATS", fused == "1")
    torch.manual_seed(29)
    x = bf(N, HW, HW, C).requires_grad_()
    w = bf(OC, 3, 3, C, scale=0.05).requires_grad_()
    g = (torch.rand(OC, device="cuda") + 0.5).bfloat16().requires_grad_()
    b = bf(OC, scale=0.1).requires_grad_()
    rm, rv = torch.zeros(OC, device="cuda"), torch.ones(OC, device="cuda")
    yc = ops.conv2d_nhwc(x, w, None, 1, 1)
    assert (getattr(yc, "_rn_bn_partials", None) is not None) == (fused == "1")
    y = ops.batch_norm_nhwc(yc, g, b, rm, rv, True, 0.1, 1e-5, relu=True)
    go = bf(*y.shape)
    y.backward(go)
    torch.cuda.synchronize()  # a fault in the native kernels surfaces here, not in the reference
    xf, wf, gf, bf_ = [t.detach().float().cpu().requires_grad_() for t in (x, w, g, b)]
    rmf, rvf = torch.zeros(OC), torch.ones(OC)
    ycf = F.conv2d(xf.permute(0, 3, 1, 2), wf.permute(0, 3, 1, 2), None, 1, 1)
    yf = F.relu(F.batch_norm(ycf, rmf, rvf, gf, bf_, True, 0.1, 1e-5)).permute(0, 2, 3, 1)
    yf.backward(go.float().cpu())
    assert rel_err(y, yf) < 2e-2
    assert rel_err(rm, rmf) < 2e-2 and rel_err(rv, rvf) < 2e-2
    for t, tf in ((x, xf), (w, wf), (g, gf), (b, bf_)):
        assert rel_err(t.grad, tf.grad) < 3e-2


def test_dropout_device_seeds_graph_capture(cuda):
    """Device-drawn dropout seeds (ops/rng.py): a captured hipGraph of a train-mode reference
    TransformerDecoder step (head dropout 0.1 + block dropout) replays with FRESH masks every replay,
    and replays reproduce eager steps started from the same device RNG state bit for bit."""
    import replicann_amd.arch.transformer as T
    from replicann_amd.ops import rng
    torch.manual_seed(0)
    m = T.TransformerDecoder(4, 256, context_size=64, p_dropout=0.1).cuda().to(torch.bfloat16).train()
    x = bf(2, 64, 256)

    def step():
        return m(x).float().sum()

    _ = step()  # warm-up (autotuner, lazy allocations) outside the capture
    torch.cuda.synchronize()
    st0 = rng.state_dict()
    eager = [step().item() for _ in range(3)]
    rng.load_state_dict(st0)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()  # side-stream warm-up required before capture
    torch.cuda.current_stream().wait_stream(s)
    rng.load_state_dict(st0)
    with torch.cuda.graph(g):
        out = step()
    rng.load_state_dict(st0)  # the capture did not run the kernels, but reset anyway
    replays = []
    for _ in range(3):
        g.replay()
        replays.append(out.item())
    assert len(set(replays)) == 3, "each replay must draw new dropout masks"
    assert replays == eager, (replays, eager)


@pytest.mark.parametrize("jump", [12.0, 6.0, 30.0])
def test_attention_fwd32_deferred_rescale_forced(cuda, jump):
    """The causal D = 64 forward (attn_fwd32_k) rescales O and the row sum only when a row's tile max exceeds
    the running max by more than 2^8 (T13): a branch bounded random data rarely takes.  Force it (MI355X guide
    rule 26): for chosen query rows one key of a LATER tile is a spike along that query (its score jumps by
    `jump` log2 units over everything before it: 12 and 30 take the rescale, 6 stays under the threshold with
    P up to 2^6), and check O, the backward's gradients and the base-2 lse the backward reads against a float64
    reference over the full tensors."""
    torch.manual_seed(21)
    B, T, H, D = 1, 512, 2, 64
    q = torch.randn(B, T, H, D, device="cuda")
    k = torch.randn(B, T, H, D, device="cuda") * 0.3
    v = torch.randn(B, T, H, D, device="cuda")
    sl2 = 0.125 * 1.4426950408889634
    for hh in range(H):
        for i in range(200, T, 7):            # query rows
            j = (i // 64 - 1) * 64 + (i % 53)  # a key in the tile before the diagonal tile (visible: j < i)
            qi = q[0, i, hh]
            k[0, j, hh] = qi / qi.dot(qi) * (jump / sl2)  # q_i · k_j = jump / sl2  →  jump in log2 units
    q, k, v = q.bfloat16(), k.bfloat16(), v.bfloat16()
    qg, kg, vg = [t.clone().requires_grad_() for t in (q, k, v)]
    o = ops.attention(qg, kg, vg, scale=0.125, causal=True)
    go = torch.randn(B, T, H, D, device="cuda").bfloat16()
    o.backward(go)
    qd, kd, vd = [t.detach().double().requires_grad_() for t in (q, k, v)]
    s = torch.einsum("bqhd,bkhd->bhqk", qd, kd) * 0.125
    s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device="cuda"), 1), float("-inf"))
    od = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), vd)
    od.backward(go.double())
    assert rel_err(o, od) < 1e-2
    for t, td in ((qg, qd), (kg, kd), (vg, vd)):
        assert rel_err(t.grad, td.grad) < 2e-2
