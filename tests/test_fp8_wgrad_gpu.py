"""fp8 weight and data gradients (csrc/include/gemm_pk.h, MN-contiguous fp8 operands read by the
transposing ds_read_b64_tr_b8; csrc/kernels/fp8.hip rn_gemm_fp8_wgrad / rn_gemm_fp8_dgrad):
dW = dYᵀ·X with dY in e5m2 and X in e4m3, both as the step produced them (token-major), fp32
split-K slabs + fixed-order reduction; dX = dY·W with the forward's e4m3 weight [out][in] read
transposed (B MN-contiguous, A K-contiguous), bf16 out.

Checked against fp32 math on the DEQUANTISED operands (so only the GEMM is under test, not the
quantisation), for GPT-2-medium shapes, ragged tiles (widths multiples of 16, not of 256), both
output dtypes, accumulate, and bitwise run-to-run determinism; and the e5m2 quantiser against
torch's float8_e5m2 cast."""

import pytest
import torch

from replicann_amd import ops

pytestmark = pytest.mark.gpu

SHAPES = [  # (tokens K, M = out features, N = in features)
    (16384, 3072, 1024),   # GPT-2-medium c_attn (K = 16 sequences)
    (8192, 4096, 1024),    # c_fc
    (8192, 1024, 4096),    # mlp c_proj
    (1024, 400, 272),      # ragged M / N
    (128, 256, 256),       # one K-tile
]


def _q(dy, x):
    gs = torch.zeros(4, device=dy.device)
    dy8 = torch.ops.replicann.bf8_quantize(dy, gs, False)
    x8, xs = ops.quantize_fp8(x)
    return dy8, gs, x8, xs


@pytest.mark.parametrize("shape", SHAPES, ids=lambda s: "x".join(map(str, s)))
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16], ids=["f32", "bf16"])
def test_fp8_wgrad_vs_fp32_on_dequantised(cuda, shape, out_dtype):
    K, M, N = shape
    g = torch.Generator(device="cpu").manual_seed(5)
    dy = (torch.randn(K, M, generator=g) * 0.01).to(cuda, torch.bfloat16)
    x = torch.randn(K, N, generator=g).to(cuda, torch.bfloat16)
    dy8, gs, x8, xs = _q(dy, x)
    # dequantised in fp32 (the bf16 dequantisers round the products to 8 significant bits)
    ref = (dy8.view(torch.float8_e5m2).float() * gs[0]).t() @ (x8.view(torch.float8_e4m3fn).float() * xs[0])
    out = torch.zeros(M, N, device=cuda, dtype=out_dtype)
    torch.ops.replicann.gemm_fp8_wgrad(dy8, x8, gs, xs, out, False, True)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < (2e-5 if out_dtype == torch.float32 else 4e-3), err
    # accumulate into an existing gradient
    base = torch.randn(M, N, generator=g).to(cuda, out_dtype)
    acc = base.clone()
    torch.ops.replicann.gemm_fp8_wgrad(dy8, x8, gs, xs, acc, True, True)
    err2 = ((acc.float() - (base.float() + ref)).norm() / (base.float() + ref).norm()).item()
    assert err2 < (2e-5 if out_dtype == torch.float32 else 4e-3), err2
    # deterministic (fixed slab order)
    out2 = torch.zeros_like(out)
    torch.ops.replicann.gemm_fp8_wgrad(dy8, x8, gs, xs, out2, False, True)
    assert torch.equal(out, out2)


DGRAD_SHAPES = [  # (tokens M, K = out features, N = in features)
    (16384, 3072, 1024),   # GPT-2-medium c_attn dgrad
    (16384, 4096, 1024),   # c_fc dgrad
    (16384, 1024, 1024),   # attention c_proj dgrad
    (1000, 400, 272),      # ragged M / K (not a K-tile multiple) / N
    (64, 128, 16),         # one K-tile, one narrow column group
    (1000, 512, 272),      # the one-wave-per-SIMD kernel (K % 128 == 0) with ragged rows and a 16-column tail
    (300, 256, 48),        # its shortest K (2 K-tiles), one partial column tile
]


@pytest.mark.parametrize("shape", DGRAD_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_fp8_dgrad_vs_fp32_on_dequantised(cuda, shape):
    M, K, N = shape
    g = torch.Generator(device="cpu").manual_seed(6)
    dy = (torch.randn(M, K, generator=g) * 0.01).to(cuda, torch.bfloat16)
    w = (torch.randn(K, N, generator=g) * 0.02).to(cuda, torch.bfloat16)
    gs = torch.zeros(4, device=cuda)
    dy8 = torch.ops.replicann.bf8_quantize(dy, gs, False)
    w8, ws = ops.quantize_fp8(w)
    ref = (dy8.view(torch.float8_e5m2).float() * gs[0]) @ (w8.view(torch.float8_e4m3fn).float() * ws[0])
    out = ops.fp8_dgrad((dy8, gs), w8, ws)
    assert out.shape == (M, N) and out.dtype == torch.bfloat16
    err = ((out.float() - ref).norm() / ref.norm()).item()
    assert err < 4e-3, err
    # e4m3 A operand too (the kernel's other A format)
    x8, xs = ops.quantize_fp8(dy)
    ref2 = (x8.view(torch.float8_e4m3fn).float() * xs[0]) @ (w8.view(torch.float8_e4m3fn).float() * ws[0])
    out2 = torch.ops.replicann.gemm_fp8_dgrad(x8, w8, xs, ws, False)
    assert ((out2.float() - ref2).norm() / ref2.norm()).item() < 4e-3
    assert torch.equal(out, ops.fp8_dgrad((dy8, gs), w8, ws))


def test_bf8_quantiser_matches_torch_cast(cuda):
    x = torch.randn(4096, 256, device=cuda).bfloat16() * 3
    st = torch.zeros(4, device=cuda)
    q = torch.ops.replicann.bf8_quantize(x, st, False)
    scale = float(st[0])
    from replicann_amd.ops.fp8 import pow2_ceil  # every fp8 / bf8 scale is a power of two
    amax = x.float().abs().max().cpu()
    assert scale == pow2_ceil(amax / 57344.0).item()
    ref = (x.float() / scale).to(torch.float8_e5m2).view(torch.uint8)
    assert (q != ref).float().mean().item() < 1e-3  # round-to-nearest-even on both sides
    # delayed pass: scale from the recorded amax (x2 headroom), new amax recorded
    q2 = torch.ops.replicann.bf8_quantize(x * 0.5, st, True)
    assert float(st[0]) == pow2_ceil(2 * amax / 57344.0).item()
    assert abs(float(st[1]) - 0.5 * float(x.float().abs().max())) < 1e-3 * float(st[1])
    deq = ops.dequantize_bf8(q2, st).float()
    assert ((deq - x.float() * 0.5).norm() / (x.float() * 0.5).norm()) < 0.1


@pytest.mark.parametrize("dgrad", [False, True], ids=["wgrad", "wgrad+dgrad"])
def test_fp8_model_wgrad_tracks_bf16_wgrad(cuda, dgrad):
    """GPT-2 (tiny, fp8 layers) one backward: fp8 weight (and data) gradients within fp8 tolerance
    of the bf16 backward on the same forward — every parameter when the data gradients are fp8 too
    (everything upstream of an fp8 dgrad sees its error)."""
    import replicann_amd as R
    from replicann_amd.ops.fp8 import fp8_states

    ids = torch.randint(0, 1000, (8, 128), device=cuda, generator=torch.Generator(device=cuda).manual_seed(2))
    grads = {}
    for wg in (False, True):
        torch.manual_seed(0)
        m = R.GPT2(R.GPT2Config.tiny(fp8=True)).to(cuda)
        for p in m.parameters():
            p.data = p.data.bfloat16()
        for st in fp8_states(m):
            st.wgrad = wg
            st.dgrad = wg and dgrad
        m(ids, ids).backward()
        grads[wg] = {n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None}
    names = [n for n in grads[True] if n.endswith(("c_attn.weight", "c_fc.weight", "mlp.c_proj.weight"))]
    if dgrad:
        names = list(grads[True])
    assert names
    for n in names:
        a, b = grads[True][n], grads[False][n]
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)) < (0.12 if dgrad else 0.08), n


@pytest.mark.parametrize("shape", [(16384, 3072, 1024), (1000, 512, 272), (300, 256, 48)], ids=lambda s: "x".join(map(str, s)))
def test_fp8_dgrad_w1_matches_older_kernel(cuda, shape, monkeypatch):
    """The one-wave-per-SIMD fp8 data gradient (default for K % 128 == 0: tr_b8 reads of W as stored,
    e5m2 A through the scaled MFMA's format operand) against the older persistent kernel on the same
    operands: the same exact products, only accumulation order and the bf16 rounding differ."""
    M, K, N = shape
    g = torch.Generator(device="cpu").manual_seed(9)
    dy = (torch.randn(M, K, generator=g) * 0.01).to(cuda, torch.bfloat16)
    w = (torch.randn(K, N, generator=g) * 0.02).to(cuda, torch.bfloat16)
    gs = torch.zeros(4, device=cuda)
    dy8 = torch.ops.replicann.bf8_quantize(dy, gs, False)
    w8, ws = ops.quantize_fp8(w)
    monkeypatch.delenv("REPLICANN_FP8_GEMM", raising=False)
    new = torch.ops.replicann.gemm_fp8_dgrad(dy8, w8, gs, ws, True)
    monkeypatch.setenv("REPLICANN_FP8_GEMM", "9")
    old = torch.ops.replicann.gemm_fp8_dgrad(dy8, w8, gs, ws, True)
    assert ((new.float() - old.float()).norm() / old.float().norm()).item() < 4e-3
    monkeypatch.delenv("REPLICANN_FP8_GEMM", raising=False)  # bitwise repeatable
    assert torch.equal(new, torch.ops.replicann.gemm_fp8_dgrad(dy8, w8, gs, ws, True))


@pytest.mark.parametrize("shape", [(16384, 3072, 1024), (1024, 400, 272), (65536, 1024, 1024)],
                         ids=lambda s: "x".join(map(str, s)))
def test_fp8_wgrad_w1_matches_older_kernel(cuda, shape, monkeypatch):
    """The one-wave-per-SIMD fp8 weight gradient (default: both operands MN-contiguous through tr_b8 reads,
    split-K over an exact division of the K-tiles, fp32 slabs, the fixed-order slab sum) against the older
    persistent kernel on the same operands, fp32 output: equal up to fp32 summation order."""
    K, M, N = shape
    g = torch.Generator(device="cpu").manual_seed(12)
    dy = (torch.randn(K, M, generator=g) * 0.01).to(cuda, torch.bfloat16)
    x = torch.randn(K, N, generator=g).to(cuda, torch.bfloat16)
    dy8, gs, x8, xs = _q(dy, x)
    monkeypatch.delenv("REPLICANN_FP8_GEMM", raising=False)
    new = torch.zeros(M, N, device=cuda, dtype=torch.float32)
    torch.ops.replicann.gemm_fp8_wgrad(dy8, x8, gs, xs, new, False, True)
    monkeypatch.setenv("REPLICANN_FP8_GEMM", "9")
    old = torch.zeros(M, N, device=cuda, dtype=torch.float32)
    torch.ops.replicann.gemm_fp8_wgrad(dy8, x8, gs, xs, old, False, True)
    assert ((new - old).norm() / old.norm()).item() < 2e-5
    monkeypatch.delenv("REPLICANN_FP8_GEMM", raising=False)
    again = torch.zeros_like(new)
    torch.ops.replicann.gemm_fp8_wgrad(dy8, x8, gs, xs, again, False, True)
    assert torch.equal(new, again)


@pytest.mark.parametrize("delayed", [False, True])
def test_act_mul_bf8_vs_torch(cuda, delayed):
    """dH = dU ⊙ d straight to e5m2 (the fused GELU backward of the fp8 MLP): the dequantised output
    against the fp32 product at e5m2 precision, the bias-gradient column sums against fp32, and the
    slot's scale / amax bookkeeping as bf8_quantize's."""
    g = torch.Generator(device="cpu").manual_seed(13)
    M, N = 3000, 4096
    du = (torch.randn(M, N, generator=g) * 0.01).to(cuda, torch.bfloat16)
    d = torch.rand(M, N, generator=g).to(cuda, torch.bfloat16) * 1.1
    ref = du.float() * d.float()
    st = torch.zeros(4, device=cuda)
    if delayed:  # a previous pass recorded amax = 2 x this one's
        st[1] = 2 * ref.abs().max()
    bg = torch.zeros(N, device=cuda, dtype=torch.bfloat16)
    q = torch.ops.replicann.act_mul_bf8(du, d, st, delayed, bg)
    from replicann_amd.ops.fp8 import pow2_ceil
    amax = ref.abs().max()
    want = pow2_ceil((2 * 2 * amax if delayed else amax).cpu() / 57344.0).item()
    assert st[0].item() == want
    assert abs(st[1].item() - amax.item()) <= 1e-6 * amax.item()
    deq = q.view(torch.float8_e5m2).float() * st[0]
    assert ((deq - ref).norm() / ref.norm()).item() < 0.1
    colsum = ref.sum(0)
    assert ((bg.float() - colsum).norm() / colsum.norm()).item() < 1e-2


def test_gelu_q8_and_act_mul_from_h(cuda):
    """The all-fp8 MLP's split activation: e4m3(gelu(h)) with a delayed scale (rolled, amax recorded) and
    the backward's dH = dU ⊙ gelu'(h) re-derived from h, against torch."""
    from replicann_amd.ops.linear import ACT_GELU, _act_grad_ref
    g = torch.Generator(device="cpu").manual_seed(14)
    M, N = 2000, 1024
    h = (torch.randn(M, N, generator=g) * 2).to(cuda, torch.bfloat16)
    u = torch.nn.functional.gelu(h.float(), approximate="tanh").bfloat16().float()
    st = torch.tensor([0.0, 3.0, 0.0, 0.0], device=cuda)  # previous amax 3
    q = torch.ops.replicann.gelu_q8(h, st)
    from replicann_amd.ops.fp8 import pow2_ceil
    assert st[0].item() == pow2_ceil(torch.tensor(2 * 3.0 / 448)).item() and st[2].item() == 3.0
    assert abs(st[1].item() - u.abs().max().item()) <= 1e-3 * u.abs().max().item()
    deq = q.view(torch.float8_e4m3fn).float() * st[0]
    assert ((deq - u).norm() / u.norm()).item() < 0.05
    du = (torch.randn(M, N, generator=g) * 0.01).to(cuda, torch.bfloat16)
    gs = torch.zeros(4, device=cuda)
    bg = torch.zeros(N, device=cuda, dtype=torch.bfloat16)
    q2 = torch.ops.replicann.act_mul_bf8(du, h, gs, False, bg, True)
    ref = _act_grad_ref(du.float(), h, ACT_GELU).float()
    deq2 = q2.view(torch.float8_e5m2).float() * gs[0]
    assert ((deq2 - ref).norm() / ref.norm()).item() < 0.1
    assert ((bg.float() - ref.sum(0)).norm() / ref.sum(0).norm()).item() < 1e-2


def test_fp8_mlp_keep_h_tracks_unfused(cuda, monkeypatch):
    """GPT-2 (tiny, fp8): the all-fp8 MLP path (h kept, gelu(h) quantised in one pass, fused GELU backward)
    trains like the REPLICANN_FP8_MLP_FUSE=0 path (bf16 c_proj dgrad, gelu'(h) saved by the epilogue) within
    fp8 noise, with finite gradients everywhere."""
    import replicann_amd as R
    import replicann_amd.ops.fp8 as F
    from replicann_amd.utils.flat import FlatParams
    from replicann_amd.optim import FusedAdamW

    def run(fuse):
        monkeypatch.setattr(F, "FP8_MLP_FUSE", fuse)
        torch.manual_seed(0)
        m = R.GPT2(R.GPT2Config.tiny(fp8=True)).to(cuda)
        for p in m.parameters():
            p.data = p.data.to(torch.bfloat16)
        for st in F.fp8_states(m):
            st.wgrad = st.dgrad = True
        flat = FlatParams(m)
        opt = FusedAdamW(flat, lr=1e-3)
        gen = torch.Generator(device=cuda).manual_seed(7)
        losses = []
        for _ in range(4):
            ids = torch.randint(0, 1000, (4, 129), device=cuda, generator=gen)
            opt.zero_grad()
            loss = m(ids[:, :-1], ids[:, 1:])
            loss.backward()
            assert torch.isfinite(flat.grad.float()).all()
            opt.step()
            losses.append(float(loss))
        return losses

    a, b = run(True), run(False)
    for x, y in zip(a, b):
        assert abs(x - y) <= 0.02 * abs(y), (a, b)


def test_fp8_mlp_ragged_tokens_gradients_match_unfused(cuda, monkeypatch):
    """with B·T % 128 != 0 the fp8 weight gradients fall back to bf16, so the MLP must not
    keep h (the bf16 fallback would take c_proj's dW from h instead of gelu(h) and c_fc's from dU instead of
    dH).  Every step's flat gradient of the fused-default model must match the FP8_MLP_FUSE=False model's."""
    import replicann_amd as R
    import replicann_amd.ops.fp8 as F
    from replicann_amd.optim import FusedAdamW
    from replicann_amd.utils.flat import FlatParams

    def run(fuse):
        monkeypatch.setattr(F, "FP8_MLP_FUSE", fuse)
        torch.manual_seed(0)
        m = R.GPT2(R.GPT2Config.tiny(fp8=True)).to(cuda)
        for p in m.parameters():
            p.data = p.data.to(torch.bfloat16)
        for st in F.fp8_states(m):
            st.wgrad = st.dgrad = True
        flat = FlatParams(m)
        opt = FusedAdamW(flat, lr=1e-3)
        gen = torch.Generator(device=cuda).manual_seed(11)
        grads = []
        for _ in range(4):
            ids = torch.randint(0, 1000, (3, 101), device=cuda, generator=gen)  # 300 tokens: % 128 != 0
            opt.zero_grad()
            m(ids[:, :-1], ids[:, 1:]).backward()
            g = flat.grad.float().clone()
            assert torch.isfinite(g).all()
            grads.append(g)
            opt.step()
        return grads

    ga, gb = run(True), run(False)
    for a, b in zip(ga, gb):
        assert ((a - b).norm() / b.norm()).item() < 0.02


def test_fp8_attention_q8_dqkv_tracks_quantise_pass(cuda, monkeypatch):
    """GPT-2 (tiny, fp8, fp8 backward): the attention backward's own e5m2 dQKV (no bf16 dQKV when c_attn
    takes both gradients in fp8) trains like the path that quantises a bf16 dQKV (REPLICANN_FP8_ATTN_Q8=0)."""
    import importlib

    import replicann_amd as R
    import replicann_amd.ops.fp8 as F
    A = importlib.import_module("replicann_amd.ops.attention")  # (ops.attention is also the function)
    from replicann_amd.optim import FusedAdamW
    from replicann_amd.utils.flat import FlatParams

    def run(q8):
        monkeypatch.setattr(A, "ATTN_Q8", q8)
        torch.manual_seed(0)
        m = R.GPT2(R.GPT2Config.tiny(fp8=True)).to(cuda)
        for p in m.parameters():
            p.data = p.data.to(torch.bfloat16)
        for st in F.fp8_states(m):
            st.wgrad = st.dgrad = True
        flat = FlatParams(m)
        opt = FusedAdamW(flat, lr=1e-3)
        gen = torch.Generator(device=cuda).manual_seed(7)
        losses, grads = [], []
        for _ in range(4):
            ids = torch.randint(0, 1000, (4, 129), device=cuda, generator=gen)
            opt.zero_grad()
            loss = m(ids[:, :-1], ids[:, 1:])
            loss.backward()
            g = flat.grad.float().clone()
            assert torch.isfinite(g).all()
            grads.append(g)
            opt.step()
            losses.append(float(loss))
        return losses, grads

    (la, ga), (lb, gb) = run(True), run(False)
    for x, y in zip(la, lb):
        assert abs(x - y) <= 0.01 * abs(y), (la, lb)
    # the first backward quantises dQKV itself either way (no delayed scale yet): identical; later ones
    # differ only by the e5m2 rounding of identical bf16 values and the weights' drift
    assert torch.equal(ga[0], gb[0])
    for a, b in zip(ga[1:], gb[1:]):
        assert ((a - b).norm() / b.norm()).item() < 0.05
