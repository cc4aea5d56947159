"""The fp8 LM head (ops/loss.py _LinearXentFp8Fn, GPT2Config.fp8_head): logits from e4m3 h · e4m3 W on the
one-wave-per-SIMD fp8 GEMM, the cross-entropy kernel writing the loss gradient as e5m2 · 2^15
(csrc/kernels/softmax_xent.hip xent_row2_k<.., Q8>), and both head gradients on the fp8 GEMMs with g / n as
an extra device scalar (the data gradient's alpha, the weight gradient's split-K reduction multiplier).

Checked against fp32 math on the DEQUANTISED operands (the same pow2 scales the kernels use), so the test
pins the kernels, not the quantisation error; the model-level test checks a GPT-2 step against the bf16 head."""

import pytest
import torch
import torch.nn.functional as F

from replicann_amd import ops
from replicann_amd.ops.fp8 import Fp8State, pow2_ceil
from replicann_amd.ops.loss import XQ8_SCALE

pytestmark = pytest.mark.gpu


def _e4m3(x):
    s = pow2_ceil(x.abs().max().float().cpu() / 448.0).to(x.device)
    return (x.float() / s).to(torch.float8_e4m3fn).float() * s


def test_xent_q8_matches_bf16_gradient(cuda):
    g = torch.Generator(device="cpu").manual_seed(3)
    M, V, nv = 256, 50304, 50257
    logits = (torch.randn(M, V, generator=g) * 3).to(cuda, torch.bfloat16)
    tg = torch.randint(0, nv, (M,), generator=g).to(cuda)
    tg[5] = -100  # an ignored row: zero gradient
    q8 = torch.empty(M, V, dtype=torch.uint8, device=cuda)
    l8, lse8 = torch.ops.replicann.xent_fwd_q8(logits, tg, nv, -100, q8)
    lg = logits.clone()
    l16, lse16 = torch.ops.replicann.xent_fwd(lg, tg, nv, -100, True)  # bf16 (softmax - onehot) in place
    assert torch.equal(l8, l16) and torch.equal(lse8, lse16)
    # the e5m2 gradient is the e5m2 rounding of the same values (scaled by 2^15); the bf16 path rounds to bf16
    # first: a bf16 value that lands exactly on an e5m2 midpoint (~2^-6 of them: bf16 keeps 6 more mantissa bits)
    # ties to even where the unrounded fp32 value rounds the other way, one e5m2 step away (measured 1.5 %)
    ref = (lg.float() * XQ8_SCALE).to(torch.float8_e5m2)
    got = q8.view(torch.float8_e5m2)
    diff = q8 != ref.view(torch.uint8)
    assert diff.float().mean().item() < 3e-2
    a, b = got.float()[diff], ref.float()[diff]
    assert bool(((a - b).abs() <= 0.25 * torch.maximum(a.abs(), b.abs()) + 2.0 ** -16).all())
    assert int(q8[5].count_nonzero()) == 0
    assert int(q8[:, nv:].count_nonzero()) == 0


@pytest.mark.parametrize("shape", [(1024, 1024, 256, 1000), (2048, 2048, 512, 2040)], ids=lambda s: "x".join(map(str, s)))
def test_fp8_head_vs_fp32_on_dequantised(cuda, shape):
    M, V, E, nv = shape
    g = torch.Generator(device="cpu").manual_seed(7)
    h = torch.randn(M, E, generator=g).to(cuda, torch.bfloat16).requires_grad_()
    w = (torch.randn(V, E, generator=g) * 0.05).to(cuda, torch.bfloat16).requires_grad_()
    tg = torch.randint(0, nv, (M,), generator=g).to(cuda)
    st = Fp8State()
    loss = ops.linear_cross_entropy(h, w, tg, n_valid_cols=nv, fp8=st)
    (loss * 0.75).backward()  # g != 1: the extra device scalar carries g / n
    # reference: the same e4m3 operands (fresh state = current scaling), fp32 math, bf16 logits, the gradient
    # rounded as the kernel rounds it (bf16 e, then e5m2 · 2^15)
    hq, wq = _e4m3(h.detach()), _e4m3(w.detach())
    logits = (hq @ wq.t()).to(torch.bfloat16).float()
    lref = F.cross_entropy(logits[:, :nv], tg)
    assert abs(loss.item() - lref.item()) < 2e-3 * abs(lref.item()), (loss.item(), lref.item())
    p = torch.softmax(logits[:, :nv], dim=1)
    d = torch.zeros(M, V, device=cuda)
    d[:, :nv] = p
    d[torch.arange(M, device=cuda), tg] -= 1.0
    d8 = (d * XQ8_SCALE).to(torch.float8_e5m2).float() / XQ8_SCALE
    scale = 0.75 / M
    gh_ref = d8 @ wq * scale
    gw_ref = d8.t() @ hq * scale
    eh = ((h.grad.float() - gh_ref).norm() / gh_ref.norm()).item()
    ew = ((w.grad.float() - gw_ref).norm() / gw_ref.norm()).item()
    # bf16 logits / softmax rounding moves a few e5m2 roundings of the gradient by one step (≤ 25 % of those
    # elements), hence a few % rather than bf16 level
    assert eh < 3e-2 and ew < 3e-2, (eh, ew)
    # and against the plain fp32 head (no quantisation): within fp8 error
    hr = h.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    (F.cross_entropy((hr @ wr.t())[:, :nv], tg) * 0.75).backward()
    cos_h = F.cosine_similarity(h.grad.float().flatten(), hr.grad.flatten(), dim=0).item()
    cos_w = F.cosine_similarity(w.grad.float().flatten(), wr.grad.flatten(), dim=0).item()
    assert cos_h > 0.99 and cos_w > 0.99, (cos_h, cos_w)


def test_gpt2_fp8_head_step_tracks_bf16_head(cuda):
    from replicann_amd.models.gpt2 import GPT2, GPT2Config

    torch.manual_seed(0)
    cfg = GPT2Config.tiny(fp8=True, fp8_head=1, n_embd=256, vocab_size=2000, vocab_pad=2048)
    m8 = GPT2(cfg).to(cuda)
    m16 = GPT2(GPT2Config.tiny(fp8=True, fp8_head=0, n_embd=256, vocab_size=2000, vocab_pad=2048)).to(cuda)
    m16.load_state_dict(m8.state_dict(), strict=False)
    for m in (m8, m16):  # bf16 parameters, fp32 scale buffers
        for p in m.parameters():
            p.data = p.data.to(torch.bfloat16)
    idx = torch.randint(0, 2000, (4, 128), device=cuda)
    tgt = torch.randint(0, 2000, (4, 128), device=cuda)
    for _ in range(2):  # first call: current scaling; second: the delayed scales
        for m in (m8, m16):
            m.zero_grad(set_to_none=True)
            m(idx, tgt).backward()
    assert m8.head8.fp8_state.ready == [True, True]
    assert float(m8.head8.fp8_scales[0, 0]) > 0 and float(m8.head8.fp8_scales[1, 0]) > 0
    for (n, a), (_, b) in zip(m8.named_parameters(), m16.named_parameters()):
        cos = F.cosine_similarity(a.grad.float().flatten(), b.grad.float().flatten(), dim=0).item()
        assert cos > 0.98, (n, cos)
    # inference does not take the fp8 head (and leaves its slots alone)
    before = m8.head8.fp8_scales.clone()
    m8.eval()
    with torch.no_grad():
        m8(idx, tgt)
    assert torch.equal(before, m8.head8.fp8_scales)


def test_fp8_head_bf16_logits_mode(cuda):
    """fp8_logits=False: the loss is the bf16 head's bit for bit, the gradients the fp8 ones."""
    g = torch.Generator(device="cpu").manual_seed(11)
    M, V, E, nv = 1024, 1024, 256, 1000
    h = torch.randn(M, E, generator=g).to(cuda, torch.bfloat16).requires_grad_()
    w = (torch.randn(V, E, generator=g) * 0.05).to(cuda, torch.bfloat16).requires_grad_()
    tg = torch.randint(0, nv, (M,), generator=g).to(cuda)
    loss2 = ops.linear_cross_entropy(h, w, tg, n_valid_cols=nv, fp8=Fp8State(), fp8_logits=False)
    loss2.backward()
    l16 = ops.linear_cross_entropy(h.detach(), w.detach(), tg, n_valid_cols=nv)
    assert torch.equal(loss2.detach(), l16)
    hr = h.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    F.cross_entropy((hr @ wr.t())[:, :nv], tg).backward()
    for a, b in ((h.grad, hr.grad), (w.grad, wr.grad)):
        assert F.cosine_similarity(a.float().flatten(), b.flatten(), dim=0).item() > 0.99
