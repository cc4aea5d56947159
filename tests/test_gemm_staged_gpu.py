"""Persistent GEMM (cfg 9) staged epilogue (csrc/include/gemm_pk.h, STG): an epilogue that reads a
full output-shaped operand — the saved activation of a fused activation backward (codes 3 / 4 / 6,
with the bias-gradient column partials), a residual, or a bf16 accumulate target — streams it
through the operand ring as two extra K-tiles instead of reading it behind a vmcnt(0) drain.

Every output must be BITWISE equal to the unstaged epilogue's (same per-element math, same column
sum order), for full and ragged tiles, short K (1-2 K-tiles per item: the epilogue-operand K-tiles
then sit right next to the next item's) and many tiles per CU — and right against fp32 math."""

import pytest
import torch

from replicann_amd import ops

pytestmark = pytest.mark.gpu

# (M, N, K, kind) — kind: act6 / act4 / act3 (dgrad nn + preact + bias grad), res (nt + residual),
# acc (nn, accumulate into a bf16 output)
CASES = [
    (65536, 3072, 768, "act6"),   # GPT-2-small fc1 dgrad with the saved gelu'
    (4096, 3072, 768, "act4"),
    (3000, 1000, 200, "act3"),    # ragged M / N / K
    (1024, 768, 64, "act6"),      # nk = 1
    (65536, 768, 768, "res"),     # attention c_proj forward + residual
    (4096, 768, 3072, "res"),     # MLP c_proj forward + residual
    (2000, 520, 136, "res"),      # ragged, nk = 3
    (4096, 768, 768, "acc"),
    (1000, 264, 128, "acc"),      # ragged, nk = 2
]


def _inputs(case, dev):
    M, N, K, kind = case
    g = torch.Generator(device="cpu").manual_seed(3)
    nt = kind == "res"
    A = (torch.randn(M, K, generator=g) * 0.5).to(dev, torch.bfloat16)
    B = (torch.randn(*((N, K) if nt else (K, N)), generator=g) * 0.5).to(dev, torch.bfloat16)
    aux = (torch.randn(M, N, generator=g)).to(dev, torch.bfloat16)
    if kind == "act6":
        aux = (torch.rand(M, N, generator=g) * 1.2 - 0.1).to(dev, torch.bfloat16)
    return A, B, aux, nt


def _run(case, dev, staged):
    M, N, K, kind = case
    A, B, aux, nt = _inputs(case, dev)
    prev = int(torch.ops.replicann.gemm_get_staged())
    torch.ops.replicann.gemm_set_staged(int(staged))
    try:
        if kind.startswith("act"):
            act = int(kind[3:])
            bg = torch.zeros(N, device=dev, dtype=torch.bfloat16)
            y = torch.ops.replicann.gemm(A, B, False, False, None, None, act, aux, None, False, 1, False, None, 9, bg)
            extra = bg
        elif kind == "res":  # (a seeded bias: both runs must see the same one)
            bias = torch.randn(N, generator=torch.Generator(device="cpu").manual_seed(4)).to(dev, torch.bfloat16)
            y = ops.gemm(A, B, tb=True, bias=bias, residual=aux, cfg=9, split_k=1)
            extra = None
        else:
            y = aux.clone()
            ops.gemm(A, B, out=y, accumulate=True, cfg=9, split_k=1)
            extra = None
        torch.cuda.synchronize()
    finally:
        torch.ops.replicann.gemm_set_staged(prev)
    return y, extra, (A, B, aux, nt)


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}x{c[1]}x{c[2]}_{c[3]}")
def test_staged_epilogue_bitwise_equal_and_correct(cuda, case):
    ys, es, (A, B, aux, nt) = _run(case, cuda, True)
    yu, eu, _ = _run(case, cuda, False)
    assert torch.equal(ys, yu)
    if es is not None:
        assert torch.equal(es, eu)
    M, N, K, kind = case
    h = A.float() @ (B.t() if nt else B).float()
    if kind == "act6":
        ref = h.bfloat16().float() * aux.float()
    elif kind == "act4":
        x = aux.float()
        t = torch.tanh(0.7978845608 * (x + 0.044715 * x ** 3))
        ref = h.bfloat16().float() * (0.5 * (1 + t) + 0.5 * x * (1 - t * t) * 0.7978845608 * (1 + 3 * 0.044715 * x * x))
    elif kind == "act3":
        ref = h.bfloat16().float() * (aux.float() > 0).float()
    elif kind == "res":  # bias + residual
        bias = torch.randn(N, generator=torch.Generator(device="cpu").manual_seed(4)).to(h.device, torch.bfloat16)
        ref = h + bias.float() + aux.float()
    else:  # acc: checked below
        ref = None
    if ref is not None:
        err = (ys.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)
        assert err < 2e-2, err
        if es is not None:  # bias gradient = column sums of the stored (bf16) output
            cs = ys.float().sum(0)
            assert ((es.float() - cs).abs().max() / cs.abs().max()) < 2e-2
    elif kind == "acc":
        ref = aux.float() + h
        assert ((ys.float() - ref).abs().max() / ref.abs().max()) < 2e-2


def test_staged_is_off_by_default(cuda):
    """Measured slower than the unstaged epilogue (profiles/gemm_staged_ab_r4f.txt): A/B only."""
    assert int(torch.ops.replicann.gemm_get_staged()) == 0
