"""The one-wave-per-SIMD persistent GEMM (tile config 11, csrc/include/gemm_w1.h) vs fp32 references.

The kernel interleaves a finished tile's epilogue into the next tile's first K-tile and keeps its
bias / DMA / store bookkeeping in hand-counted waits, so the cases below cover: several tiles per
workgroup (the epilogue path), 2 K-tiles per tile (the tightest wait counts), ragged M / N tails (the
store range checks), bias (the C-operand init), alpha, and the fp8 operands with power-of-two scales
riding the scaled MFMA's E8M0 operands.
"""

import os

import pytest
import torch

from replicann_amd import ops

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device="cuda") * scale).to(torch.bfloat16)


# (M, N, K): many tiles per CU (epilogue interleave), nk = 2 (K = 128 bf16 = 256 B), ragged M / N,
# a single tile, GPT-2-small shapes
SHAPES = [(65536, 768, 768), (65536, 512, 128), (8200, 1032, 256), (300, 200, 512), (256, 256, 128),
          (16384, 2304, 768), (4096, 3072, 1024)]


@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("with_bias", [False, True])
def test_w1_bf16_vs_fp32(cuda, M, N, K, with_bias):
    torch.manual_seed(M + N + K)
    a, b = bf(M, K), bf(N, K, scale=0.05)
    bias = bf(N) if with_bias else None
    ref = a.float() @ b.float().t()
    if with_bias:
        ref += bias.float()
    out = ops.gemm(a, b, tb=True, bias=bias, cfg=11)
    assert out.shape == (M, N)
    assert rel_err(out, ref) < 8e-3
    # the same bits as the cfg-9 kernel up to accumulation order: both are bf16 roundings of fp32 sums
    out9 = ops.gemm(a, b, tb=True, bias=bias, cfg=9)
    assert rel_err(out, out9) < 8e-3


def test_w1_bf16_alpha(cuda):
    torch.manual_seed(3)
    a, b = bf(8192, 768), bf(1024, 768, scale=0.05)
    alpha = torch.tensor([0.37], device="cuda")
    out = ops.gemm(a, b, tb=True, alpha=alpha, cfg=11)
    assert rel_err(out, 0.37 * (a.float() @ b.float().t())) < 8e-3


def test_w1_bf16_deterministic_and_ragged_rows_untouched(cuda):
    """Bitwise repeatable; rows / columns past M / N of a larger output buffer are never written."""
    torch.manual_seed(5)
    M, N, K = 1000, 776, 384
    a, b, bias = bf(M, K), bf(N, K, scale=0.05), bf(N)
    o1 = ops.gemm(a, b, tb=True, bias=bias, cfg=11)
    o2 = ops.gemm(a, b, tb=True, bias=bias, cfg=11)
    assert torch.equal(o1, o2)
    big = torch.full((M + 8, 800), 7.0, device="cuda", dtype=torch.bfloat16)
    view = big[:M, :N]
    ops.gemm(a, b, tb=True, bias=bias, cfg=11, out=view)
    assert torch.equal(view, o1)
    assert bool((big[M:] == 7.0).all()) and bool((big[:, N:] == 7.0).all())


@pytest.mark.parametrize("M,N,K", [(65536, 3072, 1024), (8192, 4096, 1024), (1000, 776, 512), (65536, 1024, 256)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_w1_fp8_vs_dequantised(cuda, M, N, K, with_bias, monkeypatch):
    torch.manual_seed(M + K)
    x, w = bf(M, K), bf(N, K, scale=0.05)
    bias = bf(N, scale=0.1) if with_bias else None
    qa, sa = ops.quantize_fp8(x)
    qb, sb = ops.quantize_fp8(w)
    for s in (sa[0], sb[0]):  # the contract the kernel relies on: power-of-two scales
        m, _ = torch.frexp(s.cpu())
        assert float(m) == 0.5
    ref = ops.dequantize_fp8(qa, sa).float() @ ops.dequantize_fp8(qb, sb).float().t()
    if with_bias:
        ref += bias.float()
    monkeypatch.setenv("REPLICANN_FP8_GEMM", "11")
    out = torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, None, 0, None)
    assert rel_err(out, ref) < 5e-3
    monkeypatch.setenv("REPLICANN_FP8_GEMM", "9")
    out9 = torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, None, 0, None)
    assert rel_err(out, out9) < 5e-3


# MN-contiguous B ([K][N], the data gradient dY·W): the transposing LDS reads, the per-lane N-tail
# check on the DMA
@pytest.mark.parametrize("M,N,K", [(65536, 768, 3072), (65536, 3072, 768), (8200, 1032, 256), (300, 200, 512),
                                   (256, 256, 128)])
def test_w1_bf16_b_mn_vs_fp32(cuda, M, N, K):
    torch.manual_seed(M + 2 * N + K)
    a, b = bf(M, K), bf(K, N, scale=0.05)
    ref = a.float() @ b.float()
    out = ops.gemm(a, b, tb=False, cfg=11)
    assert out.shape == (M, N)
    assert rel_err(out, ref) < 8e-3
    assert rel_err(out, ops.gemm(a, b, tb=False, cfg=9)) < 8e-3


def test_w1_bf16_b_mn_ragged_untouched(cuda):
    torch.manual_seed(11)
    M, N, K = 1000, 776, 384
    a, b = bf(M, K), bf(K, N, scale=0.05)
    o1 = ops.gemm(a, b, tb=False, cfg=11)
    big = torch.full((M + 8, 800), 7.0, device="cuda", dtype=torch.bfloat16)
    view = big[:M, :N]
    ops.gemm(a, b, tb=False, cfg=11, out=view)
    assert torch.equal(view, o1)
    assert rel_err(o1, a.float() @ b.float()) < 8e-3
    assert bool((big[M:] == 7.0).all()) and bool((big[:, N:] == 7.0).all())


# residual epilogue (x·Wᵀ + b + r): the residual rides bf16 MFMAs against a one-hot operand in K-tiles
# 1-4 of every tile (nk >= 6; shorter K falls back to cfg 9) — ragged rows / columns load zeros
@pytest.mark.parametrize("M,N,K", [(65536, 768, 768), (4096, 3072, 1024), (1000, 776, 512), (300, 200, 384),
                                   (8200, 1032, 3072)])
def test_w1_bf16_residual_vs_fp32(cuda, M, N, K):
    torch.manual_seed(M + 3 * N + K)
    a, b, bias, r = bf(M, K), bf(N, K, scale=0.05), bf(N), bf(M, N, scale=2.0)
    ref = a.float() @ b.float().t() + bias.float() + r.float()
    out = ops.gemm(a, b, tb=True, bias=bias, residual=r, cfg=11)
    assert rel_err(out, ref) < 8e-3
    assert rel_err(out, ops.gemm(a, b, tb=True, bias=bias, residual=r, cfg=9)) < 8e-3


def test_w1_bf16_residual_exact_passthrough(cuda):
    """A zero weight leaves bias + residual: the one-hot MFMA adds the residual exactly (bf16 values
    through fp32 sums with zeros), so the output equals the bf16 rounding of r + b."""
    torch.manual_seed(9)
    M, N, K = 2048, 1024, 768
    a, b, bias, r = bf(M, K), torch.zeros(N, K, device="cuda", dtype=torch.bfloat16), bf(N), bf(M, N, scale=3.0)
    out = ops.gemm(a, b, tb=True, bias=bias, residual=r, cfg=11)
    assert torch.equal(out, (r.float() + bias.float()).bfloat16())


@pytest.mark.parametrize("M,N,K", [(65536, 1024, 1024), (1000, 776, 768), (8192, 1024, 4096)])
def test_w1_fp8_residual_vs_dequantised(cuda, M, N, K, monkeypatch):
    torch.manual_seed(M + K + 1)
    x, w = bf(M, K), bf(N, K, scale=0.05)
    bias, r = bf(N, scale=0.1), bf(M, N)
    qa, sa = ops.quantize_fp8(x)
    qb, sb = ops.quantize_fp8(w)
    ref = ops.dequantize_fp8(qa, sa).float() @ ops.dequantize_fp8(qb, sb).float().t() + bias.float() + r.float()
    monkeypatch.delenv("REPLICANN_FP8_GEMM", raising=False)  # default: the w1 kernel
    out = torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, r, 0, None)
    assert rel_err(out, ref) < 5e-3
    monkeypatch.setenv("REPLICANN_FP8_GEMM", "0")
    assert rel_err(out, torch.ops.replicann.gemm_fp8(qa, qb, sa, sb, bias, r, 0, None)) < 5e-3
