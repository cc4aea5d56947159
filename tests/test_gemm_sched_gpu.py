"""Persistent GEMM (cfg 9) dynamic tile queue (csrc/include/gemm_pk.h, "Tile schedule"): every
output is bitwise identical to the static walk's — across operand layouts, epilogues, split-K,
small K (multi-item units), few / many tiles and a CU reservation — and the self-resetting
counters stay consistent over many back-to-back launches (a stale counter would skip tiles)."""

import pytest
import torch

from replicann_amd import ops

pytestmark = pytest.mark.gpu

# (M, N, K, ta, tb, act, split)
CASES = [
    (4096, 2304, 768, False, True, 0, 1),     # qkv-like fwd (nt)
    (3000, 1000, 200, False, True, 0, 1),     # ragged M/N/K, nk = 4 -> 2-item units
    (1024, 768, 64, False, True, 0, 1),       # nk = 1 -> 5-item units
    (4096, 3072, 768, False, True, 5, 1),     # GELU + saved derivative (two outputs)
    (4096, 768, 3072, False, False, 0, 1),    # dgrad (nn)
    (2304, 768, 8192, True, False, 0, 4),     # wgrad (tn) with split-K slabs
    (512, 512, 512, False, True, 0, 1),       # fewer tiles than CUs
    (65536, 768, 768, False, True, 0, 1),     # many tiles: home queues + shared tail
]


def _run(case, dev, sched, reserve=0):
    M, N, K, ta, tb, act, split = case
    g = torch.Generator(device="cpu").manual_seed(1)
    A = (torch.randn(*((K, M) if ta else (M, K)), generator=g) * 0.5).to(dev, torch.bfloat16)
    B = (torch.randn(*((N, K) if tb else (K, N)), generator=g) * 0.5).to(dev, torch.bfloat16)
    bias = (torch.randn(N, generator=g)).to(dev, torch.bfloat16) if act else None
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if act else None
    torch.ops.replicann.gemm_set_sched(sched)
    torch.ops.replicann.gemm_set_reserve(reserve)
    try:
        out = ops.gemm(A, B, ta=ta, tb=tb, bias=bias, act=act, preact=pre, cfg=9, split_k=split)
        torch.cuda.synchronize()
    finally:
        torch.ops.replicann.gemm_set_sched(0)
        torch.ops.replicann.gemm_set_reserve(0)
    return out, pre, (A, B)


@pytest.mark.parametrize("case", CASES, ids=lambda c: "x".join(map(str, c[:3])) + f"_{'t' if c[3] else 'n'}{'t' if c[4] else 'n'}_a{c[5]}_s{c[6]}")
@pytest.mark.parametrize("reserve", [0, 8])
def test_dynamic_equals_static_bitwise(cuda, case, reserve):
    ys, ps, (A, B) = _run(case, cuda, 0, reserve)
    yd, pd, _ = _run(case, cuda, 1, reserve)
    assert torch.equal(ys, yd)
    if ps is not None:
        assert torch.equal(ps, pd)
    # and it is the right product (fp32 reference)
    M, N, K, ta, tb, act, split = case
    if act == 0:
        ref = (A.t() if ta else A).float() @ (B.t() if tb else B).float()
        err = (yd.float() - ref).abs().max() / ref.abs().max()
        assert err < 2e-2


def test_counters_reset_over_many_launches(cuda):
    """200 launches over a 256-slot counter pool (slots revisited; a counter left non-zero by one
    launch would make a later launch skip tiles), mixing shapes that use 1- and 5-item units."""
    torch.ops.replicann.gemm_set_sched(1)
    a = torch.randn(4096, 768, device=cuda).bfloat16()
    b = torch.randn(2304, 768, device=cuda).bfloat16()
    c = torch.randn(1024, 64, device=cuda).bfloat16()
    d = torch.randn(768, 64, device=cuda).bfloat16()
    y0 = ops.gemm(a, b, tb=True, cfg=9)
    z0 = ops.gemm(c, d, tb=True, cfg=9)
    for i in range(300):
        y = ops.gemm(a, b, tb=True, cfg=9)
        z = ops.gemm(c, d, tb=True, cfg=9)
        if i % 50 == 0 or i == 299:
            torch.cuda.synchronize()
            assert torch.equal(y, y0) and torch.equal(z, z0), i
    torch.ops.replicann.gemm_set_sched(0)


def test_schedule_knobs_and_debug_cfg_rejected(cuda):
    import os
    if "REPLICANN_GEMM_SCHED" not in os.environ:  # off by default: the data-parallel reducer turns it on
        torch.ops.replicann.gemm_set_sched(0)
    assert torch.ops.replicann.gemm_get_sched() == 0
    torch.ops.replicann.gemm_set_reserve(13)  # rounded down to a multiple of 8 (one CU per dispatch group)
    assert torch.ops.replicann.gemm_get_reserve() == 8
    torch.ops.replicann.gemm_set_reserve(0)
    a = torch.randn(256, 256, device=cuda).bfloat16()
    with pytest.raises(RuntimeError):  # timing-only ablation kernels are not in a production build
        ops.gemm(a, a, tb=True, cfg=91)
