"""The LayerNorm backward kernel writing the e5m2 dY of the fp8 projection that produced its input
(csrc/kernels/layernorm.hip ln_bwd_k<.., Q8>, ops/norm.py producer_fp8): the bytes and the delayed-scaling slot
must be exactly what the projection's own quantisation pass (bf8_quantize, delayed) makes from the stored bf16
dx, so a training step is bitwise the same with and without it."""

import pytest
import torch

import replicann_amd.ops.norm as norm_mod
from replicann_amd.models.gpt2 import GPT2, GPT2Config

pytestmark = pytest.mark.gpu


def test_layernorm_bwd_q8_matches_quantisation_pass(cuda):
    torch.manual_seed(3)
    M, E = 4096, 1024
    dy = torch.randn(M, E, device=cuda).bfloat16()
    gh = torch.randn(M, E, device=cuda).bfloat16()
    h = torch.randn(M, E, device=cuda).bfloat16()
    w = (torch.rand(E, device=cuda) + 0.5).bfloat16()
    mean = h.float().mean(1)
    rstd = torch.rsqrt(h.float().var(1, unbiased=False) + 1e-5)
    ops = torch.ops.replicann
    slot = torch.tensor([0.0, 3.0, 0.0, 0.0], device=cuda)  # a seeded slot: amax 3 from "the previous step"
    slot_ref = slot.clone()
    q8 = torch.empty(M, E, dtype=torch.uint8, device=cuda)
    dx, _, _ = ops.layernorm_bwd(dy, gh, h, w, mean, rstd, None, None, None, q8, slot)
    dx_ref, _, _ = ops.layernorm_bwd(dy, gh, h, w, mean, rstd, None, None, None)
    q_ref = ops.bf8_quantize(dx_ref, slot_ref, True)
    assert torch.equal(dx, dx_ref)
    assert torch.equal(q8, q_ref.view(M, E))
    assert torch.equal(slot, slot_ref)  # same rolled scale, same recorded amax


def _step_grads(cuda, ln_q8, steps=3):
    from replicann_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    m = GPT2(GPT2Config.tiny(fp8=True, n_embd=256, vocab_size=2000, vocab_pad=2048)).to(cuda)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    # the training path: gradients accumulated in place into the flat buffer (the token-embedding scatter
    # then honours REPLICANN_DETERMINISTIC; the standalone embedding_bwd adds float atomics in arrival order)
    flat = FlatParams(m)
    idx = torch.randint(0, 2000, (4, 128), device=cuda, generator=torch.Generator(device=cuda).manual_seed(1))
    old = norm_mod.FP8_LN_Q8
    norm_mod.FP8_LN_Q8 = ln_q8
    try:
        for _ in range(steps):  # step 1 seeds the gradient slots; later steps take the fused path
            flat.zero_grad()
            m(idx, idx).backward()
    finally:
        norm_mod.FP8_LN_Q8 = old
    return m, [flat.grad.clone()]


def test_gpt2_fp8_step_bitwise_with_layernorm_e5m2(cuda, monkeypatch):
    # the default token-embedding scatter adds float atomics in arrival order (a repeated token id's rows sum
    # in whatever order the waves land): two runs whose earlier kernels differ in timing may differ in wte's
    # last bits.  The fixed-point scatter is order-independent, so the comparison is bitwise everywhere.
    monkeypatch.setenv("REPLICANN_DETERMINISTIC", "1")
    m1, g1 = _step_grads(cuda, True)
    m0, g0 = _step_grads(cuda, False)
    assert m1.h[0].attn.c_proj.fp8_state is not None and m1.h[0].attn.c_proj.fp8_state.g_ready
    for a, b in zip(g1, g0):
        assert torch.equal(a, b)
    for b1, b0 in zip(m1.buffers(), m0.buffers()):
        assert torch.equal(b1, b0)
