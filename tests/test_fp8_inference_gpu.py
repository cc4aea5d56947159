"""fp8 delayed scaling is training state: inference between training steps must not touch it.

evaluate() / generate() on an fp8 model used to roll the delayed-scale slots and record their own
batches' amax (LayerNorm's e4m3 producer, the activation quantiser, the fc1 epilogue's e4m3 output),
so the next training step quantised with a scale from an eval batch (or a 1-token decode).  With the
inference scratch slots (ops/fp8.py ``Fp8State.roll_slot``) a run that trains 3 steps, evaluates,
generates and trains 3 more is bitwise the run that trains 6 steps.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(cuda):
    import replicann_amd as R
    from replicann_amd.ops.fp8 import attach_weight_cache
    from replicann_amd.optim import FusedAdamW
    from replicann_amd.utils.flat import FlatParams

    torch.manual_seed(0)
    m = R.GPT2(R.GPT2Config.tiny(fp8=True)).to(cuda)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    flat = FlatParams(m)
    opt = FusedAdamW(flat, lr=1e-3)
    attach_weight_cache(m, flat, opt)
    return m, opt


def _batches(cuda, n):
    g = torch.Generator(device=cuda).manual_seed(7)
    return [torch.randint(0, 1000, (4, 129), device=cuda, generator=g) for _ in range(n)]


def _train(m, opt, batches):
    m.train()
    for ids in batches:
        opt.zero_grad()
        loss = m(ids[:, :-1], ids[:, 1:])
        loss.backward()
        opt.step()


def test_fp8_eval_and_generate_leave_training_state_untouched(cuda):
    from replicann_amd.training import evaluate

    batches = _batches(cuda, 6)
    m_ref, opt_ref = _setup(cuda)
    _train(m_ref, opt_ref, batches)

    m, opt = _setup(cuda)
    _train(m, opt, batches[:3])
    scales_before = {k: v.clone() for k, v in m.state_dict().items() if k.endswith("fp8_scales")}
    assert scales_before
    evald = iter([(b[:, :-1], b[:, 1:]) for b in _batches(cuda, 2)])
    loss = evaluate(m, evald, steps=2)
    assert loss
    prompt = torch.randint(0, 1000, (2, 5), device=cuda, generator=torch.Generator(device=cuda).manual_seed(3))
    m.generate(prompt, 6, temperature=0.0)
    for k, v in m.state_dict().items():  # inference rolled / recorded nothing
        if k.endswith("fp8_scales"):
            assert torch.equal(v, scales_before[k]), k
    _train(m, opt, batches[3:])

    for (n, a), (_, b) in zip(m.state_dict().items(), m_ref.state_dict().items()):
        assert torch.equal(a, b), n
