"""KV-cache incremental decoding of GPT-2 (``GPT2.decode_step`` / ``GPT2.generate``) on the CPU path:
the cached decode must reproduce the full causal forward (same math, prefix not recomputed)."""

import pytest
import torch

from replicann_amd.models import GPT2, GPT2Config
from replicann_amd.models.blocks import KVCache


def _model():
    torch.manual_seed(0)
    return GPT2(GPT2Config.tiny()).eval()


def test_generate_greedy_matches_recompute():
    m = _model()
    idx = torch.randint(0, 1000, (3, 9))
    out = m.generate(idx, 12, temperature=0)
    ref = idx
    for _ in range(12):
        ref = torch.cat([ref, m(ref)[:, -1].argmax(-1, keepdim=True)], 1)
    assert out.shape == (3, 21) and torch.equal(out, ref)


@pytest.mark.parametrize("chunks", [(8, 1, 1, 1), (5, 3, 4), (1, 1, 1, 1, 1, 1)])
def test_decode_step_matches_full_forward(chunks):
    """Multi-token appends (chunked prefill) and one-token steps, teacher-forced."""
    m = _model()
    seq = torch.randint(0, 1000, (2, sum(chunks)))
    cache = KVCache(m.config.n_layer, sum(chunks))
    full = m(seq)
    pos = 0
    for t in chunks:
        lg = m.decode_step(seq[:, pos:pos + t], cache)
        pos += t
        assert (lg - full[:, pos - 1]).abs().max().item() < 1e-4
    assert cache.pos == pos


def test_generate_sampling_reproducible_and_topk():
    m = _model()
    idx = torch.randint(0, 1000, (2, 4))
    a = m.generate(idx, 8, temperature=0.8, top_k=5, generator=torch.Generator().manual_seed(3))
    b = m.generate(idx, 8, temperature=0.8, top_k=5, generator=torch.Generator().manual_seed(3))
    assert torch.equal(a, b)
    # every sampled token is among the top-5 of its step's logits
    for t in range(4, 12):
        top = m(a[:, :t])[:, -1].topk(5, -1).indices
        assert bool((top == a[:, t:t + 1]).any(-1).all())


def test_cache_limits():
    m = _model()
    with pytest.raises(ValueError):
        m.generate(torch.zeros(1, 100, dtype=torch.long), 40)  # 140 > block_size 128
    cache = KVCache(m.config.n_layer, 4)
    m.decode_step(torch.zeros(1, 4, dtype=torch.long), cache)
    with pytest.raises(ValueError):
        m.decode_step(torch.zeros(1, 1, dtype=torch.long), cache)
    assert m.training is False
    m.train()
    m.generate(torch.zeros(1, 2, dtype=torch.long), 2)
    assert m.training is True  # generate restores the mode


def test_device_position_steps_match_host_position():
    """The capturable step (device-side position, cache rows written by index, the key mask carrying
    causality) against the host-position decode, teacher-forced, run eagerly here."""
    m = _model()
    seq = torch.randint(0, 1000, (2, 20))
    host = KVCache(m.config.n_layer, 20)
    dev = KVCache(m.config.n_layer, 20)
    m.decode_step(seq[:, :12], host)
    m.decode_step(seq[:, :12], dev)
    dev.to_device_position()
    for t in range(12, 20):
        a = m.decode_step(seq[:, t:t + 1], host)
        b = m._device_position_step(seq[:, t:t + 1], dev)
        assert (a - b).abs().max().item() < 1e-4
    assert int(dev.pos_t) == 20 and bool((dev.mask == 0).all())


def test_generate_cli_from_checkpoint(tmp_path, capsys):
    """``python -m replicann generate`` loads a training checkpoint (weights_only) and reproduces the
    model's own greedy continuation."""
    import json

    from replicann_amd import cli
    from replicann_amd.utils.checkpoint import save_checkpoint
    m = _model()
    ck = tmp_path / "ck.pt"
    save_checkpoint(str(ck), m, step=3)
    prompt = [5, 17, 256, 999]
    cli.main(["generate", "--model", "gpt2-tiny", "--checkpoint", str(ck), "--prompt", ",".join(map(str, prompt)),
              "--new", "6", "--temperature", "0", "--device", "cpu"])
    res = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    want = m.generate(torch.tensor([prompt]), 6, temperature=0)[0, 4:].tolist()
    assert res["tokens"] == [want] and res["new_tokens"] == 6


def test_top_p_nucleus():
    """top_p keeps the smallest set of most probable tokens reaching the mass (always the top one)."""
    from replicann_amd.models.gpt2 import _sample
    lg = torch.log(torch.tensor([[0.5, 0.3, 0.15, 0.05], [0.9, 0.05, 0.03, 0.02]]))
    g = torch.Generator().manual_seed(0)
    seen = {0: set(), 1: set()}
    for _ in range(300):
        t = _sample(lg.clone(), 1.0, None, g, top_p=0.75)
        seen[0].add(int(t[0])), seen[1].add(int(t[1]))
    assert seen[0] == {0, 1} and seen[1] == {0}
    m = _model()
    out = m.generate(torch.zeros(2, 3, dtype=torch.long), 5, temperature=1.0, top_p=0.9,
                     generator=torch.Generator().manual_seed(1))
    assert out.shape == (2, 8)


def test_model_copy_after_generate():
    """Stored decode graphs / caches live outside the module: deepcopy and state_dict are unaffected."""
    import copy
    m = _model()
    m.generate(torch.zeros(1, 3, dtype=torch.long), 4, temperature=0, graph=False)
    m2 = copy.deepcopy(m)
    assert set(m2.state_dict()) == set(m.state_dict())


def test_top_p_degenerate_keeps_top_token():
    """top_p <= 0 in _sample keeps the most likely token (no all -inf row, no NaN softmax); generate
    and the CLI refuse top_p outside (0, 1]."""
    import pytest

    import replicann_amd as R
    from replicann_amd.models.gpt2 import _sample

    lg = torch.tensor([[0.1, 2.0, -1.0, 0.5], [3.0, 0.0, 0.0, 0.0]])
    g = torch.Generator().manual_seed(0)
    for p in (0.0, -1.0, 1e-9):
        t = _sample(lg.clone(), 1.0, None, g, top_p=p)
        assert t.squeeze(-1).tolist() == [1, 0]
    m = R.GPT2(R.GPT2Config.tiny())
    for bad in (0.0, -0.5, 1.5):
        with pytest.raises(ValueError):
            m.generate(torch.zeros(1, 3, dtype=torch.long), 2, top_p=bad)
