"""KV-cache decoding on the HIP kernels: cached one-token steps (attention with Tq < Tk, causal
bottom-right aligned) and the hipGraph-replayed step against an fp32 ATen forward of the same weights
(the model's CPU path), head sizes 64 and 32.

Tolerance: 3e-2 relative L2 on the logits, the bf16 budget of this 2-layer model (bf16 weights,
activations and cache; its full native forward is within 1.2e-2 of the same fp32 reference)."""

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(cuda, n_head):
    import replicann_amd as R
    torch.manual_seed(0)
    m = R.GPT2(R.GPT2Config.tiny(n_embd=128, n_head=n_head, n_layer=2, block_size=128)).to(cuda)
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    return m.eval()


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _fp32_logits(m, seq):
    """fp32 ATen forward (the CPU path of GPT2.forward) of the same bf16 weights: (B, T, vocab)."""
    ref = copy.deepcopy(m).float().cpu().eval()
    with torch.no_grad():
        return ref(seq.cpu())


@pytest.mark.parametrize("n_head", [2, 4])
def test_decode_matches_full_forward(cuda, n_head):
    from replicann_amd.models.blocks import KVCache
    m = _model(cuda, n_head)
    seq = torch.randint(0, 1000, (3, 90), device=cuda)
    full = _fp32_logits(m, seq)
    with torch.no_grad():
        assert rel_err(m(seq), full) < 2e-2  # the native full forward itself
    cache = KVCache(m.config.n_layer, 90)
    lg = m.decode_step(seq[:, :70], cache)  # prefill
    assert rel_err(lg, full[:, 69]) < 3e-2
    for t in range(70, 90):  # one-token steps
        lg = m.decode_step(seq[:, t:t + 1], cache)
        assert rel_err(lg, full[:, t]) < 3e-2, t
    torch.cuda.synchronize()


def test_generate_gpu(cuda):
    m = _model(cuda, 2)
    idx = torch.randint(0, 1000, (4, 16), device=cuda)
    out = m.generate(idx, 24, temperature=0)
    assert out.shape == (4, 40) and torch.equal(out[:, :16], idx)
    with torch.no_grad():
        first = m(idx)[:, -1].float().argmax(-1)
    assert torch.equal(out[:, 16], first)
    s = m.generate(idx, 8, temperature=1.0, top_k=20, generator=torch.Generator(device=cuda).manual_seed(1))
    assert s.shape == (4, 24) and int(s.max()) < m.config.vocab_size


def test_generate_graph_matches_eager(cuda):
    """The hipGraph-replayed one-token step (device-side position, masked full-cache attention) and
    the eager host-position steps, each against the fp32 forward of the same prefix."""
    from replicann_amd.models.blocks import KVCache
    m = _model(cuda, 2)
    idx = torch.randint(0, 1000, (3, 20), device=cuda)
    seq = torch.cat([idx, torch.randint(0, 1000, (3, 12), device=cuda)], 1)
    full = _fp32_logits(m, seq)
    host = KVCache(m.config.n_layer, 32)
    dev = KVCache(m.config.n_layer, 32)
    m.decode_step(idx, host)
    m.decode_step(idx, dev)
    g, tok, out = m._capture_decode(dev, 3)
    for t in range(20, 32):
        a = m.decode_step(seq[:, t:t + 1], host)
        tok.copy_(seq[:, t:t + 1])
        g.replay()
        assert rel_err(a, full[:, t]) < 3e-2, t
        assert rel_err(out, full[:, t]) < 3e-2, t
    torch.cuda.synchronize()
    assert int(dev.pos_t) == 32
    # generate(): graph replay and eager steps give the same greedy prefix, and every replayed step's
    # logits (re-derived here by the fp32 forward of the generated prefix) make its token a top choice
    e = m.generate(idx, 12, temperature=0, graph=False)
    r = m.generate(idx, 12, temperature=0, graph=True)
    assert torch.equal(e[:, :21], r[:, :21])
    ref = _fp32_logits(m, r)
    for t in range(20, 31):
        lg = ref[:, t - 1]
        chosen = lg.gather(-1, r[:, t:t + 1].cpu()).squeeze(-1)
        # greedy on bf16 logits within the bf16 budget of the fp32 maximum
        assert bool((chosen >= lg.max(-1).values - 3e-2 * lg.abs().max(-1).values).all()), t


def test_generate_registry_bounded(cuda):
    """Serving with varying prompt lengths / batch sizes keeps at most DECODE_GRAPHS_MAX captured steps:
    lengths share a 64-token bucket, the least recently used entry is evicted."""
    from replicann_amd.models import gpt2 as G
    m = _model(cuda, 2)
    for B in (1, 2, 3):
        for T0 in (5, 9, 30, 61):
            m.generate(torch.randint(0, 1000, (B, T0), device=cuda), 3, temperature=0)
            assert len(m._decode_graphs()) <= G.DECODE_GRAPHS_MAX
    lens = {k[1] for k in m._decode_graphs()}
    assert lens <= {64, 128}
    m.generate(torch.randint(0, 1000, (5, 10), device=cuda), 4, temperature=0)
    assert len(m._decode_graphs()) <= G.DECODE_GRAPHS_MAX
    m.clear_decode_graphs()


def test_generate_graph_reuse(cuda):
    """A second generate with the same batch / length replays the stored graph (no new capture) and
    gives the same greedy tokens; another batch size captures its own; re-assigned parameters
    invalidate the stored graphs."""
    m = _model(cuda, 2)
    idx = torch.randint(0, 1000, (2, 10), device=cuda)
    a = m.generate(idx, 9, temperature=0)
    assert len(m._decode_graphs()) == 1
    b = m.generate(idx, 9, temperature=0)
    assert torch.equal(a, b) and len(m._decode_graphs()) == 1
    m.generate(idx[:1], 9, temperature=0)
    assert len(m._decode_graphs()) == 2
    with torch.no_grad():
        for p in m.parameters():
            p.data = p.data.clone()
    c = m.generate(idx, 9, temperature=0)
    assert torch.equal(a, c) and len(m._decode_graphs()) == 1
    m.clear_decode_graphs()
    assert len(m._decode_graphs()) == 0
