"""KV-cache decoding on the HIP kernels: cached one-token steps (attention with Tq < Tk, causal
bottom-right aligned) against the full bf16 forward, head sizes 64 and 32."""

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
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("n_head", [2, 4])
def test_decode_matches_full_forward(cuda, n_head):
    from replicann_amd.models.blocks import KVCache
    m = _model(cuda, n_head)
    seq = torch.randint(0, 1000, (3, 90), device=cuda)
    with torch.no_grad():
        full = m(seq)
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
    """The hipGraph-replayed one-token step (device-side position, masked full-cache attention)
    against the eager host-position steps: same first token, logits of each replay close."""
    from replicann_amd.models.blocks import KVCache
    m = _model(cuda, 2)
    idx = torch.randint(0, 1000, (3, 20), device=cuda)
    seq = torch.cat([idx, torch.randint(0, 1000, (3, 12), device=cuda)], 1)
    host = KVCache(m.config.n_layer, 32)
    dev = KVCache(m.config.n_layer, 32)
    m.decode_step(idx, host)
    m.decode_step(idx, dev)
    g, tok, out = m._capture_decode(dev, 3)
    for t in range(20, 32):
        a = m.decode_step(seq[:, t:t + 1], host)
        tok.copy_(seq[:, t:t + 1])
        g.replay()
        assert rel_err(out, a) < 3e-2, t
    torch.cuda.synchronize()
    assert int(dev.pos_t) == 32
    e = m.generate(idx, 12, temperature=0, graph=False)
    r = m.generate(idx, 12, temperature=0, graph=True)
    assert torch.equal(e[:, :21], r[:, :21])
    # every replayed step's greedy token is the argmax of the eager logits of the same prefix (up to
    # near-ties between the two attention kernels' roundings)
    host = KVCache(m.config.n_layer, 32)
    lg = m.decode_step(r[:, :20], host)
    agree = 0
    for t in range(20, 31):
        agree += int((lg.float().argmax(-1) == r[:, t]).sum())
        lg = m.decode_step(r[:, t:t + 1], host)
    assert agree >= 0.9 * 3 * 11


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
