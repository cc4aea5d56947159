"""Reference-block fused QKV: with the parameters in a FlatParams buffer the
per-head Q/K/V weights are packed back to back, the fused projection is a zero-copy view, and the
per-head gradients equal those of the plain (concatenating) module; without flat storage, eval
forwards reuse one concatenation while the weights are unchanged."""

import torch

from replicann_amd.arch.transformer import TransformerEncoder
from replicann_amd.utils.flat import FlatParams


def _model(seed=0):
    torch.manual_seed(seed)
    return TransformerEncoder(n_heads=3, embedding_size=24, p_dropout=0.0)


def test_fused_view_grads_match_plain():
    ref, m = _model(), _model()
    for mod in (ref, m):
        for h in mod._attn._heads:
            h._dropout.p = 0.0
    flat = FlatParams(m)
    heads = m._attn._heads
    ws = [h._query.weight for h in heads] + [h._key.weight for h in heads] + [h._value.weight for h in heads]
    # packed back to back in fused order
    base = ws[0].data_ptr()
    step = ws[0].numel() * ws[0].element_size()
    assert [w.data_ptr() for w in ws] == [base + i * step for i in range(len(ws))]
    w, _ = m._attn._cat_weights()
    assert w.data_ptr() == base and w.shape == (9 * 8, 24)
    ready = []
    flat.ready_hooks.append(lambda p: ready.append(id(p)))
    x = torch.randn(2, 5, 24)
    ref(x).square().sum().backward()
    flat.zero_grad()
    m(x).square().sum().backward()
    for (n, pr), pm in zip(ref.named_parameters(), m.parameters()):
        assert torch.allclose(pr.grad, pm.grad, atol=1e-5, rtol=1e-5), n
    assert {id(p) for p in ws} <= set(ready)  # every member reported final (DDP bucketing)
    # the optimizer's flat view and the per-head parameters stay one storage
    with torch.no_grad():
        flat.data.add_(1.0)
    assert torch.equal(w, torch.cat(ws, 0))


def test_eval_concat_cached_by_version():
    m = _model().eval()
    with torch.no_grad():
        w1, _ = m._attn._cat_weights()
        w2, _ = m._attn._cat_weights()
        assert w1 is w2
        m._attn._heads[0]._key.weight.add_(1.0)  # bumps _version: re-concatenate
        w3, _ = m._attn._cat_weights()
    assert w3 is not w1 and not torch.equal(w1, w3)
