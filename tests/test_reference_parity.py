"""T1 reference parity: same signatures, state_dict layout and
forward outputs as /root/reference/src/replicann (fp32, eval mode, CPU)."""

import inspect

import pytest
import torch

import replicann_amd.arch.transformer as T
import replicann_amd.nn.attention as A

ATOL = 2e-5


def _copy(ref_mod, new_mod):
    new_mod.load_state_dict(ref_mod.state_dict(), strict=True)


def _sig(f):
    return [(p.name, p.kind, p.default) for p in inspect.signature(f).parameters.values()]


def _same_keys(a, b):
    sa, sb = a.state_dict(), b.state_dict()
    assert list(sa.keys()) == list(sb.keys())
    for k in sa:
        assert sa[k].shape == sb[k].shape, k
        assert sa[k].dtype == sb[k].dtype, k


@pytest.mark.parametrize("name", ["SelfAttentionHead", "CrossAttentionHead", "MultiheadSelfAttention",
                                  "MultiheadCrossAttention"])
def test_attention_signatures(ref, name):
    r = getattr(ref.attention, name)
    n = getattr(A, name)
    assert _sig(r.__init__) == _sig(n.__init__)
    assert _sig(r.forward) == _sig(n.forward)


@pytest.mark.parametrize("name", ["TransformerEncoder", "TransformerDecoder", "TransformerCrossDecoder"])
def test_block_signatures(ref, name):
    r = getattr(ref.transformer, name)
    n = getattr(T, name)
    assert _sig(r.__init__) == _sig(n.__init__)
    assert _sig(r.forward) == _sig(n.forward)


@pytest.mark.parametrize("H,E", [(2, 8), (3, 12), (4, 10)])
def test_encoder_parity(ref, H, E):
    torch.manual_seed(0)
    r = ref.transformer.TransformerEncoder(H, E).eval()
    n = T.TransformerEncoder(H, E).eval()
    _same_keys(r, n)
    _copy(r, n)
    x = torch.randn(3, 7, E)
    torch.testing.assert_close(n(x), r(x), atol=ATOL, rtol=1e-5)
    if E % H == 0:  # the reference's return_kv path crashes otherwise (z width != E)
        yr, kr, vr = r(x, return_kv=True)
        yn, kn, vn = n(x, return_kv=True)
        for a, b in ((yn, yr), (kn, kr), (vn, vr)):
            torch.testing.assert_close(a, b, atol=ATOL, rtol=1e-5)
    # unbatched and extra leading dims
    x2 = torch.randn(5, E)
    torch.testing.assert_close(n(x2), r(x2), atol=ATOL, rtol=1e-5)
    x4 = torch.randn(2, 2, 5, E)
    torch.testing.assert_close(n(x4), r(x4), atol=ATOL, rtol=1e-5)


def test_encoder_bias_options(ref):
    torch.manual_seed(1)
    kw = dict(ffn_bias=False, ffn_hidden_size=20, head_bias=True, proj_bias=False, p_dropout=0.0)
    r = ref.transformer.TransformerEncoder(2, 8, **kw).eval()
    n = T.TransformerEncoder(2, 8, **kw).eval()
    _same_keys(r, n)
    _copy(r, n)
    x = torch.randn(2, 6, 8)
    torch.testing.assert_close(n(x), r(x), atol=ATOL, rtol=1e-5)


def test_decoder_parity_noncausal_mask(ref):
    torch.manual_seed(2)
    r = ref.transformer.TransformerDecoder(2, 8, context_size=16).eval()
    n = T.TransformerDecoder(2, 8, context_size=16).eval()
    _same_keys(r, n)
    assert list(n.state_dict())[0] == "_attn_mask"
    _copy(r, n)
    x = torch.randn(3, 9, 8)
    torch.testing.assert_close(n(x), r(x), atol=ATOL, rtol=1e-5)
    # Q2: the additive 0/1 mask is NOT causal — a future token changes position 0
    x2 = x.clone()
    x2[:, -1] += 1.0
    assert not torch.allclose(n(x)[:, 0], n(x2)[:, 0])


def test_decoder_bf16_buffer_accepted():
    # Q3 deviation: the reference raises TypeError after .to(bf16); we accept any float mask
    n = T.TransformerDecoder(2, 8, context_size=8).eval().to(torch.bfloat16)
    y = n(torch.randn(1, 4, 8, dtype=torch.bfloat16))
    assert y.dtype == torch.bfloat16 and torch.isfinite(y.float()).all()


def test_cross_decoder_parity(ref):
    torch.manual_seed(3)
    re = ref.transformer.TransformerEncoder(2, 8).eval()
    rd = ref.transformer.TransformerCrossDecoder(2, 8, context_size=12).eval()
    ne = T.TransformerEncoder(2, 8).eval()
    nd = T.TransformerCrossDecoder(2, 8, context_size=12).eval()
    _same_keys(rd, nd)
    _copy(re, ne)
    _copy(rd, nd)
    src, tgt = torch.randn(2, 10, 8), torch.randn(2, 6, 8)
    _, kr, vr = re(src, return_kv=True)
    _, kn, vn = ne(src, return_kv=True)
    torch.testing.assert_close(nd(tgt, kn, vn), rd(tgt, kr, vr), atol=ATOL, rtol=1e-5)


def test_heads_parity(ref):
    torch.manual_seed(4)
    for cls in ("SelfAttentionHead",):
        r = getattr(ref.attention, cls)(8, 4).eval()
        n = getattr(A, cls)(8, 4).eval()
        _same_keys(r, n)
        _copy(r, n)
        x = torch.randn(2, 5, 8)
        torch.testing.assert_close(n(x), r(x), atol=ATOL, rtol=1e-5)
        zr, kr, vr = r(x, None, True)
        zn, kn, vn = n(x, None, True)
        torch.testing.assert_close(zn, zr, atol=ATOL, rtol=1e-5)
        torch.testing.assert_close(kn, kr, atol=ATOL, rtol=1e-5)
        assert n.embeddings_size == r.embeddings_size and n.head_size == r.head_size
    r = ref.attention.CrossAttentionHead(8, 4).eval()
    n = A.CrossAttentionHead(8, 4).eval()
    _copy(r, n)
    x, k, v = torch.randn(2, 5, 8), torch.randn(2, 7, 4), torch.randn(2, 7, 4)
    torch.testing.assert_close(n(x, k, v), r(x, k, v), atol=ATOL, rtol=1e-5)


def test_masks(ref):
    torch.manual_seed(5)
    r = ref.attention.MultiheadSelfAttention(2, 4, 8).eval()
    n = A.MultiheadSelfAttention(2, 4, 8).eval()
    _copy(r, n)
    x = torch.randn(2, 6, 8)
    bmask = torch.triu(torch.ones(6, 6, dtype=torch.bool), 1)
    torch.testing.assert_close(n(x, mask=bmask), r(x, mask=bmask), atol=ATOL, rtol=1e-5)
    fmask = torch.randn(2, 6, 6)
    torch.testing.assert_close(n(x, mask=fmask), r(x, mask=fmask), atol=ATOL, rtol=1e-5)
    with pytest.raises(TypeError):
        n(x, mask=torch.ones(6, 6, dtype=torch.int32))


def test_mhca_parity(ref):
    torch.manual_seed(6)
    r = ref.attention.MultiheadCrossAttention(2, 4, 8).eval()
    n = A.MultiheadCrossAttention(2, 4, 8).eval()
    _same_keys(r, n)
    _copy(r, n)
    x, k, v = torch.randn(2, 5, 8), torch.randn(2, 7, 8), torch.randn(2, 7, 8)
    torch.testing.assert_close(n(x, k, v), r(x, k, v), atol=ATOL, rtol=1e-5)
    # Q6: return_kv works here (reference crashes)
    z, kk, vv = n(x, k, v, return_kv=True)
    assert z.shape == (2, 5, 8) and kk.shape == k.shape


def test_head_dropout_quirk():
    # Q4: head dropout stays 0.1 regardless of the block's p_dropout
    n = T.TransformerEncoder(2, 8, p_dropout=0.0)
    ps = [m.p for m in n.modules() if isinstance(m, torch.nn.Dropout)]
    assert ps == [0.1, 0.1, 0.0, 0.0]


def test_properties(ref):
    r = ref.transformer.TransformerEncoder(3, 12)
    n = T.TransformerEncoder(3, 12)
    for p in ("embedding_size", "head_size", "n_heads"):
        assert getattr(n, p) == getattr(r, p)
    assert n._ffn.hidden_size == r._ffn.hidden_size
    assert n._attn.head_size == r._attn.head_size


def test_train_mode_backward_runs():
    n = T.TransformerDecoder(2, 8, context_size=8).train()
    y = n(torch.randn(2, 8, 8))
    y.sum().backward()
    assert all(p.grad is not None for p in n.parameters())


def test_compat_import_paths():
    from replicann.arch.transformer import TransformerEncoder
    from replicann.nn.attention import MultiheadSelfAttention

    assert TransformerEncoder is T.TransformerEncoder
    assert MultiheadSelfAttention is A.MultiheadSelfAttention
