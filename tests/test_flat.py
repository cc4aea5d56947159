"""CPU tests of the flat-buffer gradient plumbing (direct accumulation bookkeeping)."""

import torch

from replicann_amd.ops.linear import _direct_grad, _notify
from replicann_amd.utils.flat import FlatParams


def _module():
    m = torch.nn.Module()
    m.a = torch.nn.Parameter(torch.randn(8, 4))
    m.tied = torch.nn.Parameter(torch.randn(16, 4))
    m.shared = torch.nn.Parameter(torch.randn(3))
    m.tied._rn_shared = True
    m.tied._rn_direct_uses = 2
    m.shared._rn_shared = True
    return m


def test_views_alignment_and_direct_eligibility():
    m = _module()
    flat = FlatParams(m)
    for p, off, n in flat.segments():
        assert off % 64 == 0
        assert p.data.data_ptr() == flat.data[off:].data_ptr()
        assert p.grad.data_ptr() == flat.grad[off:].data_ptr()
    assert _direct_grad(m.a) is m.a.grad
    assert _direct_grad(m.tied) is m.tied.grad      # shared, but declares its contributions
    assert _direct_grad(m.shared) is None           # shared without a contribution count
    flat.direct = False
    assert _direct_grad(m.a) is None


def test_multi_use_parameter_marked_ready_after_last_contribution():
    m = _module()
    flat = FlatParams(m)
    seen = []
    flat.ready_hooks.append(lambda p: seen.append(flat.names[id(p)]))
    _notify(m.a)
    assert seen == ["a"]
    _notify(m.tied)
    assert seen == ["a"]                            # 1 of 2
    _notify(m.tied)
    assert seen == ["a", "tied"]                    # 2 of 2
    _notify(m.tied)                                 # next micro-batch starts a new count
    flat.zero_grad()                                # ... and zero_grad resets a partial count
    _notify(m.tied)
    _notify(m.tied)
    assert seen == ["a", "tied", "tied"]


def test_wd_mask_matrices_only():
    m = _module()
    flat = FlatParams(m)
    wd = flat.wd_mask.cpu()
    for p, off, n in flat.segments():
        assert int(wd[off // 64]) == (1 if p.dim() >= 2 else 0)


def test_optimizer_state_remapped_across_flat_layouts():
    """optimizer master / moments are raw flat tensors; a checkpoint taken under another
    packing (here: the reference MHSA's fused Q/K/V group disabled) must land on the same NAMED
    parameters, not be read permuted."""
    import replicann_amd as R
    from replicann_amd.optim import FusedAdamW

    torch.manual_seed(0)
    a = R.TransformerEncoder(n_heads=2, embedding_size=16)
    fa = FlatParams(a)
    oa = FusedAdamW(fa, lr=1e-2)
    for p in fa.params:
        p.grad.copy_(torch.randn_like(p))
    oa.step()
    sd = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in oa.state_dict().items()}

    torch.manual_seed(0)
    b = R.TransformerEncoder(n_heads=2, embedding_size=16)
    for mod in b.modules():  # another packing: no fusion groups
        if hasattr(mod, "_rn_fuse_groups"):
            mod._rn_fuse_groups = lambda: []
    fb = FlatParams(b)
    assert fb.layout() != fa.layout()
    ob = FusedAdamW(fb, lr=1e-2)
    ob.load_state_dict(sd)
    names_a = {fa.names[id(p)]: p for p in fa.params}
    for p, o, n in fb.segments():
        q = names_a[fb.names[id(p)]]
        qo = fa.span(q)[0]
        assert torch.equal(ob.m[o:o + n], oa.m[qo:qo + n])
        assert torch.equal(ob.master[o:o + n], oa.master[qo:qo + n])
