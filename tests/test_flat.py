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
