"""ops.conv.GradJoin (ResNet shortcut gradients summed inside the second producing kernel): the
first node to run parks its gradient and returns None, the second returns the sum — in either
order, and the result equals autograd's own sum.  CPU: two toy autograd nodes stand in for conv1
and the shortcut (the GPU kernels' accumulate paths are covered by tests/test_resnet_join_gpu.py)."""

import torch

from replicann_amd.ops.conv import GradJoin


class _Scale(torch.autograd.Function):
    """y = a·x whose backward settles its input gradient through a join."""

    @staticmethod
    def forward(ctx, x, a, join):
        ctx.a, ctx.join = a, join
        return x * a

    @staticmethod
    def backward(ctx, g):
        gx = g * ctx.a
        return (ctx.join.settle(gx) if ctx.join is not None else gx), None, None


def _grads(use_join, order):
    x = torch.randn(5, 3, generator=torch.Generator().manual_seed(0)).requires_grad_()
    j = GradJoin() if use_join else None
    y1 = _Scale.apply(x, 2.0, j)
    y2 = _Scale.apply(x, -3.0, j)
    # the two branches reach the loss through chains of different length: vary which runs first
    if order:
        y1 = y1 * 1.5 + 0.0
    else:
        y2 = y2 * 1.5 + 0.0
    (y1.sum() * 0.5 + (y2 ** 2).sum()).backward()
    assert j is None or j.g is None  # nothing left parked
    return x.grad


def test_join_equals_autograd_sum_in_both_orders():
    for order in (False, True):
        assert torch.allclose(_grads(True, order), _grads(False, order))


def test_take_and_settle():
    j = GradJoin()
    assert j.take() is None
    a = torch.ones(3)
    assert j.settle(a) is None and j.g is a
    out = j.settle(torch.full((3,), 2.0))
    assert torch.equal(out, torch.full((3,), 3.0)) and j.g is None
    assert j.settle(None) is None and j.g is None
