"""ResNet BasicBlock input gradient with the shortcut join (ops.conv.GradJoin): x's two gradients —
conv1's dgrad and the shortcut's (identity: the BatchNorm residual gradient; downsample: the 1×1
stride-2 conv's dgrad) — are summed inside the second producing kernel (implicit dgrad GEMM
epilogue accumulate, or the col2im gather's accumulate) instead of by an autograd add.

Checked against the same block without the join and against an fp32 reference block, for the
identity block (stride-1 implicit dgrad accumulate) and the downsample block (col2im accumulate),
and that no ATen add kernel is left in the backward."""

import pytest
import torch

from replicann_amd.models.resnet import BasicBlock

pytestmark = pytest.mark.gpu


def _run(blk, x):
    x = x.clone().requires_grad_()
    blk.zero_grad(set_to_none=True)
    blk(x).float().square().mean().backward()
    return x.grad.float(), {n: p.grad.float() for n, p in blk.named_parameters()}


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize("cin,cout,stride", [(64, 64, 1), (64, 128, 2), (128, 128, 1)])
def test_block_input_grad_with_join(cuda, cin, cout, stride):
    torch.manual_seed(5)
    blk = BasicBlock(cin, cout, stride).cuda()
    ref = BasicBlock(cin, cout, stride)
    ref.load_state_dict(blk.state_dict())
    for p in blk.parameters():
        p.data = p.data.bfloat16()
    x = torch.randn(4, 16, 16, cin, device=cuda).bfloat16()
    gx_j, gp_j = _run(blk, x)
    blk.join_grads = False
    gx_n, gp_n = _run(blk, x)
    # fp32 reference on the CPU path (F.conv2d / F.batch_norm, autograd's own sum)
    xr = x.float().cpu().requires_grad_()
    ref(xr).square().mean().backward()
    assert _rel(gx_j, gx_n) < 1e-2
    # against fp32 the joined gradient is as accurate as the unjoined one (both ≈ 2 % in bf16)
    e_j, e_n = _rel(gx_j.cpu(), xr.grad), _rel(gx_n.cpu(), xr.grad)
    assert e_j < 4e-2 and e_j < 1.1 * e_n + 2e-3, (e_j, e_n)
    for n in gp_j:
        assert _rel(gp_j[n], gp_n[n]) < 1e-2, n


def test_no_aten_add_in_block_backward(cuda):
    torch.manual_seed(6)
    blk = BasicBlock(64, 64, 1).cuda()
    for p in blk.parameters():
        p.data = p.data.bfloat16()
    x = torch.randn(2, 8, 8, 64, device=cuda).bfloat16().requires_grad_()
    y = blk(x).float().square().mean()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        y.backward()
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    assert not any("CUDAFunctor_add" in n for n in names), names
