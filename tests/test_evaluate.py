"""``replicann.evaluate``: LMs are scored through their own fused loss path, classifiers through the
native cross-entropy; both must equal the plain fp32 definition of the mean token / sample loss."""

import pytest
import torch
import torch.nn.functional as F

import replicann_amd as R
from replicann_amd.training import evaluate


class _Batches:
    def __init__(self, batches):
        self.b = list(batches)

    def __next__(self):
        return self.b.pop(0)


def _lm_ref(model, batches):
    tot = n = 0.0
    for x, y in batches:
        logits = model(x).float()
        tot += float(F.cross_entropy(logits.reshape(-1, logits.shape[-1]), y.reshape(-1), reduction="sum"))
        n += y.numel()
    return tot / n


def _check_lm(dev, tol):
    torch.manual_seed(0)
    m = R.GPT2(R.GPT2Config.tiny()).to(dev)
    if dev.type == "cuda":
        m = m.to(torch.bfloat16)
    batches = [(torch.randint(0, 1000, (2, 32), device=dev), torch.randint(0, 1000, (2, 32), device=dev))
               for _ in range(3)]
    with torch.no_grad():
        want = _lm_ref(m.eval(), batches)
    got = evaluate(m, _Batches(batches), steps=3)
    assert abs(got["loss"] - want) < tol * max(1.0, want), (got, want)


def test_evaluate_lm_cpu():
    _check_lm(torch.device("cpu"), 1e-5)


def test_evaluate_classifier_cpu():
    torch.manual_seed(0)
    m = R.MLP()
    batches = [(torch.randn(8, 784), torch.randint(0, 10, (8,))) for _ in range(2)]
    with torch.no_grad():
        tot = sum(float(F.cross_entropy(m(x), y, reduction="sum")) for x, y in batches)
        cor = sum(int((m(x).argmax(-1) == y).sum()) for x, y in batches)
    got = evaluate(m, _Batches(batches), steps=2)
    assert abs(got["loss"] - tot / 16) < 1e-5 and abs(got["accuracy"] - cor / 16) < 1e-9


@pytest.mark.gpu
def test_evaluate_lm_gpu_native(cuda):
    _check_lm(cuda, 2e-2)
