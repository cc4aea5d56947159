"""End-to-end numerics on the GPU (T3): whole training runs and production-size GEMMs.

* loss trajectories of the native bf16 path (HIP kernels, autotuned GEMMs,
  direct grad accumulation, fused optimizer, whole-step hipGraph) against the
  plain-ATen fp32 reference math run on the same GPU from the same init/data;
* every GEMM tile config × split-K on the exact GPT-2 / ViT training shapes
  (fwd, dgrad, wgrad-accumulate) against an fp32 matmul.
"""

import pytest
import torch

from replicann_amd import _ext, ops
from replicann_amd.training import TrainConfig, Trainer

pytestmark = pytest.mark.gpu


def _losses(model, steps, ref, graph="auto", **kw):
    kw = {"lr": 1e-3, **kw}
    cfg = TrainConfig(model=model, steps=steps, warmup_steps=2, log_every=10**9,
                      dtype="fp32" if ref else "bf16", graph="off" if ref else graph, **kw)
    out = []
    if ref:
        with _ext.reference_path():
            t = Trainer(cfg)
            for _ in range(steps):
                out.append(float(t.step()))
    else:
        t = Trainer(cfg)
        for _ in range(steps):
            out.append(float(t.step()))
    return out


@pytest.mark.parametrize("model,kw,tol", [
    ("gpt2-tiny", dict(batch_size=8, seq_len=128), 0.03),
    ("vit-tiny", dict(batch_size=32), 0.05),
    ("resnet18-tiny", dict(batch_size=32, optimizer="sgd", lr=0.05), 0.05),
])
def test_loss_trajectory_matches_fp32_reference(cuda, model, kw, tol):
    kw = dict(kw)
    steps = 12
    nat = _losses(model, steps, False, **kw)
    ref = _losses(model, steps, True, **kw)
    rel = [abs(a - b) / abs(b) for a, b in zip(nat, ref)]
    assert max(rel) < tol, list(zip(nat, ref))
    assert nat[-1] < nat[0]  # pool of fixed batches: the model must fit it


def test_graph_replay_matches_eager(cuda):
    kw = dict(batch_size=8, seq_len=128)
    g = _losses("gpt2-tiny", 6, False, graph="on", **kw)
    e = _losses("gpt2-tiny", 6, False, graph="off", **kw)
    assert max(abs(a - b) for a, b in zip(g, e)) < 2e-3, list(zip(g, e))


def test_refblock_decoder_graph_with_head_dropout(cuda):
    """the reference TransformerDecoder blocks (head dropout 0.1, train mode) train
    under a whole-step hipGraph; with the device-drawn dropout seeds the replays follow the eager run
    (same masks, same steps) and the loss falls."""
    kw = dict(batch_size=8, seq_len=64, lr=3e-3,
              model_kwargs=dict(n_layer=2, n_head=8, n_embd=256, block_size=64))
    t = Trainer(TrainConfig(model="refblock-lm", steps=8, graph="on", log_every=10**9, **kw))
    assert t.graph_enabled() and t.model.blocks[0]._attn._heads[0]._dropout.p == 0.1
    g = [float(t.step()) for _ in range(8)]
    assert t._graph is not None
    e = _losses("refblock-lm", 8, False, graph="off", **kw)
    assert max(abs(a - b) for a, b in zip(g, e)) < 2e-3, list(zip(g, e))
    assert g[-1] < g[0]


def rel_err(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


# (M tokens, N out, K in) of GPT-2 small (B16×T1024) and ViT-B/16 (B128×197)
SHAPES = [(16384, 2304, 768), (16384, 768, 768), (16384, 3072, 768), (16384, 768, 3072),
          (25216, 2304, 768), (25216, 768, 3072)]


@pytest.mark.parametrize("M,N,K", SHAPES)
def test_production_gemm_shapes_all_configs(cuda, M, N, K):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    dy = torch.randn(M, N, device="cuda").bfloat16()
    fwd = x.float() @ w.float().t()
    dgrad = dy.float() @ w.float()
    g0 = (torch.randn(N, K, device="cuda") * 10).bfloat16()
    wgrad = g0.float() + dy.float().t() @ x.float()
    for cfg in (0, 1, 2, 6, 8):
        assert rel_err(ops.gemm(x, w, tb=True, cfg=cfg), fwd) < 1e-2, cfg
        assert rel_err(ops.gemm(dy, w, cfg=cfg), dgrad) < 1e-2, cfg
        for split in (1, 2, 4, 8, 16):
            g = g0.clone()
            ops.gemm(dy, x, ta=True, out=g, accumulate=True, split_k=split, cfg=cfg)
            assert rel_err(g, wgrad) < 1e-2, (cfg, split)
