"""T3 model smoke tests: CPU (ATen path) always; GPU (HIP kernels) when available."""

import pytest
import torch

import replicann_amd as R
from replicann_amd.training import TrainConfig, Trainer, build_model


def _lm_batch(cfg, B=2, T=32, dev="cpu"):
    x = torch.randint(0, cfg.vocab_size, (B, T + 1), device=dev)
    return x[:, :-1], x[:, 1:]


@pytest.mark.parametrize("name", ["gpt2-tiny", "vit-tiny", "resnet18-tiny", "mlp", "refblock-lm"])
def test_model_cpu_fwd_bwd(name):
    torch.manual_seed(0)
    m = build_model(name)
    if name.startswith("gpt2") or name == "refblock-lm":
        x, y = _lm_batch(m.config)
    elif name == "mlp":
        x, y = torch.rand(4, 784), torch.randint(0, 10, (4,))
    else:
        size = m.config.image_size if hasattr(m, "config") else 32
        x, y = torch.randn(2, size, size, 3), torch.randint(0, 10, (2,))
    loss = m(x, y)
    assert torch.isfinite(loss)
    loss.backward()
    assert all(p.grad is not None and torch.isfinite(p.grad).all() for p in m.parameters() if p.requires_grad)


def test_refblock_lm_trains_and_keeps_reference_layout():
    """The reference-block token model: its blocks are the reference's TransformerDecoder (state_dict
    keys as in the reference), head dropout 0.1 is active in train mode, and the loss falls."""
    m = build_model("refblock-lm", n_layer=1, n_head=4, n_embd=64, block_size=32)
    keys = [k for k in m.state_dict() if k.startswith("blocks.0.")]
    assert "blocks.0._attn._heads.0._query.weight" in keys and "blocks.0._attn_mask" in keys
    tr = Trainer(TrainConfig(model="refblock-lm", steps=30, batch_size=8, seq_len=32, lr=3e-3, device="cpu",
                             log_every=1000, model_kwargs=dict(n_layer=1, n_head=4, n_embd=64, block_size=32)))
    first = float(tr.step())
    assert tr.model.training and tr.model.blocks[0]._attn._heads[0]._dropout.p == 0.1
    out = tr.run()
    assert out["final_loss"] < first


def test_gpt2_param_count():
    m = R.GPT2(R.GPT2Config.small())
    assert abs(m.num_params() - 124.4e6) < 0.1e6
    m = R.GPT2(R.GPT2Config.medium())
    assert abs(m.num_params() - 354.8e6) < 0.5e6


def test_mlp_trains_on_cpu(tmp_path):
    cfg = TrainConfig(model="mlp", batch_size=64, steps=60, lr=3e-3, weight_decay=0.0, warmup_steps=1,
                      device="cpu", log_every=1000, metrics_path=str(tmp_path / "m.jsonl"),
                      checkpoint=str(tmp_path / "ck.pt"))
    tr = Trainer(cfg)
    first = float(tr.step(cfg.lr))
    out = tr.run()
    assert out["final_loss"] < first * 0.7
    # resume: restores the step and the weights
    cfg2 = TrainConfig(model="mlp", batch_size=64, steps=61, device="cpu", resume=str(tmp_path / "ck.pt"))
    tr2 = Trainer(cfg2)
    assert tr2.step_idx == 60
    for a, b in zip(tr.model.parameters(), tr2.model.parameters()):
        assert torch.equal(a.detach(), b.detach())


def test_evaluate_api():
    from replicann_amd.utils.data import SyntheticMNIST
    m = R.MLP()
    out = R.evaluate(m, SyntheticMNIST(32), steps=2)
    assert 0 <= out["accuracy"] <= 1 and out["loss"] > 0


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("name", ["gpt2-tiny", "vit-tiny", "resnet18-tiny"])
def test_model_gpu_fwd_bwd(cuda, name):
    torch.manual_seed(0)
    cfg = TrainConfig(model=name, batch_size=4, seq_len=64, steps=6, lr=1e-3, warmup_steps=1, log_every=1000)
    tr = Trainer(cfg)
    losses = [float(tr.step(cfg.lr)) for _ in range(6)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0]


@pytest.mark.gpu
def test_gpt2_gpu_matches_cpu_forward(cuda):
    torch.manual_seed(1)
    m = R.GPT2(R.GPT2Config.tiny(n_embd=256, n_head=4))  # head_dim 64 -> fast attention path
    x, y = _lm_batch(m.config, B=2, T=128)
    with torch.no_grad():
        ref = m(x, y).item()
        mg = m.cuda().to(torch.bfloat16)
        out = mg(x.cuda(), y.cuda()).item()
    assert abs(out - ref) / ref < 2e-2


@pytest.mark.gpu
def test_reference_blocks_gpu_match_cpu(cuda):
    from replicann_amd.arch.transformer import TransformerCrossDecoder, TransformerDecoder, TransformerEncoder
    torch.manual_seed(2)
    for blk, args in ((TransformerEncoder, {}), (TransformerDecoder, {"context_size": 64})):
        m = blk(4, 256, **args).eval()
        x = torch.randn(2, 40, 256)
        with torch.no_grad():
            ref = m(x)
            out = m.cuda().to(torch.bfloat16)(x.cuda().to(torch.bfloat16))
        assert ((out.float().cpu() - ref).norm() / ref.norm()).item() < 3e-2
    enc = TransformerEncoder(2, 64).eval()
    dec = TransformerCrossDecoder(2, 64, context_size=32).eval()
    src, tgt = torch.randn(2, 20, 64), torch.randn(2, 12, 64)
    with torch.no_grad():
        _, k, v = enc(src, return_kv=True)
        ref = dec(tgt, k, v)
        enc.cuda().to(torch.bfloat16)
        dec.cuda().to(torch.bfloat16)
        _, kg, vg = enc(src.cuda().to(torch.bfloat16), return_kv=True)
        out = dec(tgt.cuda().to(torch.bfloat16), kg, vg)
    assert ((out.float().cpu() - ref).norm() / ref.norm()).item() < 5e-2


@pytest.mark.gpu
def test_reference_block_train_step_gpu(cuda):
    from replicann_amd.arch.transformer import TransformerDecoder
    m = TransformerDecoder(4, 256, context_size=64).cuda().to(torch.bfloat16).train()
    y = m(torch.randn(2, 64, 256, device="cuda", dtype=torch.bfloat16))
    y.float().pow(2).mean().backward()
    assert all(p.grad is not None and torch.isfinite(p.grad.float()).all() for p in m.parameters())


@pytest.mark.gpu
def test_direct_grad_accumulation_matches_autograd(cuda):
    """Flat-buffer direct accumulation (kernels write .grad) == plain autograd grads, incl. 2x accumulation."""
    import copy
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(3)
    m1 = R.GPT2(R.GPT2Config.tiny(n_embd=256, n_head=4)).cuda()
    for p in m1.parameters():
        p.data = p.data.to(torch.bfloat16)
    m2 = copy.deepcopy(m1)
    flat = FlatParams(m1)
    x, y = _lm_batch(m1.config, B=2, T=64, dev="cuda")
    flat.zero_grad()
    m1(x, y).backward()
    g1 = {n: p.grad.detach().float().clone() for n, p in m1.named_parameters()}
    m1(x, y).backward()  # accumulate a second time
    m2(x, y).backward()
    for n, p in m2.named_parameters():
        ref = p.grad.float()
        err = ((g1[n] - ref).norm() / (ref.norm() + 1e-6)).item()
        assert err < 2e-2, (n, err)
        err2 = ((dict(m1.named_parameters())[n].grad.float() - 2 * ref).norm() / (2 * ref.norm() + 1e-6)).item()
        assert err2 < 3e-2, (n, err2)


@pytest.mark.gpu
def test_gpt2_fp8_train_steps(cuda):
    torch.manual_seed(4)
    cfg = TrainConfig(model="gpt2-tiny", batch_size=4, seq_len=128, steps=6, lr=1e-3, warmup_steps=1,
                      log_every=1000, model_kwargs={"fp8": True, "n_embd": 256, "n_head": 4})
    tr = Trainer(cfg)
    losses = [float(tr.step()) for _ in range(6)]
    assert all(torch.isfinite(torch.tensor(losses))) and losses[-1] < losses[0]


@pytest.mark.gpu
def test_gpt2_fp8_layernorm_fed_and_tracks_bf16(cuda):
    """fp8 GPT-2 blocks: c_attn / c_fc take their e4m3 input from the LayerNorm kernel (after the
    first, current-scaling step), the attention output projection is fp8 as configured, and the loss trajectory tracks
    the bf16 model's."""
    kw = {"n_embd": 256, "n_head": 4}

    def run(fp8):
        torch.manual_seed(4)
        cfg = TrainConfig(model="gpt2-tiny", batch_size=4, seq_len=128, steps=8, lr=1e-3, warmup_steps=1,
                          log_every=1000, graph="off", model_kwargs={**kw, "fp8": fp8})
        tr = Trainer(cfg)
        return tr, [float(tr.step()) for _ in range(8)]

    tr8, l8 = run(True)
    _, l16 = run(False)
    assert tr8.fp8_cache is not None and tr8.fp8_cache.refreshes == 8  # e4m3 weights from the optimizer
    for blk in tr8.model.h:
        assert blk.attn.c_attn.fp8_state.wcache is tr8.fp8_cache
        assert blk.attn.c_attn.fp8_state.fed >= 7 and blk.mlp.c_fc.fp8_state.fed >= 7
        assert blk.mlp.c_proj.fp8_state.fed >= 7  # from c_fc's GEMM epilogue
        # the attention output projection: fp8 with its own quantisation pass iff GPT2Config.fp8_proj
        assert (blk.attn.c_proj.fp8_state is not None) == tr8.model.config.fp8_proj
    assert all(abs(a - b) < 0.05 * abs(b) for a, b in zip(l8, l16)), (l8, l16)
