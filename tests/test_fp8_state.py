"""fp8 delayed-scaling state is persistent: the per-layer scale / amax slots are module
buffers — saved and loaded with the state_dict, rolled back by the trainer's autotuning pass — and
the host-side ready flags follow the loaded tensors."""

import pytest
import torch

import replicann_amd as R
from replicann_amd.ops.fp8 import fp8_states


def _model(head=0):
    """fp8 GPT-2 tiny; the fp8 LM head (GPU-only) off unless ``head``."""
    torch.manual_seed(0)
    return R.GPT2(R.GPT2Config.tiny(fp8=True, fp8_head=head))


def test_fp8_scales_are_state_dict_buffers():
    m = _model(head=1)
    keys = [k for k in m.state_dict() if k.endswith("fp8_scales")]
    # c_attn, c_fc, mlp c_proj (+ attention c_proj with fp8_proj) per block + the fp8 LM head's slots (fp8_head)
    per_block = 4 if m.config.fp8_proj else 3
    assert len(keys) == per_block * m.config.n_layer + (1 if m.config.fp8_head else 0)
    ids = torch.randint(0, 1000, (2, 32))
    m(ids, ids)  # first quantisation: current scaling fills the slots
    head = m.head8.fp8_state if m.head8 is not None else None
    sts = [st for st in fp8_states(m) if st is not head]  # the fp8 LM head runs on the GPU only
    assert all(st.ready == [True, True] for st in sts)
    m2 = _model(head=1)
    assert not any(any(st.ready) for st in fp8_states(m2))
    m2.load_state_dict(m.state_dict())
    for a, b in zip(fp8_states(m), fp8_states(m2)):
        assert torch.equal(a.t, b.t) and b.ready == a.ready


@pytest.mark.gpu
def test_fp8_resume_bitwise_gpu(cuda, tmp_path):
    from replicann_amd.training import TrainConfig, Trainer

    kw = dict(model="gpt2-tiny", model_kwargs={"fp8": True}, batch_size=4, seq_len=128, steps=100,
              warmup_steps=1, lr=1e-3, log_every=10**9, seed=5, graph="off")
    a = Trainer(TrainConfig(**kw))
    for _ in range(3):
        a.step()
    ck = str(tmp_path / "fp8.pt")
    a.save(ck)
    la = [float(a.step()) for _ in range(3)]
    b = Trainer(TrainConfig(**kw, resume=ck))
    lb = [float(b.step()) for _ in range(3)]
    assert la == lb


def test_fp8_checkpoint_without_scales_loads_strict():
    """A state_dict written before the fp8_scales buffer existed loads with strict=True: the
    missing slots start empty (current scaling on the first call) instead of raising."""
    m = _model()
    old = {k: v for k, v in m.state_dict().items() if not k.endswith("fp8_scales")}
    m2 = _model()
    for st in fp8_states(m2):
        st.t.fill_(3.0)
    m2.load_state_dict(old, strict=True)
    assert all(not any(st.ready) for st in fp8_states(m2))
    assert all(float(st.t.abs().sum()) == 0.0 for st in fp8_states(m2))


def test_fp8_wgrad_cpu_emulation_tracks_bf16_grads():
    """fp8 weight gradients (e5m2 dY x the forward's e4m3 input) on the CPU emulation path: every
    fp8 layer's weight gradient stays within fp8 tolerance of the unquantised one, and the gradient
    slots fill (current scaling first, delayed after)."""
    ids = torch.randint(0, 1000, (4, 32), generator=torch.Generator().manual_seed(1))  # 128 tokens
    grads = {}
    for wg in (False, True):
        m = _model()
        for st in fp8_states(m):
            st.wgrad = wg
        m(ids, ids).backward()
        grads[wg] = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        if wg:
            assert all(st.g_ready for st in fp8_states(m))
            assert all(float(st.gt[0, 0]) > 0 for st in fp8_states(m))
    fp8_w = [n for n in grads[True] if any(k in n for k in ("c_attn.weight", "c_fc.weight", "mlp.c_proj.weight"))]
    assert fp8_w
    for n in fp8_w:
        a, b = grads[True][n].float(), grads[False][n].float()
        assert ((a - b).norm() / b.norm()) < 0.1, n


def test_fp8_dgrad_cpu_emulation_tracks_bf16_grads():
    """fp8 data gradients (e5m2 dY x the forward's e4m3 weight, the weight read transposed) with
    fp8 weight gradients on the CPU emulation path: the input-side gradients (embeddings, LayerNorm
    parameters — everything upstream of an fp8 dgrad) stay within fp8 tolerance of the bf16 path, and
    dY is quantised once per layer for both gradients (one gradient-slot roll per backward)."""
    ids = torch.randint(0, 1000, (4, 32), generator=torch.Generator().manual_seed(1))
    grads = {}
    for mode in ("bf16", "fp8"):
        m = _model()
        for st in fp8_states(m):
            st.wgrad = st.dgrad = mode == "fp8"
        m(ids, ids).backward()
        grads[mode] = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
        if mode == "fp8":
            assert all(st.g_ready for st in fp8_states(m))
    assert set(grads["fp8"]) == set(grads["bf16"])
    for n in grads["fp8"]:
        a, b = grads["fp8"][n].float(), grads["bf16"][n].float()
        assert ((a - b).norm() / b.norm().clamp_min(1e-12)) < 0.15, n


def test_fp8_head_slots_checkpoint_compat():
    """The fp8 LM head's slots (GPT2Config.fp8_head) are a state_dict buffer; a checkpoint written without
    them (bf16 head, or an older fp8 model) loads strictly into a head model with empty slots, and the CPU
    path ignores the fp8 head (plain fp32 loss)."""
    from replicann_amd import ops
    from replicann_amd.ops.fp8 import Fp8State

    m_head = _model(head=1)
    assert "head8.fp8_scales" in m_head.state_dict()
    m_plain = _model(head=0)
    assert "head8.fp8_scales" not in m_plain.state_dict()
    m_head.load_state_dict(m_plain.state_dict())  # strict: the missing head slots are filled, not an error
    assert m_head.head8.fp8_state.ready == [False, False]
    torch.manual_seed(2)
    h = torch.randn(64, 128)
    w = torch.randn(1024, 128) * 0.05
    t = torch.randint(0, 1000, (64,))
    a = ops.linear_cross_entropy(h, w, t, n_valid_cols=1000, fp8=Fp8State())
    b = ops.linear_cross_entropy(h, w, t, n_valid_cols=1000)
    assert torch.equal(a, b)


def test_fp8_head_checkpoint_loads_into_model_without_head():
    """the other direction — a checkpoint with the fp8 head's slots loads strictly into a
    model built with fp8_head=0 (the slots are dropped, not an unexpected-key error)."""
    m_head = _model(head=1)
    m_plain = _model(head=0)
    m_plain.load_state_dict(m_head.state_dict())  # strict
    for k, v in m_plain.state_dict().items():
        assert torch.equal(v, m_head.state_dict()[k]), k


def test_fp8_config_env_defaults_resolved_at_construction(monkeypatch):
    """The fp8_head / fp8_proj defaults follow the environment when the config is BUILT (not at import)."""
    monkeypatch.setenv("REPLICANN_FP8_HEAD", "0")
    monkeypatch.setenv("REPLICANN_FP8_PROJ", "0")
    cfg = R.GPT2Config.tiny(fp8=True)
    assert cfg.fp8_head == 0 and cfg.fp8_proj is False
    monkeypatch.setenv("REPLICANN_FP8_HEAD", "2")
    assert R.GPT2Config.tiny(fp8=True).fp8_head == 2
    assert R.GPT2Config.tiny(fp8=True, fp8_head=1).fp8_head == 1


def test_fp8_non_pow2_scales_are_rounded_on_load():
    """a checkpoint whose slots hold non-power-of-two scales (written before every
    quantiser rounded up) loads with every positive scale rounded UP to a power of two — the one-wave fp8
    GEMM feeds only the exponent byte to the scaled MFMA — and power-of-two scales load unchanged."""
    m = _model()
    ids = torch.randint(0, 1000, (2, 32))
    m(ids, ids)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    keys = [k for k in sd if k.endswith("fp8_scales")]
    pow2 = {k: sd[k].clone() for k in keys}
    for k in keys:
        sd[k][:, 0] = sd[k][:, 0] * 0.75  # no longer powers of two
    m2 = _model()
    m2.load_state_dict(sd)
    for k, t in m2.state_dict().items():
        if k.endswith("fp8_scales"):
            s = t[:, 0]
            m_, _ = torch.frexp(s[s > 0])
            assert torch.all(m_ == 0.5), (k, s)
            assert torch.all(s >= sd[k][:, 0])  # rounded up, never down (no overflow of the e4m3 range)
            assert torch.equal(s, pow2[k][:, 0])  # 0.75 · 2^e rounds back to 2^e
    m3 = _model()
    m3.load_state_dict(m.state_dict())  # pow2 scales: unchanged, bit for bit
    for k in keys:
        assert torch.equal(m3.state_dict()[k], m.state_dict()[k])
