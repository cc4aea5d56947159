"""CPU side of the collective back-ends (replicann_amd/parallel/comm.py): back-end selection
and the one-rank DDP rehearsal (``ddp="on"``) over a gloo process group."""

import socket

import pytest
import torch
import torch.distributed as dist


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_make_comm_selection():
    from replicann_amd.parallel.comm import TorchComm, make_comm

    assert isinstance(make_comm("auto"), TorchComm)  # no process group: torch (world 1)
    assert isinstance(make_comm("torch"), TorchComm)
    with pytest.raises(ValueError):
        make_comm("bogus")


def test_one_rank_ddp_rehearsal_cpu(monkeypatch):
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", str(_free_port()))
    monkeypatch.setenv("RANK", "0")
    monkeypatch.setenv("WORLD_SIZE", "1")
    from replicann_amd.training import TrainConfig, Trainer

    def run(**kw):
        cfg = TrainConfig(model="gpt2-tiny", batch_size=2, seq_len=32, steps=50, warmup_steps=1, lr=1e-3,
                          device="cpu", log_every=10**9, bucket_mb=0.05, seed=1,
                          model_kwargs=dict(n_embd=64, n_head=2, n_layer=2, block_size=32, vocab_size=256),
                          **kw)
        tr = Trainer(cfg)
        losses = [float(tr.step()) for _ in range(3)]
        return tr, losses

    try:
        base, base_l = run()
        assert base.ddp is None
        tr, l = run(ddp="on")
        assert dist.is_initialized() and dist.get_backend() == "gloo"
        assert tr.ddp is not None and tr.ddp.comm.name == "torch" and tr.ddp.active
        assert tr.ddp.launched_in_backward > 0
        assert all(abs(a - b) < 1e-4 for a, b in zip(l, base_l)), (l, base_l)
        assert torch.allclose(tr.flat.data, base.flat.data, atol=1e-5)
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()
