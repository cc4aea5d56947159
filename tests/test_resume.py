"""Checkpoint / resume under data parallelism (CPU, gloo, 2 ranks): a run interrupted at step 3,
checkpointed (collective save: barrier, per-rank RNG + data cursor gathered to rank 0) and resumed
in fresh Trainers reproduces the uninterrupted 6-step run bit for bit on every rank.  Also: eval
reads from window 0 whatever step the checkpoint is from; per-phase metrics land in the JSONL."""

import json
import os
import socket

import numpy as np
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, ck, metrics, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist
    from replicann_amd.training import TrainConfig, Trainer
    try:
        base = dict(model="mlp", steps=6, device="cpu", batch_size=8, log_every=2, lr=5e-3, warmup_steps=2)
        full = Trainer(TrainConfig(**base, metrics_path=metrics))
        full.run()
        p_full = full.flat.data.clone()
        torch.manual_seed(999)  # disturb the RNG: the resumed run must restore its own
        part = Trainer(TrainConfig(**base, seed=0))
        for _ in range(3):
            part.step()
        part.save(ck)
        res = Trainer(TrainConfig(**base, resume=ck))
        assert res.step_idx == 3
        res.run()
        q.put((rank, p_full.numpy(), res.flat.data.clone().numpy()))
    finally:
        dist.destroy_process_group()


def test_ddp_resume_bitwise_gloo(tmp_path):
    world = 2
    ck = str(tmp_path / "ck.pt")
    metrics = str(tmp_path / "m.jsonl")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, ck, metrics, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, full, resumed in res:
        np.testing.assert_array_equal(full, resumed)
    np.testing.assert_array_equal(res[0][1], res[1][1])
    sd = torch.load(ck, weights_only=True)
    assert len(sd["ranks"]) == world and all("data" in r for r in sd["ranks"])
    assert sd["ranks"][0]["data"]["i"] == 3 and sd["step"] == 3
    rows = [json.loads(line) for line in open(metrics)]
    assert rows and all("forward_ms" in r and "backward_ms" in r and "allreduce_wait_ms" in r for r in rows)


def test_eval_starts_at_window_zero_after_checkpoint(tmp_path):
    """evaluating a step-S checkpoint must read eval window 0 first (it used to start at
    window S·grad_accum), so two checkpoints of one run are scored on the same windows."""
    from replicann_amd.training import TrainConfig, Trainer
    from replicann_amd.utils.token_data import write_token_shard
    shard = write_token_shard(tmp_path / "t.bin", np.arange(20000) % 1000)
    base = dict(model="gpt2-tiny", device="cpu", batch_size=2, seq_len=32, data=str(shard), log_every=100,
                model_kwargs={"vocab_size": 1000, "vocab_pad": 1024})
    tr = Trainer(TrainConfig(steps=3, **base))
    tr.run()
    ck = str(tmp_path / "ck.pt")
    tr.save(ck)
    ev = Trainer(TrainConfig(steps=1, resume=ck, data_mode="eval", graph="off", **base))
    fresh = Trainer(TrainConfig(steps=1, data_mode="eval", graph="off", **base))
    x1, _ = next(ev.data)
    x2, _ = next(fresh.data)
    assert torch.equal(x1, x2)
    assert int(x1[0, 0]) == 0  # window 0 of a 0,1,2,... shard
    # and the TRAIN resume continues the saved cursor (any grad_accum)
    tr2 = Trainer(TrainConfig(steps=3, resume=ck, grad_accum=2, **base))
    assert tr2.data.batch_index == tr.data.batch_index


def test_resume_with_other_world_size_is_refused(tmp_path):
    import pytest
    import torch

    from replicann_amd.models import MLP
    from replicann_amd.utils.checkpoint import load_checkpoint, rank_state, save_checkpoint

    m = MLP()
    ck = str(tmp_path / "w2.pt")
    save_checkpoint(ck, m, step=3)
    sd = torch.load(ck, weights_only=True)
    sd["ranks"] = [rank_state(), rank_state()]  # as if two ranks had saved it
    sd["world_size"] = 2
    torch.save(sd, ck)
    with pytest.raises(RuntimeError, match="saved by 2 rank"):
        load_checkpoint(ck, MLP())
    with pytest.warns(UserWarning, match="per-rank streams start fresh"):
        step, _, mine = load_checkpoint(ck, MLP(), allow_world_change=True)
    assert step == 3 and mine is None
