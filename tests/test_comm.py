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


class _FakeRccl:
    """Stand-in for the native comm ops on CPU: records the rendezvous the Python side performs."""

    def __init__(self, rank):
        self.rank = rank
        self.calls = []

    def comm_unique_id(self):
        return torch.arange(128, dtype=torch.uint8) ^ 0x5A  # a recognisable id from rank 0

    def comm_init(self, uid, rank, world, device, timeout_s):
        self.calls.append(("init", bytes(uid.numpy()), rank, world, device, timeout_s))
        return 7

    def comm_quiesce(self, h):
        pass


def _native_rendezvous_worker(rank, world, port, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from replicann_amd import _ext
        from replicann_amd.parallel.comm import NativeComm

        fake = _FakeRccl(rank)
        _ext.ops = lambda: fake  # the comm layer's only entry into the extension
        c = NativeComm(device=torch.device("cuda", rank))  # device index only: no GPU work on the fake
        q.put((rank, c.rank, c.world, c.handle, fake.calls))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_native_comm_rendezvous_multi_rank(world):
    """N>1 setup of the native communicator (not reachable on a one-GPU box, RCCL refuses two ranks
    per device): every rank receives rank 0's ncclUniqueId over the torch.distributed rendezvous
    and initialises with its own rank, the world size and its LOCAL device."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_native_rendezvous_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    uid0 = bytes((torch.arange(128, dtype=torch.uint8) ^ 0x5A).numpy())
    for rank, (r, cr, cw, h, calls) in enumerate(res):
        assert (r, cr, cw, h) == (rank, rank, world, 7)
        assert len(calls) == 1
        _, uid, crank, cworld, dev, _ = calls[0]
        assert uid == uid0 and crank == rank and cworld == world and dev == rank


def test_nccl_process_group_uses_high_priority_streams():
    """Round-3 verdict: the world > 1 default (ProcessGroupNCCL) runs its collectives on a
    high-priority stream, as the native communicator and the proxy measurements do."""
    from replicann_amd.parallel import nccl_options

    assert nccl_options().is_high_priority_stream
