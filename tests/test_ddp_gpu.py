"""DDP on the GPU code path (native kernels, direct gradient accumulation, ready hooks),
rehearsed on ONE card: 2 ranks, both on cuda:0, collectives over gloo (the reducer logic
is backend-agnostic; RCCL only changes the transport).

Checks that the all-reduced flat gradient equals the single-process gradient of the
concatenated batch, and that every bucket's all-reduce was issued from a gradient hook
during the backward (i.e. the overlap actually happens on the native path, including the
parameters whose gradients the kernels accumulate directly)."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model():
    import replicann_amd as R
    torch.manual_seed(0)
    m = R.GPT2(R.GPT2Config.tiny(n_embd=128, n_head=2, n_layer=2, block_size=128)).cuda()
    for p in m.parameters():
        p.data = p.data.to(torch.bfloat16)
    return m


def _batch(world):
    g = torch.Generator().manual_seed(5)
    ids = torch.randint(0, 1000, (2 * world, 129), generator=g)
    return ids[:, :-1].cuda(), ids[:, 1:].cuda()


def _worker(rank, world, port, q, mode="allreduce", schedule="auto"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), REPLICANN_DIST_BACKEND="gloo", REPLICANN_SHARE_DEVICE="1")
    from replicann_amd.parallel import DistributedDataParallel, init_distributed
    from replicann_amd.utils.flat import FlatParams
    init_distributed()
    try:
        m = _model()
        flat = FlatParams(m)
        ddp = DistributedDataParallel(m, flat, bucket_mb=0.25, reduce_mode=mode, schedule=schedule,
                                      window_mb=0.2)  # several buckets; windows take a few pieces each
        x, y = _batch(world)
        x, y = x[2 * rank:2 * rank + 2], y[2 * rank:2 * rank + 2]
        for _ in range(2 if schedule == "auto" else 1):  # auto: step 1 eager, step 2 windowed
            flat.zero_grad()
            ddp(x, y).backward()
            hooked = ddp.launched_in_backward
            ddp.finish()
        torch.cuda.synchronize()
        # numpy is pickled by value (a CPU tensor would travel as a shared-memory fd
        # that can vanish when this worker exits before the parent unpickles it)
        q.put((rank, (ddp.grad_source.float() / world).cpu().numpy(), hooked, len(ddp.buckets)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,schedule", [("allreduce", "eager"), ("rsag", "auto"), ("rsag", "end")])
def test_ddp_native_path_two_ranks_one_gpu(mode, schedule):
    """Two ranks on one card over gloo (torch.distributed transport with GPU tensors: the rsag
    narrowing runs on the side stream, windows are opened by the attention backward)."""
    from replicann_amd import _ext
    from replicann_amd.utils.flat import FlatParams
    assert _ext.available()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode, schedule)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda t: t[0])
    res = [(r, torch.from_numpy(g), h, nb) for r, g, h, nb in res]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = _model()
    flat = FlatParams(m)
    x, y = _batch(world)
    flat.zero_grad()
    m(x, y).backward()
    ref = flat.grad.float().cpu()
    for rank, g, hooked, nb in res:
        assert nb > 2
        # every bucket + both contributions of the tied wte (LM head, embedding) during the backward
        assert hooked == nb + 2, f"rank {rank}: only {hooked}/{nb}+2 reductions were launched during the backward"
        err = (g - ref).norm() / ref.norm()
        assert err < 2e-2, f"rank {rank}: rel err {err}"
    torch.testing.assert_close(res[0][1], res[1][1], atol=0, rtol=0)
