"""T4 distributed correctness on a fake cluster: multi-process CPU gloo, world 2 and 4.

Checks: gradients after the bucketed in-place all-reduce equal the
single-process gradients of the concatenated batch; ``no_sync`` accumulation;
odd bucket boundaries (tiny bucket size → many buckets); unused parameters;
the initial broadcast; and identical parameters across ranks after optimizer
steps."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(12, 33)
        self.b = torch.nn.Linear(33, 7)
        self.unused = torch.nn.Linear(3, 3)  # never receives a gradient

    def forward(self, x, y):
        return torch.nn.functional.cross_entropy(self.b(torch.relu(self.a(x))), y)


def _worker(rank, world, port, bucket_mb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from replicann_amd.optim import FusedAdamW
        from replicann_amd.parallel import DistributedDataParallel
        from replicann_amd.utils.flat import FlatParams

        torch.manual_seed(100 + rank)  # different init per rank: broadcast must fix it
        net = Net()
        flat = FlatParams(net)
        ddp = DistributedDataParallel(net, flat, bucket_mb=bucket_mb)
        g = torch.Generator().manual_seed(7)
        X = torch.randn(world * 8, 12, generator=g)
        Y = torch.randint(0, 7, (world * 8,), generator=g)
        x, y = X[rank * 8:(rank + 1) * 8], Y[rank * 8:(rank + 1) * 8]
        # 1) plain sync step
        flat.zero_grad()
        ddp(x, y).backward()
        ddp.finish()
        grad_avg = flat.grad.clone() / world
        # 2) no_sync accumulation over two half-batches, then a synced one
        flat.zero_grad()
        with ddp.no_sync():
            ddp(x[:4], y[:4]).backward()
        ddp(x[4:], y[4:]).backward()
        ddp.finish()
        grad_acc = flat.grad.clone() / world
        # 3) optimizer keeps ranks identical
        opt = FusedAdamW(flat, lr=1e-2, grad_scale=1 / world)
        for _ in range(3):
            flat.zero_grad()
            ddp(x, y).backward()
            ddp.finish()
            opt.step()
        params = flat.data.clone()
        # numpy copies are pickled by value: torch tensors would travel as shared-memory
        # fds that vanish when this worker exits before the parent unpickles them
        q.put((rank, grad_avg.numpy(), grad_acc.numpy(), params.numpy(), len(ddp.buckets), None))
    finally:
        dist.destroy_process_group()


def _single_process_grad(init_weight_rank0, world):
    from replicann_amd.utils.flat import FlatParams
    torch.manual_seed(100)
    net = Net()
    flat = FlatParams(net)
    g = torch.Generator().manual_seed(7)
    X = torch.randn(world * 8, 12, generator=g)
    Y = torch.randint(0, 7, (world * 8,), generator=g)
    flat.zero_grad()
    # the DDP loss is a per-rank mean; average of rank means == mean over the batch here
    net(X, Y).backward()
    return flat.grad.clone(), net


@pytest.mark.parametrize("world,bucket_mb", [(2, 0.0005), (2, 64.0), (4, 0.001)])
def test_ddp_gloo(world, bucket_mb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    res = [(r, torch.from_numpy(ga), torch.from_numpy(gc), torch.from_numpy(pp), nb, w)
           for r, ga, gc, pp, nb, w in res]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref_grad, net = _single_process_grad(res[0][5], world)
    if bucket_mb < 0.01:
        assert res[0][4] > 2, "tiny bucket size should produce several buckets"
    for rank, grad_avg, grad_acc, params, _, _ in res:
        torch.testing.assert_close(grad_avg, ref_grad, atol=1e-6, rtol=1e-5)
        torch.testing.assert_close(grad_acc, ref_grad * 2, atol=1e-6, rtol=1e-5)  # sum of 2 half-batch means
        torch.testing.assert_close(params, res[0][3], atol=0, rtol=0)
