"""Process-group setup and data parallelism (N15/N16)."""

from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist

from .comm import NativeComm, TorchComm, make_comm
from .ddp import DistributedDataParallel


def dist_env():
    """(rank, local_rank, world_size) from torchrun-style env vars (defaults: single process)."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("LOCAL_RANK", 0)),
            int(os.environ.get("WORLD_SIZE", 1)))


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def nccl_options():
    """ProcessGroupNCCL (RCCL) options of the world > 1 step: collectives on a HIGH-priority stream.

    The DDP schedule (parallel/ddp.py, windows.py) issues bucket collectives beside the attention
    backward so that RCCL's workgroups interleave with that kernel's short workgroups; that only
    works if the command processor dispatches them ahead of the compute stream's queued work, which
    is what the native communicator's stream (csrc/comm) and the 1-GPU proxy measurements
    (profiles/ddp_window_proxy_r3ze.txt) assume.  torch's default is a normal-priority stream."""
    opts = dist.ProcessGroupNCCL.Options()
    opts.is_high_priority_stream = True
    return opts


def init_distributed(backend=None, timeout_s=600, force=False):
    """Initialise torch.distributed from env:// if WORLD_SIZE>1 (or ``force``: also a
    one-process group, for the one-GPU rehearsal of the data-parallel step).

    GPU → backend "nccl" (RCCL over xGMI), one process per GPU, device =
    LOCAL_RANK.  CPU → "gloo".  Returns (rank, local_rank, world, device).
    """
    rank, local_rank, world = dist_env()
    # Rehearsal knobs for a 1-GPU box (never needed on a real node):
    #   REPLICANN_DIST_BACKEND=gloo  collectives over gloo (GPU tensors staged through the host)
    #   REPLICANN_SHARE_DEVICE=1     every rank on cuda:0
    backend = backend or os.environ.get("REPLICANN_DIST_BACKEND") or None
    gpu = torch.cuda.is_available() and backend != "gloo"
    share = os.environ.get("REPLICANN_SHARE_DEVICE") == "1"
    if torch.cuda.is_available() and (gpu or share):
        dev_idx = 0 if share else local_rank
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    use_gpu = gpu
    if (world > 1 or force) and not dist.is_initialized():
        if world == 1:
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        be = backend or ("nccl" if use_gpu else "gloo")
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
            kw["pg_options"] = nccl_options()
        dist.init_process_group(**kw)
    return rank, local_rank, world, device


__all__ = ["DistributedDataParallel", "NativeComm", "TorchComm", "dist_env", "init_distributed", "make_comm",
           "nccl_options"]
